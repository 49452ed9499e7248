#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/attn_bench.py vit vit1024 llm llm_mha > gpurun_out/r6c_attn.txt 2>&1 || exit $?
cat gpurun_out/r6c_attn.txt
timeout -k 10 600 python3 -u -m pytest tests/test_dp8_trajectory_gpu.py -v -s --timeout 600 --timeout-method thread > gpurun_out/r6c_dp8.log 2>&1
echo "dp8 rc=$?"
grep -a "dp8 vs" gpurun_out/r6c_dp8.log | cut -c1-1500
