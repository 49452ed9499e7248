#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/r6f_attn_tests.log 2>&1 || { tail -30 gpurun_out/r6f_attn_tests.log; exit 1; }
tail -1 gpurun_out/r6f_attn_tests.log
for r in 1 2; do
for e in "SLX_ATTN_QTAIL=1" "SLX_ATTN_QTAIL=0" "SLX_ATTN_TAIL_FIRST=0"; do
  env $e timeout -k 10 120 python3 tools/attn_bench.py vit 2>&1 | grep -v amdgpu.ids | sed "s/^/$e /"
done
done | tee gpurun_out/r6f_attn_bench.txt
timeout -k 10 120 python3 tools/attn_bench.py vit1024 2>&1 | grep -v amdgpu.ids
