#!/bin/bash
# attention row-tail fold: kernel tests, the isolated shapes with the fold on / off, the step A/B, parity at depth
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r6d}
timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py -q -x --timeout 120 --timeout-method thread > gpurun_out/${T}_attn_tests.log 2>&1 || { tail -30 gpurun_out/${T}_attn_tests.log; exit 1; }
tail -2 gpurun_out/${T}_attn_tests.log
for e in 1 0 1 0; do
  SLX_ATTN_QTAIL=$e timeout -k 10 120 python3 tools/attn_bench.py vit vit1024 2>&1 | grep -v amdgpu.ids | sed "s/^/qtail=$e /"
done | tee gpurun_out/${T}_attn_bench.txt
bash tools/step_ab.sh "SLX_ATTN_QTAIL=0" "SLX_ATTN_QTAIL=1" 2 | tee gpurun_out/${T}_step_ab.txt
timeout -k 10 900 python3 -u -m pytest tests/test_fullgeom_parity_gpu.py tests/test_vla_parity_gpu.py tests/test_fulldepth_parity_gpu.py tests/test_base_parity_gpu.py -q -rf -s --timeout 900 --timeout-method thread > gpurun_out/${T}_parity.log 2>&1
echo "parity rc=$?"
tail -3 gpurun_out/${T}_parity.log
