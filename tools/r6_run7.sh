#!/bin/bash
# LayerNorm backward (D = 1024) branch-free kernel: tests, isolated A/B, step A/B
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r6i}
timeout -k 10 300 python3 -u -m pytest tests/test_norm_gpu.py -q -rf --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
for v in 0 1 0 1; do
  echo "SLX_NORM_W1024=$v" | tee -a gpurun_out/${T}_norm_bench.txt
  SLX_NORM_W1024=$v timeout -k 10 120 python3 -u tools/norm_bench.py | tee -a gpurun_out/${T}_norm_bench.txt || exit 1
done
bash tools/step_ab.sh "SLX_NORM_W1024=0" "SLX_NORM_W1024=1" 2 | tee gpurun_out/${T}_step_ab.txt
