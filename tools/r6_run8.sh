#!/bin/bash
# RMSNorm / short LayerNorm backward row kernel with unconditional loads: tests + library A/B on the step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r6j}
timeout -k 10 300 python3 -u -m pytest tests/test_norm_gpu.py tests/test_deterministic_gpu.py -q -rf --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
LIBS="abx/base.so in-tree" bash tools/lib_ab_step.sh 2 | tee gpurun_out/${T}_lib_ab.txt
