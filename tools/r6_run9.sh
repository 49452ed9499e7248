#!/bin/bash
# LoRA pack walking its destination + the one-output ordered reduction: tests + library A/B on the step
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r6k}
timeout -k 10 900 python3 -u -m pytest tests/test_norm_gpu.py tests/test_adamw_gpu.py tests/test_lora_dropout_gpu.py tests/test_vla_parity_gpu.py tests/test_fullgeom_parity_gpu.py tests/test_deterministic_gpu.py tests/test_resume_gpu.py tests/test_ddp_gpu.py tests/test_ddp_rccl_gpu.py tests/test_dp8_trajectory_gpu.py -q -rf --timeout 800 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
LIBS="abx/base.so in-tree" bash tools/lib_ab_step.sh 2 | tee gpurun_out/${T}_lib_ab.txt
bash tools/step_ab.sh "SLX_NORM_FWD_RPW=1" "SLX_NORM_FWD_RPW=2" 2 | tee gpurun_out/${T}_rpw_ab.txt
