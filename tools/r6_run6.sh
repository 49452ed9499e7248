#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
T=${1:-r6h}
timeout -k 10 900 python3 -u -m pytest tests/test_lora_dropout_gpu.py tests/test_vla_parity_gpu.py tests/test_fullgeom_parity_gpu.py tests/test_deterministic_gpu.py tests/test_resume_gpu.py tests/test_driving_dropin_gpu.py tests/test_dropin_loop_gpu.py -q -rf --timeout 600 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/step_ab.sh "SLX_DROPBITS_FUSED=0" "SLX_DROPBITS_FUSED=1" 2 | tee gpurun_out/${T}_step_ab.txt
