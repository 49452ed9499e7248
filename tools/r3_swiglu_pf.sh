# SwiGLU-backward epilogue prefetch: the GEMM/LoRA/VLA GPU tests on the new build, then prev vs new on the step.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/swpf; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_lora_dropout_gpu.py tests/test_vla_parity_gpu.py tests/test_fullgeom_parity_gpu.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ROUNDS=3 bash tools/r3_lib_ab_step.sh
