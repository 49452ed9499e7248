# Round 4: grouped LoRA parameter gradients (slx_lora_grad): tests, then the step A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_lora_dropout_gpu.py tests/test_side_stream_gpu.py -m gpu -x -q -s --timeout 150 --timeout-method thread > gpurun_out/r4_lg_tests.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_lg_tests.log | tail -40; exit 1; }
grep -h "worst (side" gpurun_out/r4_lg_tests.log || true
tail -1 gpurun_out/r4_lg_tests.log
bash tools/step_ab.sh "SLX_LORA_GRAD_GROUP=0" "SLX_LORA_GRAD_GROUP=1" 2
bash tools/step_ab.sh "SLX_LORA_GRAD_GROUP=1 SLX_LORA_GRAD_ITEMS=256" "SLX_LORA_GRAD_GROUP=1 SLX_LORA_GRAD_ITEMS=1024" 1
