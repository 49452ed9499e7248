# Round 4: attention-half LoRA gradient jobs deferred into the next layer's launch (SLX_LORA_GRAD_DEFER).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_side_stream_gpu.py -m gpu -x -q -k group --timeout 200 --timeout-method thread > gpurun_out/r4_defer_tests.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_defer_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4_defer_tests.log
SLX_LORA_GRAD_DEFER=1 timeout -k 10 300 python3 -u -m pytest tests/test_fullgeom_parity_gpu.py tests/test_ddp_rccl_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_defer_parity.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_defer_parity.log | tail -30; exit 1; }
tail -1 gpurun_out/r4_defer_parity.log
bash tools/step_ab.sh "SLX_LORA_GRAD_DEFER=0" "SLX_LORA_GRAD_DEFER=1" 2
