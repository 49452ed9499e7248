# Round 4: the InternViT fc1 GEMM storing gelu'(h) as its aux (SLX_GELU_AUX_GRAD): GEMM tests, the engine's parity
# tests with the knob on, then the step A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q -k "aux_grad or fe" --timeout 150 --timeout-method thread > gpurun_out/r4_ga_tests.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_ga_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4_ga_tests.log
SLX_GELU_AUX_GRAD=1 timeout -k 10 300 python3 -u -m pytest tests/test_fullgeom_parity_gpu.py tests/test_vla_parity_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4_ga_parity.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_ga_parity.log | tail -30; exit 1; }
tail -1 gpurun_out/r4_ga_parity.log
bash tools/step_ab.sh "SLX_GELU_AUX_GRAD=0" "SLX_GELU_AUX_GRAD=1" 2
