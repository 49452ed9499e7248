# Round 4: FE on single-round launches of every epilogue (SLX_GEMM_FE1=2) vs STORE only (1): tests, step A/B.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SLX_GEMM_FE1=2 timeout -k 10 300 python3 -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/r4_fe2_tests.log 2>&1 || { grep -v amdgpu.ids gpurun_out/r4_fe2_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/r4_fe2_tests.log
bash tools/step_ab.sh "SLX_GEMM_FE1=1" "SLX_GEMM_FE1=2" 2
