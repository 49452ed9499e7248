# ADVICE fixes: fold hand-off fences, fold/unfolded remainder test, decode timeout check, f32-oracle waypoint bound
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R3TAG:-r3i}; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_decode_gpu.py tests/test_vla_parity_gpu.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
tail -3 $O/tests.log
