# SimLingo-Base GPU parity incl. the full-width fixture
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R3TAG:-r3n}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_base_parity_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/tests.log; exit 1; }
grep -E "PASS|FAIL" $O/tests.log | tail -10
