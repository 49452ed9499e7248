# GEMM tests, then the VLA step with and without the FE member (SLX_GEMM_FE, alternating processes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/feab
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gemm_tests.log; exit 1; }
tail -2 $O/gemm_tests.log
for fe in 1 0 1 0; do
  SLX_GEMM_FE=$fe timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/bench_fe$fe.json 2>$O/bench_fe$fe.err || { tail -5 $O/bench_fe$fe.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_fe$fe.json').read().strip().splitlines()[-1]);print('fe=$fe',d['value'],d['ms_per_step'],d['roofline']['achieved'],d.get('roofline_fc1',{}).get('achieved'))"
done
