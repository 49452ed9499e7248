# round-5 GPU call: the tests named in $TESTS (default: the precise / drift / parity files), then optionally the bench
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r5}
TESTS=${TESTS:-tests/test_vla_parity_gpu.py tests/test_drift_gpu.py}
timeout -k 10 900 python3 -u -m pytest $TESTS -x -v -s --timeout 600 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -60 gpurun_out/${TAG}_tests.log; exit 1; }
tail -5 gpurun_out/${TAG}_tests.log
if [ "${BENCH:-0}" = "1" ]; then
timeout -k 10 500 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
fi
