# full GPU suite + smoke + default bench line (with the CPU baseline) on the current build
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r5full}
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1
cat gpurun_out/${TAG}_smoke.log | tail -2
if [ "${BENCH:-1}" = "1" ]; then
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
fi
