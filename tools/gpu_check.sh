# One GPU round-trip: the -m gpu suite, the default bench line, and a steady-state kernel profile of the VLA step.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-chk}
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -3 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
if [ "${PROFILE:-1}" = "1" ]; then
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 70 > gpurun_out/${TAG}_steps.txt
head -25 gpurun_out/${TAG}_steps.txt
fi
