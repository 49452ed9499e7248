# Round-2 iteration: full -m gpu suite, decode attention trace, norm microbench, default bench line, steady-state
# step profile, decode profile. Every GPU step has its own time limit; the first failure ends the script.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2}
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 120 python3 tools/dec_attn_trace.py 680 > gpurun_out/${TAG}_dectrace.txt 2>&1
cat gpurun_out/${TAG}_dectrace.txt
timeout -k 10 120 python3 tools/norm_bench.py > gpurun_out/${TAG}_norm.txt 2>&1
timeout -k 10 120 python3 tools/attn_bench.py >> gpurun_out/${TAG}_norm.txt 2>&1
cat gpurun_out/${TAG}_norm.txt
timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 70 > gpurun_out/${TAG}_steps.txt
head -30 gpurun_out/${TAG}_steps.txt
bash tools/dec_prof.sh ${TAG}_dec
