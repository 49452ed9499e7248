# kernel trace of the default bench + the first steady step's dispatch sequence (site attribution by position)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${TAG:-r5s}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 90 --dump gpurun_out/${TAG}_seq.txt > gpurun_out/${TAG}_steps.txt
head -5 gpurun_out/${TAG}_steps.txt
