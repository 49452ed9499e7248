# Kernel-trace profile of the bench step on the current build: steady-step table sorted by time
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r6p}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 90 --dump gpurun_out/${TAG}_seq.txt > gpurun_out/${TAG}_steps.txt
head -6 gpurun_out/${TAG}_steps.txt
rm -rf gpurun_out/${TAG}_prof
