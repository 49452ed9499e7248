# Round 4: the steady-step kernel profile of the default bench command with the two weight-gradient pairs split
# (tools/prof_steps.py --alternate), plus the rocprofv3 --stats summary of the same run.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r4pp}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --top 12 --alternate v3_pair_kernel > gpurun_out/${TAG}_steps_pairs.txt
cat gpurun_out/${TAG}_steps_pairs.txt
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
tail -3 gpurun_out/${TAG}_prof.log
rm -rf gpurun_out/${TAG}_prof
