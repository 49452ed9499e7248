# End-of-session validation: the -m gpu suite, smoke(), the default bench line (with the CPU baseline), a
# steady-state profile of the VLA step and the decode profile.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-final}
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 70 > gpurun_out/${TAG}_steps.txt
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --top 40 > gpurun_out/${TAG}_steps_byname.txt
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --top 12 --alternate v3_pair_kernel > gpurun_out/${TAG}_steps_pairs.txt
head -12 gpurun_out/${TAG}_steps.txt
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \;
rm -rf gpurun_out/${TAG}_prof
bash tools/dec_prof.sh ${TAG}_dec
