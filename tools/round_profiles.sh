# Round-end evidence: GPU tests, the bench line, a steady-state kernel profile and the PMC pass, all under
# gpurun_out/; copy the summaries into profiles/ afterwards. usage: bash tools/round_profiles.sh TAG
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-r2}
timeout -k 10 500 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -2 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python3 bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format rocpd csv -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 70 > gpurun_out/${TAG}_steps.txt
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --top 50 > gpurun_out/${TAG}_steps_byname.txt
find gpurun_out/${TAG}_prof -name "*stats*.csv" -exec cp {} gpurun_out/${TAG}_kernel_stats.csv \; || true
rm -rf gpurun_out/${TAG}_prof
head -12 gpurun_out/${TAG}_steps.txt
bash tools/pmc_step.sh ${TAG}
