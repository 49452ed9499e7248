# Decode (agent inference) measurement: bench_infer.py's JSON line and a rocprofv3 kernel summary of the
# graph-replayed decode step (per generated token).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-dec}
timeout -k 10 300 python3 bench_infer.py --frames 3 > gpurun_out/${TAG}_infer.json 2> gpurun_out/${TAG}_infer.err
cat gpurun_out/${TAG}_infer.json
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/${TAG}_prof -o run -- python3 bench_infer.py --frames 2 --warmup 1 > gpurun_out/${TAG}_prof.log 2>&1
python3 tools/prof_db.py gpurun_out/${TAG}_prof 300 30 > gpurun_out/${TAG}_summary.txt
head -12 gpurun_out/${TAG}_summary.txt
rm -rf gpurun_out/${TAG}_prof
