# kernel-trace stats of the default bench step -> gpurun_out/${TAG}_steps.txt (per-kernel table) and ${TAG}_seq.txt
# (first steady step's dispatch sequence). usage: bash tools/prof_quick_step.sh TAG [ENV=VAL ...]
cd $GRAFT_REPO_ROOT
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
for e in "$@"; do export "$e"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format rocpd csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-extras > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/prof_steps.py gpurun_out/${TAG}_prof --warmup 2 --grid --top 60 --dump gpurun_out/${TAG}_seq.txt > gpurun_out/${TAG}_steps.txt
rm -rf gpurun_out/${TAG}_prof
