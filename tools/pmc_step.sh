# Hardware counters of the steady-state VLA step: three rocprofv3 --pmc passes (SQ group, FETCH_SIZE, WRITE_SIZE),
# each its own run of a 2-step bench, then tools/pmc_step.py parse. usage: bash tools/pmc_step.sh TAG [bench args]
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=${1:-pmc}
shift || true
ARGS="--steps 2 --warmup 1 --no-cpu-baseline $*"
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d gpurun_out/${TAG}_sq -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_sq.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_f -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_f.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_w -o run -- python3 bench.py $ARGS > gpurun_out/${TAG}_w.log 2>&1
python3 tools/pmc_step.py parse --sq gpurun_out/${TAG}_sq --fetch gpurun_out/${TAG}_f --write gpurun_out/${TAG}_w --out gpurun_out/${TAG}_pmc.json --top 45 > gpurun_out/${TAG}_pmc.txt
rm -rf gpurun_out/${TAG}_sq gpurun_out/${TAG}_f gpurun_out/${TAG}_w
head -30 gpurun_out/${TAG}_pmc.txt
