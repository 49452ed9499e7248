# A/B of builds of libslx_hip.so on the bench step (alternating processes, N=1, config 3, --no-extras);
# LIBS = space-separated library paths ("in-tree" = the in-tree build). usage: LIBS="abx/x.so in-tree" bash tools/lib_ab_step.sh [pairs]
set -e
cd $GRAFT_REPO_ROOT
LIBS=${LIBS:-"abx/base.so in-tree"}
N="${1:-3}"
for r in $(seq 1 $N); do
  for L in $LIBS; do
    if [ "$L" = "in-tree" ]; then unset SLX_LIB_PATH; else export SLX_LIB_PATH=$L; fi
    timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 --no-extras --no-cpu-baseline > /tmp/ab.json
    python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(sys.argv[1], d['value'], d['ms_per_step'])" "$L"
  done
done
