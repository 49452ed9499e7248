# Step-only A/B of the in-tree build against tools/_ab/prev.so (alternating processes, one box): ROUNDS pairs.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/libab; mkdir -p $O
for r in $(seq ${ROUNDS:-3}); do
  for lib in prev new; do
    if [ $lib = prev ]; then export SLX_LIB_PATH=$PWD/tools/_ab/prev.so; else unset SLX_LIB_PATH; fi
    timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/b_$lib.json 2>$O/b_$lib.err || { tail -5 $O/b_$lib.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_$lib.json').read().strip().splitlines()[-1]);print('$lib',d['value'],d['ms_per_step'])"
  done
done
