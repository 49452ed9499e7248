# A/B of an environment knob on the VLA step (alternating processes): ENVAB="NAME" VALS="1 0 1 0"
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/envab; mkdir -p $O
for v in ${VALS:-1 0 1 0}; do
  env $ENVAB=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/b$v.json 2>$O/b$v.err || { tail -5 $O/b$v.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b$v.json').read().strip().splitlines()[-1]);print('$ENVAB=$v',d['value'],d['ms_per_step'])"
done
