# Re-check of env-knob defaults on the current build: for each "NAME:a,b" pair, alternating runs a b a b.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/knobs; mkdir -p $O
for spec in ${KNOBS:-SLX_SPLIT_REDUCE_MAX:2,4 SLX_GEMM_FOLD_SPLIT:16,8 SLX_SWIGLU_BWD_VARIANT:2,7}; do
  name=${spec%%:*}; vals=${spec#*:}; a=${vals%%,*}; b=${vals#*,}
  for v in $a $b $a $b; do
    env $name=$v timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/b.json 2>$O/b.err || { tail -5 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('$name=$v',d['value'],d['ms_per_step'])"
  done
done
