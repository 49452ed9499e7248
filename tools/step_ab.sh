# Round 4 step-level A/B: alternating bench processes on one box (N=1, config 3, --no-extras, no CPU baseline).
# usage: bash tools/step_ab.sh "ENV_A" "ENV_B" [pairs]   e.g. "SLX_GEMM_FE=0" "SLX_GEMM_FE=1"
set -e
cd $GRAFT_REPO_ROOT
A="$1"; B="$2"; N="${3:-2}"
for r in $(seq 1 $N); do
  for e in "$A" "$B"; do
    env $e timeout -k 10 240 python3 bench.py --steps 8 --warmup 2 --no-extras --no-cpu-baseline > /tmp/ab.json
    python3 -c "import json,sys; d=json.load(open('/tmp/ab.json')); print(sys.argv[1], d['value'], d['ms_per_step'], d.get('step_mfma_frac'))" "$e"
  done
done
