# LoRA dB GEMM K-split cap A/B on the VLA step (alternating processes).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/dbab; mkdir -p $O
for sp in ${SPLITS:-0 8 4 12 0 8 4 12}; do
  SLX_LORA_DB_SPLIT=$sp timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/b$sp.json 2>$O/b$sp.err || { tail -5 $O/b$sp.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b$sp.json').read().strip().splitlines()[-1]);print('split=$sp',d['value'],d['ms_per_step'])"
done
