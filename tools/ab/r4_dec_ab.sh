# Round 4 decode A/B: the split attention merged by the O GEMV (SLX_DEC_SPLIT_O=1) vs one MFMA workgroup per kv head
# + the O GEMV, in alternating bench_infer processes.
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for f in 0 1; do
    SLX_DEC_SPLIT_O=$f timeout -k 10 200 python3 bench_infer.py --frames 3 2>/dev/null > gpurun_out/dec_split_$f.json
    python3 -c "import json; d=json.load(open('gpurun_out/dec_split_$f.json')); print('split_o=$f', d['decode_ms_per_token'], d['value'])"
  done
done
