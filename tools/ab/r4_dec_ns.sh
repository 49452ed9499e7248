# Round 4: decode split-attention workgroups per kv head (SLX_DEC_SPLIT_NS 4 vs 8), alternating bench_infer runs.
set -e
cd $GRAFT_REPO_ROOT
for r in 1 2; do
  for n in 8 4; do
    SLX_DEC_SPLIT_NS=$n timeout -k 10 200 python3 bench_infer.py --frames 3 2>/dev/null > gpurun_out/dec_ns_$n.json
    python3 -c "import json; d=json.load(open('gpurun_out/dec_ns_$n.json')); print('split_ns=$n', d['decode_ms_per_token'], d['value'])"
  done
done
