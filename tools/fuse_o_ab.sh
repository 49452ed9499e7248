# A/B of the fused attention + O projection decode launch (SLX_DEC_FUSE_O) in alternating bench_infer runs.
cd $GRAFT_REPO_ROOT
for f in 0 1 0 1; do
  SLX_DEC_FUSE_O=$f timeout -k 10 200 python3 bench_infer.py --frames 3 2>/dev/null > gpurun_out/fuse_$f.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/fuse_$f.json')); print('fuse_o=$f', d['decode_ms_per_token'], d['value'])"
done
