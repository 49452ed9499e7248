# decode Infinity Cache prefetch A/B: alternating bench_infer runs, SLX_DEC_PREFETCH workgroups x LAG
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/dec_prefetch_ab.txt
: > $out
for rep in 1 2; do
  for cfg in "0 1" "128 1" "256 1" "64 1" "128 2"; do
    set -- $cfg
    r=$(SLX_DEC_PREFETCH=$1 SLX_DEC_PREFETCH_LAG=$2 timeout -k 10 150 python3 bench_infer.py --frames 3 | tail -1) || exit 1
    ms=$(python3 -c "import json,sys; print(json.loads(sys.argv[1])['decode_ms_per_token'])" "$r")
    echo "rep=$rep prefetch=$1 lag=$2 decode_ms_per_token=$ms" | tee -a $out
  done
done
