# A/B of the ViT attention dispatch order (SLX_ATTN_TAIL_FIRST) in alternating bench runs + the attention microbench,
# then a fresh FC1 HBM-traffic pass (tools/pmc_fc1.sh).
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 200 python3 -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1 || { tail -20 gpurun_out/tail_tests.log; exit 1; }
SLX_ATTN_TAIL_FIRST=1 timeout -k 10 200 python3 -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread >> gpurun_out/tail_tests.log 2>&1 || { tail -20 gpurun_out/tail_tests.log; exit 1; }
grep passed gpurun_out/tail_tests.log
for t in 0 1 0 1; do
  SLX_ATTN_TAIL_FIRST=$t timeout -k 10 120 python3 tools/attn_bench.py 2>/dev/null | grep vit | sed "s/^/tail_first=$t /" || exit 1
  SLX_ATTN_TAIL_FIRST=$t timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/tail.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/tail.json')); print('tail_first=$t', d['value'], d['ms_per_step'])"
done
bash tools/pmc_fc1.sh && cat gpurun_out/vla_fc1_traffic.json
for r in 2 4 1 2 4 1; do
  SLX_DEC_GEMV_RSW=$r timeout -k 10 200 python3 bench_infer.py --frames 3 2>/dev/null > gpurun_out/rsw.json || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/rsw.json')); print('swiglu_rows_per_wave=$r', d['decode_ms_per_token'])"
done
