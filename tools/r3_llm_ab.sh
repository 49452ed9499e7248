# Round-3: LLM gate/up dgrad on v3 + 2-way split-K reduced in-launch vs v2; VLA step with / without split_ws
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${R3TAG:-r3f}; mkdir -p $O
VARIANTS=0,2,7 timeout -k 10 200 python -u tools/gemm_bench.py llm_gu_dgradx llm_qkv_dgrad llm_down_dgrad > $O/gb.txt 2>&1; cat $O/gb.txt
for w in 0 1 0 1; do SLX_SPLIT_WS=$w timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/bench_w$w.json 2>$O/bench_w$w.err || { tail -5 $O/bench_w$w.err; exit 1; }; python -c "import json;d=json.loads(open('$O/bench_w$w.json').read().strip().splitlines()[-1]);print('split_ws=$w',d['value'],d['ms_per_step'],d['roofline']['achieved'],d.get('roofline_fc1',{}).get('achieved'))"; done
