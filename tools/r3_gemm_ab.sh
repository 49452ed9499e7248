# Round-3 GEMM A/B on one GPU: GEMM tests (all variants), epilogue-heavy InternViT shapes and hot-path shapes per
# variant (interleaved in one process), then the VLA step with the automatic choice's v3 member switched by
# SLX_V3_KIND (alternating processes).
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/${R3TAG:-r3b}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gemm_tests.log; exit 1; }
tail -2 $O/gemm_tests.log
VARIANTS=${EPI_VARIANTS:-7,9,10,2} timeout -k 10 300 python -u tools/gemm_epi_bench.py fc1 fc2bwd fc2 proj nt_plain nn_plain > $O/epi.txt 2>&1 && cat $O/epi.txt || exit 1
VARIANTS=${GB_VARIANTS:-7,9,10,2} timeout -k 10 300 python -u tools/gemm_bench.py vit_qkv vit_fc1_dgrad vit_proj llm_gateup llm_down_dgrad llm_qkv_dgrad sq8192 > $O/gb.txt 2>&1 && cat $O/gb.txt || exit 1
for k in ${KINDS:-7 9 10 7 9 10}; do SLX_V3_KIND=$k timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/bench_k$k.json 2>$O/bench_k$k.err || { tail -5 $O/bench_k$k.err; exit 1; }; python -c "import json;d=json.loads(open('$O/bench_k$k.json').read().strip().splitlines()[-1]);print('kind=$k',d['value'],d['ms_per_step'],d['roofline']['achieved'],d.get('roofline_fc1',{}).get('achieved'))"; done
