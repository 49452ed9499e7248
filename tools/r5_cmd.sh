set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_variants_gpu.py tests/test_fullgeom_parity_gpu.py tests/test_vla_parity_gpu.py > gpurun_out/tail_tests.log 2>&1 || { tail -30 gpurun_out/tail_tests.log; exit 1; }
tail -2 gpurun_out/tail_tests.log
for r in 1 2; do
  for t in 0 1; do SLX_ATTN_TAILV=$t timeout -k 10 120 python3 tools/attn_bench.py vit 2>&1 | grep -v amdgpu.ids | sed "s/^/tailv=$t /"; done
done
bash tools/step_ab.sh "SLX_ATTN_TAILV=0" "SLX_ATTN_TAILV=1" 2
