set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_attention_gpu.py tests/test_attention_variants_gpu.py tests/test_decode_gpu.py tests/test_fullgeom_parity_gpu.py > gpurun_out/attn_tests.log 2>&1 || { tail -30 gpurun_out/attn_tests.log; exit 1; }
tail -2 gpurun_out/attn_tests.log
LIBS="abx/kvsalu.so in-tree" SHAPES=llm bash tools/lib_ab_attn.sh
bash tools/step_ab.sh "SLX_LIB_PATH=abx/base.so" "SLX_ATTN_DMA=1" 2
