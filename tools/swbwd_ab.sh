# A/B of the main loop under the SwiGLU-backward epilogue GEMM (K = 64): 0 = automatic (v3), 2 = v2 128^2 2 blocks/CU,
# 5 = v2 256x128.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SLX_SWIGLU_BWD_VARIANT=2 timeout -k 10 300 python3 -u -m pytest tests/test_fullgeom_parity_gpu.py tests/test_lora_dropout_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/sw_tests.log 2>&1 || { tail -30 gpurun_out/sw_tests.log; exit 1; }
tail -1 gpurun_out/sw_tests.log
for v in 0 2 5 0 2 5; do
  SLX_SWIGLU_BWD_VARIANT=$v timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/sw.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/sw.json')); print('swiglu_bwd_variant=$v', d['value'], d['ms_per_step'])"
done
