set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gemm_gpu.py tests/test_fullgeom_parity_gpu.py tests/test_base_parity_gpu.py tests/test_vla_parity_gpu.py tests/test_deterministic_gpu.py > gpurun_out/resid_tests.log 2>&1 || { tail -30 gpurun_out/resid_tests.log; exit 1; }
tail -2 gpurun_out/resid_tests.log
bash tools/step_ab.sh "SLX_LIB_PATH=abx/pre_resid.so" "SLX_ATTN_DMA=1" 2
