# Folded M-remainder (SLX_GEMM_FOLD_REM, SLX_GEMM_FOLD_SPLIT) check and A/B: GEMM + parity tests, then alternating benches.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_gpu.py tests/test_fullgeom_parity_gpu.py tests/test_vla_parity_gpu.py tests/test_base_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fold_tests.log 2>&1 || { tail -40 gpurun_out/fold_tests.log; exit 1; }
tail -1 gpurun_out/fold_tests.log
for c in "0 8" "1 8" "1 16" "1 12" "0 8" "1 8" "1 16" "1 12"; do
  set -- $c
  SLX_GEMM_FOLD_REM=$1 SLX_GEMM_FOLD_SPLIT=$2 timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fold.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/fold.json')); print('fold=$1 split=$2', d['value'], d['ms_per_step'])"
done
