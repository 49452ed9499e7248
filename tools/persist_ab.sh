# A/B of the persistent v3 GEMM grid (SLX_GEMM_PERSIST=k: at most 256 k blocks walking the tiles) on the VLA step.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SLX_GEMM_PERSIST=1 timeout -k 10 300 python3 -u -m pytest tests/test_gemm_gpu.py tests/test_fullgeom_parity_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/persist_tests.log 2>&1 || { tail -30 gpurun_out/persist_tests.log; exit 1; }
tail -1 gpurun_out/persist_tests.log
for k in 0 1 2 0 1; do
  SLX_GEMM_PERSIST=$k timeout -k 10 300 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/persist_$k.json 2>/dev/null
  python3 -c "import json; d=json.load(open('gpurun_out/persist_$k.json')); print('persist=$k', d['value'], d['ms_per_step'])"
done
