# A/B of the in-tree build against tools/_ab/prev.so on the VLA step (alternating processes), plus the GEMM tests and
# the epilogue-heavy InternViT GEMMs of both builds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/libab; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread > $O/gemm_tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/gemm_tests.log; exit 1; }
tail -1 $O/gemm_tests.log
for lib in prev new; do
  if [ $lib = prev ]; then export SLX_LIB_PATH=$PWD/tools/_ab/prev.so; else unset SLX_LIB_PATH; fi
  VARIANTS=0 timeout -k 10 200 python -u tools/gemm_epi_bench.py fc1 fc2bwd > $O/epi_$lib.txt 2>&1 && sed "s/^/$lib /" $O/epi_$lib.txt | grep -v amdgpu || exit 1
done
for lib in prev new prev new; do
  if [ $lib = prev ]; then export SLX_LIB_PATH=$PWD/tools/_ab/prev.so; else unset SLX_LIB_PATH; fi
  timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-extras > $O/b_$lib.json 2>$O/b_$lib.err || { tail -5 $O/b_$lib.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$lib.json').read().strip().splitlines()[-1]);print('$lib',d['value'],d['ms_per_step'],d.get('roofline_fc1',{}).get('achieved'))"
done
