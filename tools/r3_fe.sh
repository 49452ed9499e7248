# FE (register-direct epilogue + early prefetch, variant 11) on one GPU: GEMM tests, then K-sweeps and the
# epilogue-heavy InternViT shapes against variants 7/8 (interleaved in one process).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/fe
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread ${FE_K:+-k "$FE_K"} > $O/gemm_tests.log 2>&1 || { echo TESTFAIL; tail -60 $O/gemm_tests.log; exit 1; }
tail -2 $O/gemm_tests.log
for v in 7 11; do VARIANT=$v KS=1024,4096 timeout -k 10 120 python -u tools/gemm_ksweep.py 4096 1024 >> $O/ks.txt 2>&1 || exit 1; done
for v in 7 11; do OUT=f32 VARIANT=$v KS=1024,4096 timeout -k 10 120 python -u tools/gemm_ksweep.py 1024 >> $O/ks.txt 2>&1 || exit 1; done
cat $O/ks.txt
VARIANTS=7,8,11 timeout -k 10 300 python -u tools/gemm_epi_bench.py fc1 fc2bwd fc2 proj nt_plain nn_plain > $O/epi.txt 2>&1 && cat $O/epi.txt || exit 1
