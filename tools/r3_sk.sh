# Stream-K + FE on one GPU: GEMM tests (stream-K, FE), FE debug pattern check, stream-K A/B, FE sweeps.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sk
mkdir -p $O
timeout -k 10 120 python -u tools/fe_dbg.py > $O/fe_dbg.txt 2>&1; cat $O/fe_dbg.txt
timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -k "stream_k or fe" > $O/tests.log 2>&1 || { echo TESTFAIL; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
SLX_GEMM_SK=0 timeout -k 10 120 python -u tools/sk_bench.py > $O/skb.txt 2>&1 && timeout -k 10 120 python -u tools/sk_bench.py >> $O/skb.txt 2>&1 && cat $O/skb.txt || exit 1
VARIANTS=7,8,11 timeout -k 10 300 python -u tools/gemm_epi_bench.py fc1 fc2bwd fc2 proj nt_plain nn_plain > $O/epi.txt 2>&1 && cat $O/epi.txt || exit 1
