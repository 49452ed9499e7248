# LDS counters of the v3 GEMM main loop per operand layout (NT / NN / TN; M 16384, N 4096, K 4096): is the slower
# NN / TN main loop an LDS bank-conflict or an LDS-wait cost of the transposing fragment reads?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lpmc; mkdir -p $O
for L in NT NN TN; do
  LAYOUT=$L KS=4096 M=16384 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY --output-format csv -d $O/$L -o run -- python3 tools/gemm_ksweep.py 4096 > $O/$L.log 2>&1 || { tail -5 $O/$L.log; exit 1; }
  echo "== $L"; grep "TF" $O/$L.log | head -2
  python3 tools/pmc_kernels.py $O/$L gemm_bf16
  rm -rf $O/$L
done
