# Mainloop cost per K-step by operand layout (NT / NN / TN) and LDS counters of the TN weight-gradient form.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tn
mkdir -p $O
for L in NT NN TN; do
  LAYOUT=$L KS=1024,4096 timeout -k 10 120 python -u tools/gemm_ksweep.py 1024 >> $O/sweep.txt 2>&1 || exit 1
done
cat $O/sweep.txt
for L in NT TN; do
  LAYOUT=$L KS=4096 timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES --output-format csv -d $O/pmc_$L -o run -- python3 tools/gemm_ksweep.py 1024 > $O/pmc_$L.log 2>&1 || exit 1
  python3 tools/pmc_kernels.py $O/pmc_$L gemm > $O/pmc_$L.txt && cat $O/pmc_$L.txt
  rm -rf $O/pmc_$L
done
