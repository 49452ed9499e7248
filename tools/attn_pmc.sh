# Attention kernels' SQ counters on the two hot shapes (tools/attn_bench.py), two passes of <= 8 SQ counters.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES --output-format csv -d gpurun_out/apmc1 -o run -- python3 tools/attn_bench.py > gpurun_out/apmc1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/apmc2 -o run -- python3 tools/attn_bench.py > gpurun_out/apmc2.log 2>&1
python3 tools/pmc_kernels.py gpurun_out/apmc1 attn_ > gpurun_out/r4_attn_pmc.txt
python3 tools/pmc_kernels.py gpurun_out/apmc2 attn_ >> gpurun_out/r4_attn_pmc.txt
rm -rf gpurun_out/apmc1 gpurun_out/apmc2
cat gpurun_out/r4_attn_pmc.txt
