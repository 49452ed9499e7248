# attention PMC record per dispatch (ViT and Qwen2 named by grid), three passes of <= 8 SQ / 2 GRBM counters
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
P="--output-format csv -- python3 tools/attn_bench.py vit llm"  # the two step shapes only (vit1024 / llm_mha share their grids)
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/ap1 -o run $P > gpurun_out/ap1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/ap2 -o run $P > gpurun_out/ap2.log 2>&1
python3 tools/pmc_dispatch.py tools/attn_sites.json gpurun_out/ap1 gpurun_out/ap2 > gpurun_out/attn_pmc_dispatch.jsonl
rm -rf gpurun_out/ap1 gpurun_out/ap2
cat gpurun_out/attn_pmc_dispatch.jsonl
