# LoRA dA chunking A/B (SLX_LORA_DA_BLOCKS) on the Qwen2 shapes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${R3TAG:-r3m}; mkdir -p $O
for B in 512 256 128 64; do
  echo "== SLX_LORA_DA_BLOCKS=$B" >> $O/lora_ab.txt
  SLX_LORA_DA_BLOCKS=$B timeout -k 10 120 python -u tools/lora_bench.py >> $O/lora_ab.txt 2>&1 || { tail -20 $O/lora_ab.txt; exit 1; }
done
cat $O/lora_ab.txt
