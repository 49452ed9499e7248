set -e
cd $GRAFT_REPO_ROOT
bash tools/step_ab.sh "SLX_LORA_DX_GROUPS=1" "SLX_LORA_DX_GROUPS=2" 2
bash tools/step_ab.sh "SLX_ATTN_DMA=0" "SLX_ATTN_DMA=1" 1
bash tools/step_ab.sh "SLX_LORA_DA_SLAB=0" "SLX_LORA_DA_SLAB=1" 2
