# Round 4: LDS-DMA staged attention kernels vs the register-staged ones, all builds in ONE process (tools/attn_ab.py:
# interleaved, 7 reps, outputs compared with the first build), then the attention GPU tests on the in-tree library.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
AB_DIR=ab_builds timeout -k 10 240 python3 tools/attn_ab.py run reg dma2 dq3s dqs pp5
timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py tests/test_attention_variants_gpu.py tests/test_lora_dropout_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
