# Round 4: LDS-DMA staged attention kernels vs the register-staged ones (SLX_ATTN_DMA=0), alternating processes on one
# box; outputs of both compared bit for bit; then the attention GPU tests.
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  SLX_ATTN_DMA=0 timeout -k 10 120 python3 tools/attn_bench.py --save gpurun_out/attn_reg.pt
  SLX_ATTN_DMA=1 timeout -k 10 120 python3 tools/attn_bench.py --save gpurun_out/attn_dma.pt
done
timeout -k 10 120 python3 - <<'PY'
import torch
a = torch.load("gpurun_out/attn_reg.pt", weights_only=True)
b = torch.load("gpurun_out/attn_dma.pt", weights_only=True)
for s in a:
    for k in a[s]:
        x, y = a[s][k], b[s][k]
        same = torch.equal(x.view(torch.int16) if x.dtype == torch.bfloat16 else x, y.view(torch.int16) if y.dtype == torch.bfloat16 else y)
        print(s, k, "bit-identical" if same else f"DIFF max {(x.float() - y.float()).abs().max().item():.3g}")
PY
rm -f gpurun_out/attn_reg.pt gpurun_out/attn_dma.pt
timeout -k 10 300 python3 -u -m pytest tests/test_attention_gpu.py -x -q --timeout 120 --timeout-method thread 2>&1 | tail -3
