import sys
import torch
sys.path.insert(0, '.')
from simlingo_amd import kernels as K
dev = torch.device("cuda")
for (M, kin, ns) in [(64, 128, 1), (64, 128, 2), (64, 128, 3), (798, 128, 1)]:
    g = torch.Generator(device=dev).manual_seed(1)
    x = torch.randn(M, kin, device=dev, generator=g).bfloat16()
    As = [(torch.randn(32, kin, device=dev, generator=g) * 0.1).bfloat16() for _ in range(ns)]
    dt = torch.randn(M, 32 * ns, device=dev, generator=g).bfloat16().float()
    dAs = [torch.zeros(32, kin, device=dev) for _ in range(ns)]
    dx0 = torch.zeros(M, kin, device=dev)
    dx = dx0.clone()
    K.lora_bwd(x, dt, As, [None] * ns, dAs, dx=dx, p=0.0)
    torch.cuda.synchronize()
    ref = sum(dt[:, 32*j:32*j+32].double() @ As[j].double() for j in range(ns))
    err = (dx.double() - ref).abs()
    print(M, kin, ns, "max err", err.max().item(), "ref max", ref.abs().max().item(),
          "bad rows", (err.max(1).values > 1e-3).nonzero().flatten()[:10].tolist(),
          "bad cols", (err.max(0).values > 1e-3).nonzero().flatten()[:10].tolist(),
          "ratio", (dx.double() / ref)[0, :4].tolist())
