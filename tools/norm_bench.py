"""Isolated timing of the InternViT LayerNorm backward with the fused layer-scale branch (slx_norm_bwd, D = 1024,
16 x 1025 rows): f32 vs bf16 dy."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
M, D = 16400, 1024
x = torch.randn(M, D, device=dev)
gamma, beta = torch.rand(D, device=dev) + 0.5, torch.randn(D, device=dev)
y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
d = K.norm_desc(x, gamma, beta, y, mean, rstd, M, D, 1e-6)
K.norm_fwd(d)
dyf = torch.randn(M, D, device=dev)
dyb = dyf.bfloat16()
dx = torch.randn(M, D, device=dev)
ls = torch.rand(D, device=dev) * 0.2
yb = torch.randn(M, D, device=dev).bfloat16()
g = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
dgm, dbt, dls, dbias = (torch.zeros(D, device=dev) for _ in range(4))
ws = torch.empty(K.norm_ws_floats(D), device=dev)


def run(dy, fused):
    K.norm_bwd(d, dy, dx, dx_accumulate=True, dgamma=dgm, dbeta=dbt, ws=ws, param_accumulate=True,
               ls_branch=(ls, yb, g, dls, dbias) if fused else None)


for fused in (True, False):
    res = {}
    for name, dy in (("f32", dyf), ("bf16", dyb)):
        run(dy, fused)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                run(dy, fused)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) / 20 * 1e3)
        res[name] = sorted(ts)[2]
    print(f"ls_fused={fused}: " + " | ".join(f"dy {k}: {v:.1f} us" for k, v in res.items()), flush=True)
