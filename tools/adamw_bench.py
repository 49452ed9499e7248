"""slx_adamw alone at the VLA step's flat size (N env, default 315M parameters): us per call and GB/s at 30 B/param
(read p g m v, write p m v + bf16 copy). Usage: [SLX_LIB_PATH=...] python tools/adamw_bench.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

n = int(os.environ.get("N", str(315_000_000)))
dev = torch.device("cuda")
p, g, m, v = (torch.rand(n, device=dev) for _ in range(4))
pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
ss = torch.ones(1, device=dev)
run = lambda: K.call("slx_adamw", K.P(p), K.P(g), K.P(m), K.P(v), K.P(pbf), n, 1e-6, 0.9, 0.999, 1e-8, 0.1, 3,  # noqa
                     K.P(ss), 0.3, 1.0, K.stream_ptr())
run()
torch.cuda.synchronize()
ts = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        run()
    e1.record()
    torch.cuda.synchronize()
    ts.append(e0.elapsed_time(e1) / 10 * 1e3)
us = sorted(ts)[2]
print(f"{os.environ.get('SLX_LIB_PATH', 'new')}: adamw n={n}: {us:.1f} us  {30 * n / us / 1e3:.0f} GB/s", flush=True)
