"""InternViT weight-gradient pairs through slx_gemm_bf16_pair, as the engine calls them (TN, f32 accumulate, K = 16400
tokens): fc2.w + fc1.w and proj.w + qkv.w. Run under different SLX_SPLIT_REDUCE_MAX to compare the in-launch slab
reduction with f32 atomics for the 4-way split of the proj + qkv pair. Median of 5 x 10 calls."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
T = 16400
r = lambda *s: (torch.randn(*s, device=dev) * 0.1).bfloat16()  # noqa: E731
g, o, h1, hact, dh, h2 = r(T, 1024), r(T, 1024), r(T, 1024), r(T, 4096), r(T, 4096), r(T, 1024)
dqkv = r(T, 3072)
Gp, Gq = torch.zeros(1024, 1024, device=dev), torch.zeros(3072, 1024, device=dev)
G2, G1 = torch.zeros(1024, 4096, device=dev), torch.zeros(4096, 1024, device=dev)
KS = int(os.environ.get("KSMAX", "0"))  # cap on the pair's K splits (0 = the launcher's one-round choice)
pairs = {"fc2+fc1": lambda: K.mm_pair((g, hact, G2), (dh, h2, G1), ksplit_max=KS),
         "proj+qkv": lambda: K.mm_pair((g, o, Gp), (dqkv, h1, Gq), ksplit_max=KS)}
for name, run in pairs.items():
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
    print(f"SLX_SPLIT_REDUCE_MAX={os.environ.get('SLX_SPLIT_REDUCE_MAX', '2')} KSMAX={KS} {name}: {sorted(ts)[2]:.1f} us", flush=True)
