"""slx_gemm_bf16 vs slx_gemm_lt (hipBLASLt) on plain NT step GEMM shapes (HIP events, median of 5 x 20 calls).
usage: python tools/gemm_lt_probe.py [M,N,K,f32 ...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
SHAPES = [  # (M, N, K, f32 out, site)
    (6384, 960, 9728, True, "Qwen2 gate/up dgrad"),
    (6384, 896, 4928, True, "Qwen2 down fwd (+resid)"),
    (6384, 896, 960, True, "Qwen2 o fwd (+resid)"),
    (6384, 1024, 1152, True, "Qwen2 q|k|v dgrad"),
    (6384, 960, 896, True, "Qwen2 o dgrad"),
    (6384, 4928, 896, False, "Qwen2 down dgrad"),
    (16400, 1024, 1024, False, "ViT proj dgrad"),
    (16400, 1024, 3072, False, "ViT qkv dgrad"),
    (16400, 1024, 4096, False, "ViT fc1 dgrad"),
]
if sys.argv[1:]:
    SHAPES = [tuple(int(x) for x in a.split(",")[:3]) + (a.split(",")[3] == "1", a) for a in sys.argv[1:]]


def t(fn, n=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / n)
    return sorted(ts)[2] * 1e3


for M, N, Kd, f32, site in SHAPES:
    A = torch.randn(M, Kd, device=dev).bfloat16()
    B = torch.randn(N, Kd, device=dev).bfloat16()
    D = torch.empty(M, N, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
    fl = 2.0 * M * N * Kd
    ours = t(lambda: K.mm(A, B, D))
    lt = t(lambda: K.mm_lt(A, B, D))
    print(f"{site:26s} {M}x{N}x{Kd} {'f32' if f32 else 'bf16'}: slx {ours:6.1f} us ({fl / ours / 1e6:5.0f} TF) | "
          f"hipBLASLt {lt:6.1f} us ({fl / lt / 1e6:5.0f} TF)", flush=True)
