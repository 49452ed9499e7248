"""Main-loop / split-K A/B for the Qwen2 data-gradient GEMMs (f32 [dx | dT] outputs, K-concatenated LoRA):
gate|up dgrad (6384 x 960 x 9728), o dgrad (6384 x 960 x 896), qkv dgrad (6384 x 1024 x 1152).
HIP events, random operands, cases interleaved in one process; prints the median per case."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
SHAPES = {"gu": (6384, 960, 9728), "o": (6384, 960, 896), "qkv": (6384, 1024, 1152)}
CONF = [("auto", 0, 0), ("v3", 7, -1), ("v3 s2", 7, 2), ("v3 s3", 7, 3), ("v3 s4", 7, 4), ("v2 s2", 2, 2),
        ("v256x128", 5, -1), ("v256x128 s2", 5, 2)]
cases = {}
for name, (M, N, Kd) in SHAPES.items():
    A = torch.randn(M, Kd, device=dev).bfloat16()
    B = torch.randn(Kd, N, device=dev).bfloat16()
    C = torch.empty(M, N, device=dev)
    for cname, v, sp in CONF:
        def f(A=A, B=B, C=C, M=M, N=N, Kd=Kd, v=v, sp=sp):
            K.gemm(A, B, C, M, N, Kd, K.GEMM_NN, Kd, N, N, variant=v, ksplit_max=sp)
        cases[f"{name:4s} {cname}"] = (f, 2.0 * M * N * Kd)
for f, _ in cases.values():
    f()
torch.cuda.synchronize()
times = {k: [] for k in cases}
for _ in range(5):
    for k, (f, _) in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 5 * 1e3)
for k, v in times.items():
    v.sort()
    t = v[len(v) // 2]
    print(f"{k:20s} {t:8.1f} us {cases[k][1] / t / 1e6:7.0f} TF", flush=True)
