"""Proxy timings for grouping the InternViT weight-gradient GEMMs into single v3 launches.

fc1 + fc2 weight gradients (4096x1024 and 1024x4096, K = 16400 tokens) grouped into one launch is timed as a
batch-2 v3 launch of the 4096x1024 shape (same tiles and K per block); qkv + proj (3072 + 1024 rows) grouped
is timed as one 4096x1024 v3 launch. Baselines: the shapes as the engine runs them today (automatic variant).
HIP events, random operands, interleaved repeats in one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
T = 16400


def operands(M, N, batch=1):
    A = torch.randn(batch, T, M, device=dev).bfloat16()
    B = torch.randn(batch, T, N, device=dev).bfloat16()
    C = torch.zeros(batch, M, N, device=dev)
    return A, B, C


def run(M, N, batch=1, variant=0, split=0):
    A, B, C = operands(M, N, batch)

    def f():
        K.gemm(A, B, C, M, N, T, K.GEMM_TN, M, N, N, accumulate=True, batch=batch, sA=T * M, sB=T * N, sC=M * N,
               variant=variant, ksplit_max=split)
    return f


def pair(s1, s2, split=0, ws=True, variant=None):
    o1 = [t[0] for t in operands(*s1)]
    o2 = [t[0] for t in operands(*s2)]
    d = [K._gemm_desc(o[0], o[1], o[2], *K._mm_dims(o[0], o[1], o[2], True, False), o[0].stride(0), o[1].stride(0),
                      o[2].stride(0), accumulate=True, ksplit_max=split, split_ws=ws, variant=variant) for o in (o1, o2)]

    def f():
        K.check(K.lib().slx_gemm_bf16_pair(K.ctypes.byref(d[0]), K.ctypes.byref(d[1]), K.stream_ptr()), "pair")
    return f


if os.environ.get("SPLIT_AB"):  # in-launch split-K reduction vs f32 atomics (round 3)
    cases = {
        "fc2+fc1 pair atomics": pair((1024, 4096), (4096, 1024), ws=False),
        "fc2+fc1 pair in-launch reduce": pair((1024, 4096), (4096, 1024), ws=True),
        "proj+qkv pair atomics": pair((1024, 1024), (3072, 1024), ws=False),
        "proj+qkv pair in-launch reduce": pair((1024, 1024), (3072, 1024), ws=True),
        "fc2+fc1 pair reduce v8": pair((1024, 4096), (4096, 1024), ws=True, variant=8),
    }
else:
  cases = {
    "fc2+fc1 pair (auto split)": pair((1024, 4096), (4096, 1024)),
    "proj+qkv pair (auto split)": pair((1024, 1024), (3072, 1024)),
    "proj+qkv pair split 3": pair((1024, 1024), (3072, 1024), 3),
    "fc1_wgrad_auto": run(4096, 1024),
    "fc2_wgrad_auto": run(1024, 4096),
    "qkv_wgrad_auto": run(3072, 1024),
    "proj_wgrad_auto": run(1024, 1024),
    "fc12_group_v3s2 (b2 4096x1024)": run(4096, 1024, batch=2, variant=7, split=2),
    "fc12_group_v3s3 (b2 4096x1024)": run(4096, 1024, batch=2, variant=7, split=3),
    "qkvproj_group_v3s4 (4096x1024)": run(4096, 1024, variant=7, split=4),
    "qkvproj_group_v3s3 (4096x1024)": run(4096, 1024, variant=7, split=3),
    "fc1_wgrad_v3s4": run(4096, 1024, variant=7, split=4),
  }
for f in cases.values():
    f()
torch.cuda.synchronize()
times = {k: [] for k in cases}
for _ in range(5):
    for k, f in cases.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            f()
        e1.record()
        torch.cuda.synchronize()
        times[k].append(e0.elapsed_time(e1) / 5 * 1e3)
for k, v in times.items():
    v.sort()
    print(f"{k:36s} {v[len(v) // 2]:8.1f} us", flush=True)
