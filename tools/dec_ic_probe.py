"""Decode Infinity Cache probe: (1) the gate/up GEMV (Qwen2-0.5B, 9728 x 896 bf16) cold vs right after its weights
were read by slx_dec_prefetch; (2) slx_dec_prefetch's own bandwidth per workgroup count; (3) whether two branches of a
captured hipGraph (GEMVs on one stream, a prefetch on a forked one) run concurrently."""
import ctypes
import statistics

import torch

from simlingo_amd import kernels as K
from simlingo_amd import decode as D

dev = torch.device("cuda", 0)
lib = K.lib()
N, Kd = 9728, 896
W = (torch.randn(N, Kd, device=dev) * 0.02).to(torch.bfloat16)
xb = torch.randn(Kd, device=dev).to(torch.bfloat16)
out = torch.zeros(N // 2, dtype=torch.bfloat16, device=dev)
desc = D._gemv_desc(D.DEC_SWIGLU, W, N, Kd, xb=xb, out=out)
flush = torch.empty(1 << 30, dtype=torch.uint8, device=dev)
sink = torch.zeros(256, dtype=torch.int32, device=dev)


def prefetch(ts, nb):
    ptrs = (ctypes.c_void_p * 4)(*([t.data_ptr() for t in ts] + [0] * (4 - len(ts))))
    nbytes = (ctypes.c_int64 * 4)(*([t.numel() * t.element_size() for t in ts] + [0] * (4 - len(ts))))
    K.check(lib.slx_dec_prefetch(ptrs, nbytes, len(ts), nb, None, K.P(sink), K.stream_ptr()), "slx_dec_prefetch")


def gemv():
    K.check(lib.slx_dec_gemv(ctypes.byref(desc), K.stream_ptr()), "slx_dec_gemv")


def timed(fn, reps=20, pre=None):
    ts = []
    for _ in range(reps):
        if pre:
            pre()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return statistics.median(ts)


gemv(); prefetch([flush], 1024); torch.cuda.synchronize()
cold = timed(gemv, pre=lambda: prefetch([flush], 1024))
warm_ic = timed(gemv, pre=lambda: (prefetch([flush], 1024), prefetch([W], 256)))
hot = timed(gemv)
print(f"gate/up GEMV {N}x{Kd} ({W.numel() * 2 / 1e6:.1f} MB): cold {cold:.2f} us, after prefetch {warm_ic:.2f} us, "
      f"back-to-back {hot:.2f} us", flush=True)
Wl = torch.empty(30 << 20, dtype=torch.uint8, device=dev)
for nb in (64, 128, 256, 512, 1024, 2048):
    t = timed(lambda: prefetch([Wl], nb), pre=lambda: prefetch([flush], 1024))
    print(f"prefetch 30 MiB cold, {nb} workgroups: {t:.2f} us = {Wl.numel() / t / 1e3:.0f} GB/s", flush=True)

# graph concurrency: 20 GEMVs on the capture stream, a 1 GiB prefetch on a forked stream
side = torch.cuda.Stream(dev)


def capture(main, branch):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        cur = torch.cuda.current_stream()
        if branch:
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                prefetch([flush], 256)
        if main:
            for _ in range(20):
                gemv()
        if branch:
            cur.wait_stream(side)
    return g


for name, m, b in (("gemv x20", True, False), ("prefetch 1 GiB", False, True), ("both, forked", True, True)):
    g = capture(m, b)
    g.replay(); torch.cuda.synchronize()
    print(f"graph {name}: {timed(g.replay):.1f} us", flush=True)
