"""Per-tile cost split of the v3 GEMM: time vs K at fixed M x N (NT, bf16 out, random operands). The slope over K is
the main loop's cost per 64-deep K-step, the intercept the per-tile fixed cost (prologue fill + epilogue + stores).
Usage: python tools/gemm_ksweep.py [N ...]   (default N = 4096 1024)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
M = int(os.environ.get("M", "16384"))
VARIANT = int(os.environ.get("VARIANT", "7"))
OUT = os.environ.get("OUT", "bf16")
LAYOUT = os.environ.get("LAYOUT", "NT")  # NT: A [M][K], B [N][K]; NN: B [K][N]; TN: A [K][M], B [K][N]
KS = [int(k) for k in os.environ.get("KS", "512,1024,2048,4096").split(",")]


def timeit(run, reps=10):
    run()
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[2] * 1e3


for N in [int(a) for a in sys.argv[1:]] or [4096, 1024]:
    pts = []
    for Kd in KS:
        A = torch.randn(*((Kd, M) if LAYOUT == "TN" else (M, Kd)), device=dev).to(torch.bfloat16)
        B = (torch.randn(*((N, Kd) if LAYOUT == "NT" else (Kd, N)), device=dev) * 0.03).to(torch.bfloat16)
        C = torch.empty(M, N, device=dev, dtype=torch.bfloat16 if OUT == "bf16" else torch.float32)
        lay = {"NT": K.GEMM_NT, "NN": K.GEMM_NN, "TN": K.GEMM_TN}[LAYOUT]
        lda = M if LAYOUT == "TN" else Kd
        ldb = Kd if LAYOUT == "NT" else N
        us = timeit(lambda: K.gemm(A, B, C, M, N, Kd, lay, lda, ldb, N, variant=VARIANT, ksplit_max=-1))
        tiles = (M // 256) * (N // 256)
        rounds = tiles / 256
        pts.append((Kd, us))
        print(f"{LAYOUT} N={N} K={Kd}: {us:7.1f} us  {2.0 * M * N * Kd / us / 1e6:6.0f} TF  per-round {us / rounds:6.2f} us", flush=True)
    if len(pts) < 2:
        continue
    # least squares us = a + b * (K / 64)
    xs = [k / 64 for k, _ in pts]
    ys = [u for _, u in pts]
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    b = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
    a = my - b * mx
    rounds = (M // 256) * (N // 256) / 256
    print(f"N={N}: per round: fixed {a / rounds:.2f} us + {b / rounds * 1e3:.0f} ns per K-step "
          f"(ideal K-step at 2.4 GHz: {2048 / 2.4:.0f} ns)", flush=True)
