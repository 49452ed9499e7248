"""Microbenchmark of the LoRA side kernels on the Qwen2 shapes of config 3 (M = 8 x 798 rows, dropout 0.1):
per site group, slx_lora_down and slx_lora_bwd (dA + dx) times and the HBM rate their compulsory bytes imply."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
M, d, F = 6384, 896, 4864
GROUPS = {"qkv": (d, 3), "o": (d, 1), "gu": (d, 2), "down": (F, 1)}


def t_ms(fn, n=20):
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
    return sorted(ts)[2]


for name, (kin, ns) in GROUPS.items():
    x = torch.randn(M, kin, device=dev).bfloat16()
    As = [(torch.randn(32, kin, device=dev) * 0.05).bfloat16() for _ in range(ns)]
    bits = [torch.empty(M, kin // 32, device=dev, dtype=torch.int32) for _ in range(ns)]
    K.dropout_bits([(17 + j, bits[j], kin, kin) for j in range(ns)], M, 0.1)
    t = torch.empty(M, 32 * ns, device=dev).bfloat16()
    Af = [K.lora_pack_a(a) for a in As]  # the engine keeps these packed copies (refreshed per optimizer step)
    td = t_ms(lambda: K.lora_down(x, Af, t, [0] * ns, p=0.1, bits=bits, packed=True))
    dt = torch.randn(M, 32 * ns, device=dev)
    dAs = [torch.zeros(32, kin, device=dev) for _ in range(ns)]
    dx = torch.zeros(M, kin, device=dev)
    Ax = [K.lora_pack_a(a, 1) for a in As]
    tb = t_ms(lambda: K.lora_bwd(x, dt, Ax, bits, dAs, dx=dx, p=0.1, packed=True))
    ta = t_ms(lambda: K.lora_bwd(x, dt, Ax, bits, dAs, p=0.1, packed=True))
    xb = M * kin * 2 / 1e9
    bb = ns * M * kin / 8 / 1e9
    print(f"{name:5s} kin {kin} ns {ns}: down {td * 1e3:6.1f} us ({(xb + bb) / td:5.2f} TB/s) | dA {ta * 1e3:6.1f} us "
          f"({(xb + bb) / ta:5.2f} TB/s) | dx {(tb - ta) * 1e3:6.1f} us "
          f"({(xb + bb + 2 * M * kin * 4 / 1e9) / max(tb - ta, 1e-9):5.2f} TB/s)", flush=True)
