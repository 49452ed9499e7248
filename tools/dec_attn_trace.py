"""Phase timeline of the decode attention kernel (slx_dec_attn) at the agent geometry: Qwen2-0.5B (14 q / 2 kv
heads), a 1024-row cache with the token at position 680. Prints the kernel time (HIP events, 200 back-to-back
launches) and, from one traced launch, workgroup (0,0)'s phase timestamps and the merger's, in microseconds."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import decode  # noqa: E402,F401  (registers the slx_dec_* signatures)
from simlingo_amd import kernels as K  # noqa: E402

K.register("slx_dec_attn_set_trace", [K.c_vp])
dev = torch.device("cuda")
Hq, Hkv, lmax, pos = 14, 2, 1024, int(sys.argv[1]) if len(sys.argv) > 1 else 680
ld = (Hq + 2 * Hkv) * 64
cache = (torch.randn(lmax, ld, device=dev) * 0.5).bfloat16()
cos, sin = K.rope_tables(lmax, 1e6, dev)
st = torch.tensor([pos, 0, 0, 100, -1, 0, 0, 0], dtype=torch.int32, device=dev)
ws = torch.zeros(K.lib().slx_dec_attn_ws_floats(Hq, Hkv, lmax), device=dev)
out = torch.empty(Hq * 64, dtype=torch.bfloat16, device=dev)
lib = K.lib()


def call():
    K.check(lib.slx_dec_attn(K.P(cache), ld, Hq, Hkv, K.P(cos), K.P(sin), lmax, K.P(ws), K.P(out), K.P(st),
                             K.stream_ptr()), "slx_dec_attn")


for _ in range(20):
    call()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    call()
e1.record()
torch.cuda.synchronize()
print(f"slx_dec_attn: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per launch (back to back, incl. boundaries)")
tr = torch.zeros(64 + 256, dtype=torch.int64, device=dev)
for rep in range(3):
    tr.zero_()
    lib.slx_dec_attn_set_trace(ctypes.c_void_p(tr.data_ptr()))
    call()
    torch.cuda.synchronize()
    lib.slx_dec_attn_set_trace(ctypes.c_void_p(0))
    t = tr.cpu().tolist()
    ns = lib.slx_dec_attn_nsplit(lmax)
    starts = [v for v in t[64:64 + Hkv * ns] if v]
    base = min(starts)
    us = lambda v: f"{(v - base) * 0.01:6.2f}" if v else "   -  "  # 100 MHz wall clock
    names = ["start", "st loaded", "K/V/q in LDS", "scores", "softmax", "published", "arrived", "-", "merge start",
             "m/l loaded", "merged"]
    print(f"rep {rep}: workgroup starts span {(max(starts) - base) * 0.01:.2f} us over {len(starts)} workgroups")
    print("   " + "  ".join(f"{n}={us(t[i])}" for i, n in enumerate(names) if n != "-"))
