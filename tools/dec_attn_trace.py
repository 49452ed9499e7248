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


K.register("slx_dec_attn_force_split", [ctypes.c_int])
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for split in (0, 1):
    lib.slx_dec_attn_force_split(split)
    for _ in range(20):
        call()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(200):
        call()
    e1.record()
    torch.cuda.synchronize()
    form = "split + last-arriver merge" if split else "one workgroup per kv head (MFMA)"
    print(f"slx_dec_attn [{form}]: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per launch (back to back, incl. boundaries)")
lib.slx_dec_attn_force_split(0)
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

# ---- the layer's GEMVs (QKV with the fused RMSNorm, down + residual) -------------------------------------------------
from simlingo_amd.decode import DEC_RESID, DEC_STORE_ROW, _gemv_desc  # noqa: E402

d, F = 896, 4864
X = torch.randn(d, device=dev)
gamma = torch.rand(d, device=dev) + 0.5
Wqkv = (torch.randn(ld, d, device=dev) * 0.02).bfloat16()
bias = torch.randn(ld, device=dev)
Wd = (torch.randn(d, F, device=dev) * 0.02).bfloat16()
act = torch.randn(F, device=dev).bfloat16()
gemvs = {
    "qkv (N 1152, K 896, norm fused)": _gemv_desc(DEC_STORE_ROW, Wqkv, ld, d, X=X, gamma=gamma, eps=1e-6, bias=bias,
                                                  out=cache, out_ld=ld, state=st),
    "down (N 896, K 4864, + resid)": _gemv_desc(DEC_RESID, Wd, d, F, xb=act, resid=X.clone(), state=st),
}
for name, desc in gemvs.items():
    def gcall(desc=desc):
        K.check(lib.slx_dec_gemv(ctypes.byref(desc), K.stream_ptr()), "slx_dec_gemv")
    for _ in range(20):
        gcall()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(200):
        gcall()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name}: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us per launch (back to back)")
    big = torch.zeros(128 + 4096, dtype=torch.int64, device=dev)
    for rep in range(2):
        big.zero_()
        torch.empty(64 << 20, dtype=torch.uint8, device=dev).fill_(1)  # evict: the weights come from HBM as in a step
        torch.cuda.synchronize()
        lib.slx_dec_attn_set_trace(ctypes.c_void_p(big.data_ptr()))
        gcall()
        torch.cuda.synchronize()
        lib.slx_dec_attn_set_trace(ctypes.c_void_p(0))
        t = big.cpu().tolist()
        starts = [v for v in t[128:] if v]
        base = min(starts)
        print(f"   rep {rep}: {len(starts)} workgroups start over {(max(starts) - base) * 0.01:.2f} us; workgroup 0: "
              f"loads issued {(t[32] - base) * 0.01:.2f}, x ready {(t[33] - base) * 0.01:.2f}, "
              f"rows done {(t[34] - base) * 0.01:.2f} us")
