"""Microbenchmark of slx_attn_fwd / slx_attn_bwd on the two hot-path shapes (HIP events).
FLOPs: fwd 4*B*Hq*S_q*S_k*64 (halved for causal), bwd 2.5x fwd."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
SHAPES = {"vit": dict(B=16, S=1025, Hq=16, Hkv=16, causal=False), "llm": dict(B=8, S=798, Hq=14, Hkv=2, causal=True),
          # the InternViT shape without its class token: what the 1025th row's tail blocks cost
          "vit1024": dict(B=16, S=1024, Hq=16, Hkv=16, causal=False),
          # Qwen2 without the GQA sharing (7 times the K/V heads): what the grouped K/V costs or saves
          "llm_mha": dict(B=8, S=798, Hq=14, Hkv=14, causal=True)}


def timeit(fn, n=10):
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


save = None
args = sys.argv[1:]
if "--save" in args:
    i = args.index("--save")
    save = args[i + 1]
    args = args[:i] + args[i + 2:]
outs = {}
for name in args or list(SHAPES):
    c = SHAPES[name]
    B, S, Hq, Hkv = c["B"], c["S"], c["Hq"], c["Hkv"]
    torch.manual_seed(0)
    qkv = (torch.randn(B * S, (Hq + 2 * Hkv) * 64, device=dev) * 0.5).bfloat16()
    q, k, v = qkv[:, :Hq * 64], qkv[:, Hq * 64:(Hq + Hkv) * 64], qkv[:, (Hq + Hkv) * 64:]
    o = torch.empty(B * S, Hq * 64, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * Hq * S, device=dev)
    seql = torch.full((B,), S, dtype=torch.int32, device=dev)
    kw = dict(B=B, S=S, Hq=Hq, Hkv=Hkv, causal=c["causal"])
    if c["causal"]:
        kw["seqlens"] = seql
    fl = 4.0 * B * Hq * S * S * 64 * (0.5 if c["causal"] else 1.0)
    tf = timeit(lambda: K.attn_fwd(q, k, v, o, lse, **kw))
    dout = torch.randn(B * S, Hq * 64, device=dev).bfloat16()
    dqkv = torch.empty_like(qkv)
    ws = K.attn_ws(B, S, Hq, Hkv, dev)
    tb = timeit(lambda: K.attn_bwd(q, k, v, o, lse, dout, dqkv[:, :Hq * 64], dqkv[:, Hq * 64:(Hq + Hkv) * 64],
                                   dqkv[:, (Hq + Hkv) * 64:], ws, **kw))
    print(f"{name}: fwd {tf * 1e3:7.1f} us {fl / tf / 1e9:6.0f} TF | bwd {tb * 1e3:7.1f} us {2.5 * fl / tb / 1e9:6.0f} TF"
          "", flush=True)
    if save:
        outs[name] = {"o": o.cpu(), "lse": lse.cpu(), "dqkv": dqkv.cpu()}
if save:
    torch.save(outs, save)
