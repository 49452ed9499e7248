"""Data-gradient GEMMs dX = dY @ W of the step, timed in the two layouts the weight can be held in: W [out,in]
(NN, what the step runs today) and a transposed copy W^T [in,out] (NT, the forward's layout). Default variant
selection, alternating order, median of 5.  Usage: python tools/nn_vs_nt.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
Mv = int(os.environ.get("MV", "16400"))
R = int(os.environ.get("R", "6384"))
SHAPES = [  # name, M, N(=in), K(=out), epi
    ("vit.qkv", Mv, 1024, 3072, None),
    ("vit.proj", Mv, 1024, 1024, None),
    ("vit.fc1", Mv, 1024, 4096, None),
    ("vit.fc2+gelu'", Mv, 4096, 1024, "gelu_bwd"),
    ("llm.qkv", R, 896, 1152, None),
    ("llm.o", R, 896, 896, None),
    ("llm.gate_up", R, 896, 9728, None),
    ("llm.down", R, 4864, 896, None),
]
if os.environ.get("ONLY"):
    SHAPES = [x for x in SHAPES if x[0] in os.environ["ONLY"].split(",")]
SHAPES += [("llm.lm_head", int(os.environ.get("RLOSS", "128")), 896, 151680, None)] if os.environ.get("LMHEAD") else []


def timeit(run, reps=10):
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        run()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


tot = [0.0, 0.0]
for name, M, N, Kd, epi in SHAPES:
    dy = torch.randn(M, Kd, device=dev).to(torch.bfloat16)
    W = (torch.randn(Kd, N, device=dev) * 0.03).to(torch.bfloat16)  # [out, in]: NN operand
    WT = W.t().contiguous()  # [in, out]: NT operand
    out = torch.empty(M, N, device=dev, dtype=torch.float32 if os.environ.get("OUTF32") else torch.bfloat16)
    kw = {}
    if epi == "gelu_bwd":
        aux = torch.randn(M, N, device=dev).to(torch.bfloat16)
        kw = dict(epi=K.EPI_GELU_BWD, aux=aux, ldaux=N)
    nn = lambda: K.mm(dy, W, out, tb=False, **kw)  # noqa: E731
    nt = lambda: K.mm(dy, WT, out, tb=True, **kw)  # noqa: E731
    r0 = out.clone()
    nn()
    torch.cuda.synchronize()
    r0.copy_(out)
    nt()
    torch.cuda.synchronize()
    diff = (out.float() - r0.float()).abs().max().item()
    a, b = [], []
    for _ in range(5):
        a.append(timeit(nn))
        b.append(timeit(nt))
    ta, tbb = sorted(a)[2], sorted(b)[2]
    tot[0] += ta
    tot[1] += tbb
    fl = 2.0 * M * N * Kd
    print(f"{name:16s} M={M} N={N} K={Kd}: NN {ta:7.1f} us ({fl / ta / 1e6:5.0f} TF)  NT {tbb:7.1f} us "
          f"({fl / tbb / 1e6:5.0f} TF)  ratio {tbb / ta:.3f}  max|diff| {diff:.3g}", flush=True)
print(f"sum NN {tot[0]:.1f} us  NT {tot[1]:.1f} us", flush=True)
