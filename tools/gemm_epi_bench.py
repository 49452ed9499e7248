"""A/B of slx_gemm_bf16 main-loop variants on the epilogue-heavy InternViT GEMMs of the VLA step, with the real
fused epilogues (random operands, variants interleaved in one process):
  fc1      16400 x 4096 x 1024 NT, bias + GELU, bf16 out + bf16 pre-activation aux
  fc2bwd   16400 x 4096 x 1024 NN, GELU' against the bf16 aux, bf16 out, fc1.b column sums
  nn_plain / nn_f32 / fc2bwd_nocs / nt_plain: the same shapes with plain bf16 / f32 stores, GELU' without the column
           sums, and the fc1 NT shape without bias/GELU (epilogue ablations)
  fc2      16400 x 1024 x 4096 NT, bias + layer-scale residual (f32), f32 out + bf16 branch aux
  proj     16400 x 1024 x 1024 NT, same epilogue as fc2
VARIANTS=0,2,5,7 (env) selects the variants (0 = the host cost model's choice)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

dev = torch.device("cuda")
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "0,2,5,7").split(",")]
M = 16400


def case(name):
    bf = torch.bfloat16
    if name == "fc1":
        N, Kd = 4096, 1024
        A, B = torch.randn(M, Kd, device=dev).to(bf), (torch.randn(N, Kd, device=dev) * 0.03).to(bf)
        C, aux, bias = torch.empty(M, N, device=dev, dtype=bf), torch.empty(M, N, device=dev, dtype=bf), torch.randn(N, device=dev)
        return N, Kd, lambda v: K.gemm(A, B, C, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=K.EPI_GELU, bias=bias, aux_out=aux,
                                       ldaux_out=N, variant=v)
    if name in ("nn_plain", "nn_f32", "fc2bwd_nocs", "nt_plain"):  # epilogue ablations of the fc1/fc2-dgrad shapes
        N, Kd = 4096, 1024
        bt = (Kd, N) if name != "nt_plain" else (N, Kd)
        A, B = torch.randn(M, Kd, device=dev).to(bf), (torch.randn(*bt, device=dev) * 0.03).to(bf)
        C = torch.empty(M, N, device=dev, dtype=torch.float32 if name == "nn_f32" else bf)
        aux = torch.randn(M, N, device=dev).to(bf)
        lay, ldb = (K.GEMM_NT, Kd) if name == "nt_plain" else (K.GEMM_NN, N)
        kw = dict(epi=K.EPI_GELU_BWD, aux=aux, ldaux=N) if name == "fc2bwd_nocs" else {}
        return N, Kd, lambda v: K.gemm(A, B, C, M, N, Kd, lay, Kd, ldb, N, variant=v, **kw)
    if name == "fc2bwd":
        N, Kd = 4096, 1024
        A, B = torch.randn(M, Kd, device=dev).to(bf), (torch.randn(Kd, N, device=dev) * 0.03).to(bf)
        C, aux, cs = torch.empty(M, N, device=dev, dtype=bf), torch.randn(M, N, device=dev).to(bf), torch.zeros(N, device=dev)
        return N, Kd, lambda v: K.gemm(A, B, C, M, N, Kd, K.GEMM_NN, Kd, N, N, epi=K.EPI_GELU_BWD, aux=aux, ldaux=N,
                                       colsum=cs, variant=v)
    N, Kd = (1024, 4096) if name == "fc2" else (1024, 1024)
    A, B = torch.randn(M, Kd, device=dev).to(bf), (torch.randn(N, Kd, device=dev) * 0.03).to(bf)
    C, resid, ls = torch.empty(M, N, device=dev), torch.randn(M, N, device=dev), torch.rand(N, device=dev)
    aux, bias = torch.empty(M, N, device=dev, dtype=bf), torch.randn(N, device=dev)
    return N, Kd, lambda v: K.gemm(A, B, C, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=K.EPI_RESID_LS, bias=bias, resid=resid,
                                   ldr=N, ls=ls, aux_out=aux, ldaux_out=N, variant=v)


for name in sys.argv[1:] or ["fc1", "fc2bwd", "fc2", "proj"]:
    N, Kd, run = case(name)
    times = {v: [] for v in VARIANTS}
    for v in VARIANTS:
        run(v)
    torch.cuda.synchronize()
    for _ in range(5):
        for v in VARIANTS:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run(v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / 10)
    line = f"{name:7s} {M}x{N}x{Kd} "
    for v in VARIANTS:
        ms = sorted(times[v])[2]
        line += f"| v{v}: {ms * 1e3:6.1f} us {2.0 * M * N * Kd / ms / 1e9:5.0f} TF "
    print(line, flush=True)
