"""A/B microbenchmark of slx_gemm_bf16 main-loop variants on the hot-path shapes (HIP events,
random operands, variants interleaved in one process)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K  # noqa: E402

SHAPES = {  # name: (M, N, K, layout)
    "vit_qkv": (16400, 3072, 1024, K.GEMM_NT),
    "vit_fc1": (16400, 4096, 1024, K.GEMM_NT),
    "vit_fc2": (16400, 1024, 4096, K.GEMM_NT),
    "vit_proj": (16400, 1024, 1024, K.GEMM_NT),
    "vit_fc2_dgrad": (16400, 4096, 1024, K.GEMM_NN),
    "vit_fc1_dgrad": (16400, 1024, 4096, K.GEMM_NN),
    "vit_fc1_wgrad": (4096, 1024, 16400, K.GEMM_TN),
    "vit_qkv_wgrad": (3072, 1024, 16400, K.GEMM_TN),
    "vit_proj_wgrad": (1024, 1024, 16400, K.GEMM_TN),
    "llm_gu_dgradx": (6384, 960, 9728, K.GEMM_NN),
    "llm_qkv_dgrad": (6384, 1024, 1152, K.GEMM_NN),
    "llm_down_dgrad": (6384, 4928, 896, K.GEMM_NN),
    "llm_qkv": (6384, 1152, 896, K.GEMM_NT),
    "llm_gateup": (6384, 9728, 896, K.GEMM_NT),
    "llm_down": (6384, 896, 4864, K.GEMM_NT),
    "llm_gu_dgrad": (6384, 896, 9728, K.GEMM_NN),
    "llm_gu_dgrad_nt": (6384, 960, 9728, K.GEMM_NT),   # the step's form: [dx | dt] over the transposed W_cat copy
    "sq8192": (8192, 8192, 8192, K.GEMM_NT),
    "tn8192": (8192, 8192, 8192, K.GEMM_TN),   # both operands MN-contiguous (tr-reads), no split-K
    "nn8192": (8192, 8192, 8192, K.GEMM_NN),
    "tn4096x1024x8192": (4096, 1024, 8192, K.GEMM_TN),  # one split of the fc1.w gradient
    # weight gradients with a transposed (feature-major) copy of the forward activation X:
    # TT: dW = dY^T . Xt^T  (A = dY [tok][out] MN-contiguous, B = Xt [in][tok] K-contiguous)
    # NN: dW^T = Xt . dY     (A = Xt K-contiguous, B = dY [tok][out] MN-contiguous; output transposed)
    "vit_fc1_wgrad_tt": (4096, 1024, 16400, K.GEMM_TT),
    "vit_fc1_wgrad_nn": (1024, 4096, 16400, K.GEMM_NN),
    "vit_fc2_wgrad_tt": (1024, 4096, 16400, K.GEMM_TT),
    "vit_fc2_wgrad_nn": (4096, 1024, 16400, K.GEMM_NN),
    "vit_qkv_wgrad_tt": (3072, 1024, 16400, K.GEMM_TT),
    "vit_qkv_wgrad_nn": (1024, 3072, 16400, K.GEMM_NN),
    "vit_proj_wgrad_tt": (1024, 1024, 16400, K.GEMM_TT),
    "vit_proj_wgrad_nn": (1024, 1024, 16400, K.GEMM_NN),
    # NT: both operands token-contiguous copies (dY^T and X^T, tokens padded to 16448 = 257 * 64)
    "vit_fc1_wgrad_nt": (4096, 1024, 16448, K.GEMM_NT),
    "vit_fc2_wgrad_nt": (1024, 4096, 16448, K.GEMM_NT),
    "vit_qkv_wgrad_nt": (3072, 1024, 16448, K.GEMM_NT),
}
VARIANTS = [int(v) for v in os.environ.get("VARIANTS", "1,2,3,4,5,6").split(",")]
dev = torch.device("cuda")
only = sys.argv[1:] or list(SHAPES)
for name in only:
    M, N, Kd, lay = SHAPES[name]
    A = (torch.randn(M, Kd, device=dev) if lay in (K.GEMM_NT, K.GEMM_NN) else torch.randn(Kd, M, device=dev)).bfloat16()
    B = (torch.randn(N, Kd, device=dev) if lay in (K.GEMM_NT, K.GEMM_TT) else torch.randn(Kd, N, device=dev)).bfloat16()
    # weight/data gradients are f32 outputs in the engine (split-K eligible)
    C = torch.empty(M, N, device=dev, dtype=torch.float32 if "grad" in name else torch.bfloat16)
    ref = None
    if M * N * Kd < 3e11:
        a = A.float() if lay in (K.GEMM_NT, K.GEMM_NN) else A.float().t()
        b = B.float().t() if lay in (K.GEMM_NT, K.GEMM_TT) else B.float()
        ref = a @ b
    times = {v: [] for v in VARIANTS}
    errs = {}
    for v in VARIANTS:
        K.gemm(A, B, C, M, N, Kd, lay, A.stride(0), B.stride(0), C.stride(0), variant=v)
        torch.cuda.synchronize()
        if ref is not None:
            errs[v] = ((C.float() - ref).abs().max() / ref.abs().max()).item()
    for rnd in range(5):
        for v in VARIANTS:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            n = 10
            e0.record()
            for _ in range(n):
                K.gemm(A, B, C, M, N, Kd, lay, A.stride(0), B.stride(0), C.stride(0), variant=v)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / n)
    # vendor library (hipBLASLt via torch.mm) on the same layout, for headroom
    a_ = A if lay in (K.GEMM_NT, K.GEMM_NN) else A.t()
    b_ = B.t() if lay in (K.GEMM_NT, K.GEMM_TT) else B
    Cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    tl = []
    for rnd in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            torch.mm(a_, b_, out=Cb)
        e1.record()
        torch.cuda.synchronize()
        tl.append(e0.elapsed_time(e1) / 10)
    line = f"{name:14s} {M:6d}x{N:5d}x{Kd:5d} | blasLt {2.0 * M * N * Kd / sorted(tl)[2] / 1e9:6.0f} TF "
    for v in VARIANTS:
        ms = sorted(times[v])[len(times[v]) // 2]
        tf = 2.0 * M * N * Kd / ms / 1e9
        line += f"| v{v}: {tf:6.0f} TF" + (f" e{errs[v]:.0e}" if v in errs else "")
    print(line, flush=True)
