"""Microbenchmark of slx_gemm_bf16 on the hot-path shapes (HIP events, random operands)."""
import sys
import torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from simlingo_amd import kernels as K

SHAPES = {  # name: (M, N, K, layout)
    "vit_qkv": (16400, 3072, 1024, K.GEMM_NT),
    "vit_fc1": (16400, 4096, 1024, K.GEMM_NT),
    "vit_fc2": (16400, 1024, 4096, K.GEMM_NT),
    "vit_fc1_dgrad": (16400, 1024, 4096, K.GEMM_NN),
    "vit_fc1_wgrad": (4096, 1024, 16400, K.GEMM_TN),
    "llm_gateup": (6384, 9728, 896, K.GEMM_NT),
    "llm_down_dgrad": (6384, 4864, 896, K.GEMM_NN),
    "sq8192": (8192, 8192, 8192, K.GEMM_NT),
}
dev = torch.device("cuda")
for name, (M, N, Kd, lay) in SHAPES.items():
    A = (torch.randn(M, Kd, device=dev) if lay in (K.GEMM_NT, K.GEMM_NN) else torch.randn(Kd, M, device=dev)).bfloat16()
    B = (torch.randn(N, Kd, device=dev) if lay in (K.GEMM_NT, K.GEMM_TT) else torch.randn(Kd, N, device=dev)).bfloat16()
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    f = lambda: K.gemm(A, B, C, M, N, Kd, lay, A.stride(0), B.stride(0), C.stride(0))
    for _ in range(3): f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    tf = 2.0 * M * N * Kd / ms / 1e9
    print(f"{name:16s} M={M:6d} N={N:6d} K={Kd:6d}  {ms*1e3:9.1f} us  {tf:7.1f} TFLOP/s  ({tf/2500*100:5.1f}% of 2.5PF)", flush=True)
    ref = A.float() if lay in (K.GEMM_NT, K.GEMM_NN) else A.float().t()
    if M * N * Kd < 2e11:
        bb = B.float().t() if lay in (K.GEMM_NT, K.GEMM_TT) else B.float()
        err = (C.float() - ref @ bb).abs().max().item()
        print(f"   max err {err:.3e}")
