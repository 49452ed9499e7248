"""slx_gemm_bf16 vs hipBLASLt (torch.mm, out_dtype f32) vs slx_gemm_lt on plain step GEMM shapes (HIP events)."""
import torch, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd import kernels as K
dev = torch.device("cuda")
def t(fn, n=20):
    fn(); torch.cuda.synchronize(); ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n): fn()
        e1.record(); torch.cuda.synchronize(); ts.append(e0.elapsed_time(e1) / n)
    return sorted(ts)[2] * 1e3
for (M, N, Kd) in [(6384, 960, 9728), (6384, 896, 4864), (16400, 1024, 1024), (6384, 4928, 896)]:
    A = torch.randn(M, Kd, device=dev).bfloat16(); B = torch.randn(N, Kd, device=dev).bfloat16()
    Cf = torch.empty(M, N, device=dev); Cb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    fl = 2.0 * M * N * Kd
    ours_f = t(lambda: K.mm(A, B, Cf)); ours_b = t(lambda: K.mm(A, B, Cb))
    lt_b = t(lambda: torch.mm(A, B.t(), out=Cb))
    try:
        lt_f = t(lambda: torch.mm(A, B.t(), out_dtype=torch.float32))
    except Exception as e:
        lt_f = float('nan'); print(e)
    ref = A.float() @ B.float().t()
    d = (torch.mm(A, B.t(), out_dtype=torch.float32) - ref).abs().max().item()
    print(f"{M}x{N}x{Kd}: ours f32 {ours_f:.1f} us ({fl/ours_f/1e6:.0f} TF) bf16 {ours_b:.1f} | blasLt bf16 {lt_b:.1f} f32 {lt_f:.1f} us ({fl/lt_f/1e6:.0f} TF) maxdiff {d:.2e}", flush=True)
