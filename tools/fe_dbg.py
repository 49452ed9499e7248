import sys, torch
sys.path.insert(0, "/root/repo")
from simlingo_amd import kernels as K
dev = torch.device("cuda")
M, N, Kd = 8192, 2304, 192
g = torch.Generator(device=dev).manual_seed(1)
x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
w = (torch.randn(N, Kd, device=dev, generator=g) * 0.1).bfloat16()
bias = torch.randn(N, device=dev, generator=g)
pre = x.float() @ w.float().t() + bias
def report(name, out, ref, atol):
    bad = ~((out.float() - ref).abs() <= atol + 1e-2 * ref.abs())
    nb = int(bad.sum())
    print(name, "bad", nb, flush=True)
    if nb:
        idx = bad.nonzero()
        r, c = idx[:, 0], idx[:, 1]
        print("  rows%16", torch.bincount(r % 16, minlength=16).tolist())
        print("  cols%64", torch.bincount(c % 64, minlength=64).tolist())
        print("  tile rows", torch.bincount(r // 256).tolist()[:40])
        print("  tile cols", torch.bincount(c // 256).tolist())
        print("  wave col (c%256)//64", torch.bincount((c % 256) // 64, minlength=4).tolist(), "wave row (r%256)//128", torch.bincount((r % 256) // 128, minlength=2).tolist())
for v in (8, 11):
    plain = torch.full((M, N), float('nan'), device=dev).bfloat16()
    K.gemm(x, w, plain, M, N, Kd, K.GEMM_NT, Kd, Kd, N, bias=bias, variant=v)
    report(f"v{v} plain", plain, pre, 3e-2)
    h = torch.full((M, N), float('nan'), device=dev).bfloat16(); hpre = h.clone()
    K.gemm(x, w, h, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=K.EPI_GELU, bias=bias, aux_out=hpre, ldaux_out=N, variant=v)
    report(f"v{v} hpre", hpre, pre, 3e-2)
    report(f"v{v} h", h, torch.nn.functional.gelu(pre), 3e-2)
    o32 = torch.full((M, N), float('nan'), device=dev)
    K.gemm(x, w, o32, M, N, Kd, K.GEMM_NT, Kd, Kd, N, variant=v, ksplit_max=-1)
    report(f"v{v} f32", o32, pre - bias, 3e-3)
