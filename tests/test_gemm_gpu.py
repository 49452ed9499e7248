"""GEMM parity: HIP bf16 MFMA GEMM vs a plain PyTorch fp32 matmul of the same bf16 operands."""
import pytest
import torch

from simlingo_amd import kernels as K

pytestmark = pytest.mark.gpu

SHAPES = [(128, 128, 64), (200, 136, 72), (1000, 520, 1032), (33, 8, 8), (16400 // 8, 3072 // 4, 1024)]


def _ref(a, b):
    return a.float() @ b.float()


@pytest.mark.parametrize("M,N,Kd", SHAPES)
@pytest.mark.parametrize("layout", [K.GEMM_NT, K.GEMM_NN, K.GEMM_TN, K.GEMM_TT])
@pytest.mark.parametrize("out_f32", [True, False])
def test_gemm_layouts(dev, M, N, Kd, layout, out_f32):
    a_contig = Kd if layout in (K.GEMM_NT, K.GEMM_NN) else M
    b_contig = Kd if layout in (K.GEMM_NT, K.GEMM_TT) else N
    if a_contig % 8 or b_contig % 8:
        with pytest.raises(RuntimeError, match="multiple of 8"):
            A = torch.zeros(8, 8, device=dev, dtype=torch.bfloat16)
            K.gemm(A, A, A, M, N, Kd, layout, 8, 8, 8)
        return
    g = torch.Generator(device=dev).manual_seed(M * 7 + N + Kd + layout)
    a = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    b = torch.randn(Kd, N, device=dev, generator=g).bfloat16()
    # materialise the storage each layout expects
    A = a if layout in (K.GEMM_NT, K.GEMM_NN) else a.t().contiguous()
    B = b.t().contiguous() if layout in (K.GEMM_NT, K.GEMM_TT) else b
    C = torch.empty(M, N, device=dev, dtype=torch.float32 if out_f32 else torch.bfloat16)
    K.gemm(A, B, C, M, N, Kd, layout, A.stride(0), B.stride(0), C.stride(0))
    ref = _ref(a, b)
    tol = 2e-3 * Kd ** 0.5 + (0 if out_f32 else 1e-2 * ref.abs().max().item())
    assert (C.float() - ref).abs().max().item() < tol


def test_gemm_epilogues(dev):
    M, N, Kd = 300, 256, 192
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = torch.randn(N, Kd, device=dev, generator=g).bfloat16() * 0.1
    bias = torch.randn(N, device=dev, generator=g)
    ref = x.float() @ w.float().t() + bias
    # bias + alpha + accumulate
    C = torch.ones(M, N, device=dev)
    K.linear(x, w, C, bias=bias, alpha=1.0, accumulate=True)
    torch.testing.assert_close(C, ref + 1, atol=2e-3, rtol=2e-3)
    # gelu with pre-activation aux
    h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.linear(x, w, y, bias=bias, epi=K.EPI_GELU, aux_out=h, ldaux_out=N)
    torch.testing.assert_close(h.float(), ref, atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(y.float(), torch.nn.functional.gelu(h.float()), atol=3e-2, rtol=1e-2)
    # residual + layer scale
    resid = torch.randn(M, N, device=dev, generator=g)
    ls = torch.rand(N, device=dev, generator=g)
    out = torch.empty(M, N, device=dev)
    yb = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.linear(x, w, out, bias=bias, epi=K.EPI_RESID_LS, resid=resid, ldr=N, ls=ls, aux_out=yb, ldaux_out=N)
    torch.testing.assert_close(out, resid + ls * ref, atol=3e-3, rtol=3e-3)
    # gelu backward
    dy = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w2 = torch.randn(Kd, N, device=dev, generator=g).bfloat16()  # "weight" [Nout=Kd][Kin=N]
    dh = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.dgrad(dy, w2, dh, epi=K.EPI_GELU_BWD, aux=h, ldaux=N)
    hh = h.float().requires_grad_()
    torch.nn.functional.gelu(hh).backward(dy.float() @ w2.float())
    torch.testing.assert_close(dh.float(), hh.grad, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("M,N,Kd,layout", [(896, 32, 6384, K.GEMM_TN), (32, 4864, 6384, K.GEMM_TN),
                                            (1024, 1024, 16400, K.GEMM_TN), (128, 96, 2048, K.GEMM_NT)])
@pytest.mark.parametrize("accumulate", [False, True])
def test_gemm_split_k(dev, M, N, Kd, layout, accumulate):
    """Under-filled f32 GEMMs take the split-K path (f32 atomics); compare with an fp32 reference."""
    g = torch.Generator(device=dev).manual_seed(M + N)
    a = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    b = torch.randn(Kd, N, device=dev, generator=g).bfloat16()
    A = a if layout in (K.GEMM_NT, K.GEMM_NN) else a.t().contiguous()
    B = b.t().contiguous() if layout in (K.GEMM_NT, K.GEMM_TT) else b
    C0 = torch.randn(M, N, device=dev, generator=g)
    C = C0.clone()
    bias = torch.randn(N, device=dev, generator=g)
    K.gemm(A, B, C, M, N, Kd, layout, A.stride(0), B.stride(0), C.stride(0), bias=bias, alpha=0.5,
           accumulate=accumulate)
    ref = 0.5 * (a.float() @ b.float()) + bias + (C0 if accumulate else 0)
    assert (C - ref).abs().max().item() < 2e-3 * Kd ** 0.5


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11])
@pytest.mark.parametrize("layout", [K.GEMM_NT, K.GEMM_NN, K.GEMM_TN, K.GEMM_TT])
def test_gemm_variants(dev, variant, layout):
    """Every main-loop variant (v1 register-staged, v2 LDS-DMA rings) on ragged M/N and K tails."""
    M, N, Kd = 304, 392, 640 if layout != K.GEMM_TN else 600
    g = torch.Generator(device=dev).manual_seed(variant * 10 + layout)
    a = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    b = torch.randn(Kd, N, device=dev, generator=g).bfloat16()
    A = a if layout in (K.GEMM_NT, K.GEMM_NN) else a.t().contiguous()
    B = b.t().contiguous() if layout in (K.GEMM_NT, K.GEMM_TT) else b
    for out_dtype in (torch.float32, torch.bfloat16):
        C = torch.empty(M, N, device=dev, dtype=out_dtype)
        K.gemm(A, B, C, M, N, Kd, layout, A.stride(0), B.stride(0), C.stride(0), variant=variant, ksplit_max=-1)
        ref = a.float() @ b.float()
        tol = 2e-3 * Kd ** 0.5 + (0 if out_dtype == torch.float32 else 1e-2 * ref.abs().max().item())
        assert (C.float() - ref).abs().max().item() < tol


@pytest.mark.parametrize("variant", [1, 2, 7, 8, 9, 10, 11])
def test_gemm_unaligned_output_and_all_epilogues(dev, variant):
    """Scalar epilogue fallback (C rows not 16-B aligned) and every epilogue through the DMA kernel."""
    M, N, Kd = 200, 128, 256
    g = torch.Generator(device=dev).manual_seed(7)
    x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, Kd, device=dev, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    ref = x.float() @ w.float().t() + bias
    big = torch.zeros(M, N + 5, device=dev)
    C = big[:, 3:3 + N]
    K.linear(x, w, C, bias=bias, variant=variant)
    torch.testing.assert_close(C, ref, atol=3e-3, rtol=3e-3)
    # SwiGLU backward epilogue: aux = [g | u] (width 2N)
    gu = torch.randn(M, 2 * N, device=dev, generator=g).bfloat16()
    dy = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    wd = (torch.randn(Kd, N, device=dev, generator=g) * 0.1).bfloat16()  # [Nout=Kd][Kin=N]
    dgu = torch.empty(M, 2 * N, device=dev, dtype=torch.bfloat16)
    K.gemm(dy, wd, dgu, M, N, Kd, K.GEMM_NN, Kd, N, 2 * N, epi=K.EPI_SWIGLU_BWD, aux=gu, ldaux=2 * N, variant=variant)
    gg, uu = gu.float()[:, :N].requires_grad_(), gu.float()[:, N:].requires_grad_()
    (torch.nn.functional.silu(gg) * uu).backward(dy.float() @ wd.float())
    torch.testing.assert_close(dgu[:, :N].float(), gg.grad, atol=5e-2, rtol=2e-2)
    torch.testing.assert_close(dgu[:, N:].float(), uu.grad, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("variant", [7, 8, 9, 10, 11])
@pytest.mark.parametrize("Kd", [64, 128, 192, 1024])
@pytest.mark.parametrize("layout", [K.GEMM_NT, K.GEMM_NN, K.GEMM_TN])
def test_gemm_v3_pipeline_depths(dev, Kd, layout, variant):
    """v3 (256x256 ping-pong) prologue/steady-state/drain paths: 1, 2, 3 and 16 K-tiles; multi-tile grid with
    ragged edges; split-K (f32 atomics) on the same kernel."""
    M, N = 600, 520
    g = torch.Generator(device=dev).manual_seed(Kd + layout)
    a = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    b = torch.randn(Kd, N, device=dev, generator=g).bfloat16()
    A = a if layout in (K.GEMM_NT, K.GEMM_NN) else a.t().contiguous()
    B = b.t().contiguous() if layout in (K.GEMM_NT, K.GEMM_TT) else b
    ref = a.float() @ b.float()
    for ks in (-1, 0):
        C = torch.full((M, N), 3.0, device=dev)
        K.gemm(A, B, C, M, N, Kd, layout, A.stride(0), B.stride(0), C.stride(0), variant=variant, ksplit_max=ks,
               accumulate=True)
        assert (C - 3.0 - ref).abs().max().item() < 2e-3 * Kd ** 0.5


@pytest.mark.parametrize("variant", [0, 7, 8, 9, 10, 11])
def test_gemm_v3_m_tail_peel_epilogues(dev, variant):
    """M = 2*256 + 16: v3 runs the first 512 rows and the 16-row remainder is peeled into a v2 launch with offset
    C/aux/aux_out/resid pointers (InternViT: 16400 = 64*256 + 16). Fused epilogues must agree across the seam."""
    M, N, Kd = 528, 512, 256
    g = torch.Generator(device=dev).manual_seed(21)
    x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, Kd, device=dev, generator=g) * 0.1).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    pre = x.float() @ w.float().t() + bias
    # GELU (bf16 out + pre-activation aux_out)
    h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    hpre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(x, w, h, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=K.EPI_GELU, bias=bias, aux_out=hpre, ldaux_out=N,
           variant=variant)
    torch.testing.assert_close(hpre.float(), pre, atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(h.float(), torch.nn.functional.gelu(hpre.float()), atol=3e-2, rtol=1e-2)
    # RESID_LS (f32 out = resid + ls * y)
    resid = torch.randn(M, N, device=dev, generator=g)
    ls = torch.rand(N, device=dev, generator=g)
    out = torch.empty(M, N, device=dev)
    K.gemm(x, w, out, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=K.EPI_RESID_LS, bias=bias, resid=resid, ldr=N, ls=ls,
           variant=variant)
    torch.testing.assert_close(out, resid + ls * pre, atol=3e-3, rtol=3e-3)
    # GELU_BWD (NN, bf16 out, aux = pre-activation)
    dy = torch.randn(M, N, device=dev, generator=g).bfloat16()
    dx = torch.empty(M, Kd, device=dev, dtype=torch.bfloat16)
    K.gemm(dy, w, dx, M, Kd, N, K.GEMM_NN, N, Kd, Kd, epi=K.EPI_GELU_BWD, aux=x, ldaux=Kd, variant=variant)
    xx = x.float().requires_grad_()
    torch.nn.functional.gelu(xx).backward(dy.float() @ w.float())
    torch.testing.assert_close(dx.float(), xx.grad, atol=5e-2, rtol=2e-2)


@pytest.mark.parametrize("variant", [7, 8, 9, 10, 11])
def test_gemm_v3_overlapped_last_tile(dev, variant):
    """Write-once epilogues run the partial last M tile of v3 shifted to end at M (rows shared with the previous
    tile are recomputed): the shared rows must be bit-identical to a launch without a remainder, the tail rows
    correct; an accumulating launch (C += ...) still takes the peel path and must not double-add."""
    M, N, Kd = 528, 512, 256
    g = torch.Generator(device=dev).manual_seed(33)
    x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, Kd, device=dev, generator=g) * 0.1).bfloat16()
    full = torch.empty(M, N, device=dev)
    K.gemm(x, w, full, M, N, Kd, K.GEMM_NT, Kd, Kd, N, variant=variant, ksplit_max=-1)
    head = torch.empty(512, N, device=dev)
    K.gemm(x, w, head, 512, N, Kd, K.GEMM_NT, Kd, Kd, N, variant=variant, ksplit_max=-1)
    torch.cuda.synchronize()
    assert torch.equal(full[:512], head)
    torch.testing.assert_close(full, x.float() @ w.float().t(), atol=2e-3, rtol=2e-3)
    acc = torch.ones(M, N, device=dev)
    K.gemm(x, w, acc, M, N, Kd, K.GEMM_NT, Kd, Kd, N, variant=variant, ksplit_max=-1, accumulate=True)
    torch.testing.assert_close(acc, 1.0 + x.float() @ w.float().t(), atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("p,use_bits,resid_bf16", [(0.0, False, False), (0.1, False, False), (0.1, True, False),
                                                   (0.1, True, True)])
def test_gemm_dropmask_swiglu_epilogue(dev, p, use_bits, resid_bf16):
    """EPI_DROPMASK_SWIGLU: dgu = SwiGLU'(gu) applied to (resid + keep * dT.A): the Qwen2 down-projection LoRA
    dropout dgrad fused into the SwiGLU backward (engine._lora_bwd, swiglu=...). resid_bf16: the base gradient as the
    bf16 dgrad output (slx_gemm_desc.resid_bf16), dT read from its trailing 64 columns as the engine does."""
    from simlingo_amd.dropmask import keep_scale
    M, F, seed = 300, 256, 4242
    g = torch.Generator(device=dev).manual_seed(3)
    dT = torch.randn(M, 64, device=dev, generator=g).bfloat16()
    A = (torch.randn(64, F, device=dev, generator=g) * 0.1).bfloat16()
    base = torch.randn(M, F + 64, device=dev, generator=g)
    if resid_bf16:
        base = base.bfloat16()
        base[:, F:] = dT
        dT = base[:, F:]
    gu = torch.randn(M, 2 * F, device=dev, generator=g).bfloat16()
    dgu = torch.empty(M, 2 * F, device=dev, dtype=torch.bfloat16)
    bits = None
    if use_bits:  # the keep bits slx_lora_down stores (host mirror), read instead of the hash
        from simlingo_amd.dropmask import keep_bits
        bits = torch.from_numpy(keep_bits(seed, M, F, F, p).view("int32")).to(dev)
    K.gemm(dT, A, dgu, M, F, 64, K.GEMM_NN, dT.stride(0), F, 2 * F, epi=K.EPI_DROPMASK_SWIGLU, resid=base,
           ldr=F + 64, aux=gu, ldaux=2 * F, seed=seed if not use_bits else seed + 1, drop_p=p, ldmask=F, maskbits=bits)
    mask = torch.from_numpy(keep_scale(seed, M, F, F, p)).to(dev) if p > 0 else 1.0
    d = base[:, :F].float() + mask * (dT.float() @ A.float())
    gg, uu = gu.float()[:, :F].requires_grad_(), gu.float()[:, F:].requires_grad_()
    (torch.nn.functional.silu(gg) * uu).backward(d)
    torch.testing.assert_close(dgu[:, :F].float(), gg.grad, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(dgu[:, F:].float(), uu.grad, atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("variant", [0, 8, 9, 10, 11])
@pytest.mark.parametrize("epi,M", [(K.EPI_GELU_BWD, 16400), (K.EPI_GELU_BWD, 1000), (K.EPI_QGELU_BWD, 2308),
                                   (K.EPI_STORE, 1000)])
def test_gemm_colsum_bias_grad(dev, epi, M, variant):
    """colsum: the epilogue adds the column sums of its f32 output into a [N] vector (fc1.b's gradient from the
    GELU_BWD dgrad). M = 16400 (remainder 16) and 2308 (remainder 4) fold their M % 256 rows into the main launch's
    last tiles; M = 1000 (remainder 232 > 64) runs them as a peeled 128-row-tile pass instead."""
    N, Kd = 512, 256
    g = torch.Generator(device=dev).manual_seed(M + epi)
    dy = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = torch.randn(Kd, N, device=dev, generator=g).bfloat16() * 0.1
    h = torch.randn(M, N, device=dev, generator=g).bfloat16()
    out = torch.empty(M, N, device=dev, dtype=torch.float32 if epi == K.EPI_STORE else torch.bfloat16)
    cs = torch.full((N,), 0.5, device=dev)
    K.mm(dy, w, out, tb=False, epi=epi, aux=h if epi != K.EPI_STORE else None, ldaux=N, colsum=cs, variant=variant)
    pre = dy.float() @ w.float()
    if epi == K.EPI_GELU_BWD:
        x = h.float()
        grad = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
        ref = pre * grad
    elif epi == K.EPI_QGELU_BWD:
        x = h.float()
        s = torch.sigmoid(1.702 * x)
        ref = pre * s * (1 + 1.702 * x * (1 - s))
    else:
        ref = pre
    torch.testing.assert_close(out.float(), ref, atol=3e-2 * Kd ** 0.5 / 16, rtol=2e-2)
    torch.testing.assert_close(cs, 0.5 + ref.sum(0), atol=2e-3 * M ** 0.5, rtol=1e-3)


@pytest.mark.parametrize("Kd", [192, 1024])
@pytest.mark.parametrize("M", [8192, 8192 + 16, 8192 + 240])
def test_gemm_fe_epilogues(dev, M, Kd):
    """Variant 11 (v3 with the register-direct epilogue, FE): 288 or more 256 x 256 tiles, so blocks 0-31 walk two
    tiles and the second one's first two K-steps are issued inside the first one's epilogue. Every FE epilogue
    against torch, the output against the LDS-staged variant 8 of the same main loop (<= 1 bf16 ulp), and the
    folded 16-row remainder (M = 8208) next to it."""
    N = 2304
    g = torch.Generator(device=dev).manual_seed(M + Kd)
    x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, Kd, device=dev, generator=g) * (2.0 / Kd ** 0.5)).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    pre = x.float() @ w.float().t() + bias
    outs = {}
    for v in (8, 11):
        h = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        hpre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(x, w, h, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=K.EPI_GELU, bias=bias, aux_out=hpre, ldaux_out=N, variant=v)
        plain = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(x, w, plain, M, N, Kd, K.GEMM_NT, Kd, Kd, N, bias=bias, variant=v)
        plain32 = torch.empty(M, N, device=dev)
        K.gemm(x, w, plain32, M, N, Kd, K.GEMM_NT, Kd, Kd, N, variant=v, ksplit_max=-1)
        resid = torch.randn(M, N, device=dev, generator=torch.Generator(device=dev).manual_seed(1))
        ls = torch.rand(N, device=dev, generator=torch.Generator(device=dev).manual_seed(2))
        out = torch.empty(M, N, device=dev)
        y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(x, w, out, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=K.EPI_RESID_LS, bias=bias, resid=resid, ldr=N, ls=ls,
               aux_out=y, ldaux_out=N, variant=v)
        dy = torch.randn(M, Kd, device=dev, generator=torch.Generator(device=dev).manual_seed(3)).bfloat16()
        dx = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        cs = torch.full((N,), 0.5, device=dev)
        wt = w.t().contiguous()  # [Kd][N]: NN
        K.gemm(dy, wt, dx, M, N, Kd, K.GEMM_NN, Kd, N, N, epi=K.EPI_GELU_BWD, aux=hpre, ldaux=N, colsum=cs, variant=v)
        dq = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        K.gemm(dy, wt, dq, M, N, Kd, K.GEMM_NN, Kd, N, N, epi=K.EPI_QGELU_BWD, aux=hpre, ldaux=N, variant=v)
        torch.cuda.synchronize()
        outs[v] = dict(h=h, hpre=hpre, plain=plain, plain32=plain32, out=out, y=y, dx=dx, cs=cs, dq=dq)
    o = outs[11]
    torch.testing.assert_close(o["hpre"].float(), pre, atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(o["h"].float(), torch.nn.functional.gelu(o["hpre"].float()), atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(o["plain"].float(), pre, atol=3e-2, rtol=1e-2)
    torch.testing.assert_close(o["plain32"], pre - bias, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(o["out"], resid + ls * pre, atol=3e-3, rtol=3e-3)
    torch.testing.assert_close(o["y"].float(), pre, atol=3e-2, rtol=1e-2)
    hx = o["hpre"].float()
    gd = 0.5 * (1 + torch.erf(hx / 2 ** 0.5)) + hx * torch.exp(-0.5 * hx * hx) / (2 * torch.pi) ** 0.5
    ref = (dy.float() @ w.float().t()) * gd
    torch.testing.assert_close(o["dx"].float(), ref, atol=3e-2, rtol=2e-2)
    torch.testing.assert_close(o["cs"], 0.5 + ref.sum(0), atol=2e-3 * M ** 0.5, rtol=1e-3)
    s = torch.sigmoid(1.702 * hx)
    torch.testing.assert_close(o["dq"].float(), (dy.float() @ w.float().t()) * s * (1 + 1.702 * hx * (1 - s)), atol=3e-2,
                               rtol=2e-2)
    for k in o:  # same main loop as variant 8: equal up to the epilogue's rounding (column sums: summation order)
        if k == "cs":
            continue
        a, b = o[k].float(), outs[8][k].float()
        tol = 1e-5 if o[k].dtype == torch.float32 else 8e-3
        assert ((a - b).abs() <= tol * (1 + b.abs())).all(), k


@pytest.mark.parametrize("M,variant", [(6384, 0), (6384, 2), (6384, 7), (600, 0), (8432, 0)])
def test_gemm_rope_epilogue(dev, M, variant):
    """RoPE fused into the bf16 STORE epilogue (slx_gemm_desc.rope_*): the Qwen2 q|k|v projection with bias, rotation
    on the q and k head slots (columns < 16 * 64), v untouched; position = row % S. Against torch (rotation of the f32
    product, one rounding) and no further from it than the separate GEMM + slx_rope (two roundings)."""
    from simlingo_amd import kernels as KK
    S, N, Kd = 798, 1152, 1024
    g = torch.Generator(device=dev).manual_seed(M + variant)
    x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, Kd, device=dev, generator=g) * 0.03).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    cos, sin = KK.rope_tables(S, 1e6, dev)
    fused = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(x, w, fused, M, N, Kd, K.GEMM_NT, Kd, Kd, N, bias=bias, rope=(cos, sin, S, 1024), variant=variant)
    sep = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    K.gemm(x, w, sep, M, N, Kd, K.GEMM_NT, Kd, Kd, N, bias=bias, variant=variant)
    K.rope(sep, M, S, 16, cos, sin)
    y = x.float() @ w.float().t() + bias
    pos = torch.arange(M, device=dev) % S
    c, s_ = cos[pos].repeat(1, 1), sin[pos]
    ref = y.clone()
    for h in range(16):
        a, b = y[:, 64 * h:64 * h + 32], y[:, 64 * h + 32:64 * h + 64]
        ref[:, 64 * h:64 * h + 32] = a * c - b * s_
        ref[:, 64 * h + 32:64 * h + 64] = b * c + a * s_
    torch.testing.assert_close(fused.float(), ref, atol=2e-2, rtol=1e-2)
    assert torch.equal(fused[:, 1024:], sep[:, 1024:])  # v columns: plain epilogue
    # one rounding instead of two: never further from the f32 rotation than the separate pass
    ef, es = (fused.float() - ref).abs().max().item(), (sep.float() - ref).abs().max().item()
    assert ef <= es + 1e-6, (ef, es)


_FOLD_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from simlingo_amd import kernels as K
dev = torch.device("cuda")
g = torch.Generator(device=dev).manual_seed(5)
for M in (1088, 16400):
    dy = torch.randn(M, 256, device=dev, generator=g).bfloat16()
    w = torch.randn(256, 512, device=dev, generator=g).bfloat16() * 0.1
    h = torch.randn(M, 512, device=dev, generator=g).bfloat16()
    out = torch.empty(M, 512, device=dev, dtype=torch.bfloat16)
    cs = torch.full((512,), 0.5, device=dev)
    K.mm(dy, w, out, tb=False, epi=K.EPI_GELU_BWD, aux=h, ldaux=512, colsum=cs, variant=7)
    acc = torch.full((M, 512), 0.25, device=dev)
    K.mm(dy, w, acc, tb=False, accumulate=True, variant=7)
    torch.cuda.synchronize()
    torch.save({"out": out.float().cpu(), "cs": cs.cpu(), "acc": acc.cpu()}, sys.argv[2] + f"_{M}.pt")
"""


@pytest.mark.parametrize("fold", ["1", "0"])
def test_gemm_fold_remainder_accumulate_and_unfolded_path(dev, fold, tmp_path):
    """The folded M-remainder (M % 256 <= 64 rows summed into the main launch's last tiles through the arrival
    hand-off) with a 64-row remainder (M = 1088) and with 16 rows (16400), in the GELU'+colsum epilogue and in an
    accumulating f32 store; SLX_GEMM_FOLD_REM=0 runs the same remainder as its own split-K + rows-epilogue launches
    (gemm_remainder + rows_epilogue with colsum). The env var is read once per process, so each form runs in a child
    process (the GPU work is a few ms)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SLX_GEMM_FOLD_REM=fold)
    subprocess.run([sys.executable, "-c", _FOLD_SCRIPT, root, str(tmp_path / "r")], env=env, check=True, timeout=240)
    g = torch.Generator(device=dev).manual_seed(5)
    for M in (1088, 16400):
        dy = torch.randn(M, 256, device=dev, generator=g).bfloat16()
        w = torch.randn(256, 512, device=dev, generator=g).bfloat16() * 0.1
        h = torch.randn(M, 512, device=dev, generator=g).bfloat16()
        r = torch.load(tmp_path / f"r_{M}.pt", weights_only=True)
        pre = dy.float() @ w.float()
        x = h.float()
        ref = pre * (0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5)
        torch.testing.assert_close(r["out"].to(dev), ref, atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(r["cs"].to(dev), 0.5 + ref.sum(0), atol=2e-3 * M ** 0.5, rtol=1e-3)
        torch.testing.assert_close(r["acc"].to(dev), 0.25 + pre, atol=2e-3, rtol=1e-3)


def test_batched_splitk_accumulate_tn(dev):
    """Batched TN weight-gradient GEMM with split-K f32 atomics accumulating into C (the LoRA dB pairs k|v and
    gate|up: A = adjacent column blocks of dy, B = adjacent 32-column blocks of t, C = B-gradient slices sC apart)."""
    g = torch.Generator(device=dev).manual_seed(21)
    M, out, r = 3000, 640, 32
    dy = torch.randn(M, 2 * out + 16, device=dev, generator=g).bfloat16()
    t = torch.randn(M, 2 * r + 64, device=dev, generator=g).bfloat16()
    flat = torch.zeros(3 * out * r + 4096, device=dev)
    sC = out * r + 1024
    C0, C1 = flat[:out * r].view(out, r), flat[sC:sC + out * r].view(out, r)
    C0.fill_(0.5)
    C1.fill_(-0.25)
    K.gemm(dy, t, C0, out, r, M, K.GEMM_TN, dy.stride(0), t.stride(0), r, alpha=2.0, accumulate=True, batch=2,
           sA=out, sB=r, sC=sC)
    torch.cuda.synchronize()
    want0 = 0.5 + 2.0 * dy[:, :out].float().t() @ t[:, :r].float()
    want1 = -0.25 + 2.0 * dy[:, out:2 * out].float().t() @ t[:, r:2 * r].float()
    torch.testing.assert_close(C0, want0, atol=2e-2, rtol=1e-3)
    torch.testing.assert_close(C1, want1, atol=2e-2, rtol=1e-3)
    assert torch.all(flat[out * r:sC] == 0) and torch.all(flat[sC + out * r:] == 0)  # nothing written between


@pytest.mark.parametrize("variant", [7, 8])
@pytest.mark.parametrize("shapes,split", [(((1024, 512), (512, 1024)), 0), (((768, 256), (256, 264)), 3),
                                          (((136, 64), (256, 200)), 1)])
def test_gemm_pair_wgrad(dev, shapes, split, variant):
    """slx_gemm_bf16_pair: two accumulating TN weight-gradient GEMMs (dW_i += dY_i^T X_i) in one launch, each vs
    torch fp32 on the same bf16 operands (M-remainder tiles, split-K on and off)."""
    T = 1040
    g = torch.Generator(device=dev).manual_seed(sum(sum(s) for s in shapes) + split)
    ops, refs = [], []
    for (N, Kd) in shapes:
        dy = torch.randn(T, N, device=dev, generator=g).bfloat16()
        x = torch.randn(T, Kd, device=dev, generator=g).bfloat16()
        C = torch.randn(N, Kd, device=dev, generator=g)
        refs.append(C + dy.float().t() @ x.float())
        ops.append((dy, x, C))
    K.mm_pair(ops[0], ops[1], ksplit_max=split, variant=variant)
    for (_, _, C), ref in zip(ops, refs):
        assert (C - ref).abs().max().item() < 2e-3 * T ** 0.5
    with pytest.raises(RuntimeError, match="one layout and one K"):
        K.mm_pair(ops[0], (ops[1][0][:512], ops[1][1][:512], ops[1][2]))


@pytest.mark.parametrize("variant", [7, 8])
@pytest.mark.parametrize("split", [2])
def test_gemm_splitk_in_launch_reduction(dev, split, variant):
    """Split-K f32 weight-gradient GEMMs on the 256x256 kernel reduce their partials inside the launch (the last
    arriving split of each tile sums the others' slabs in split order): bitwise identical across calls whatever the
    arrival order, equal to the f32-atomics path within rounding, counters left zero (repeated calls agree), and
    the same through slx_gemm_bf16_pair."""
    T, M, N = 4096, 768, 520
    g = torch.Generator(device=dev).manual_seed(split * 7 + variant)
    dy = torch.randn(T, M, device=dev, generator=g).bfloat16()
    x = torch.randn(T, N, device=dev, generator=g).bfloat16()
    c0 = torch.randn(M, N, device=dev, generator=g)
    ref = c0 + dy.float().t() @ x.float()
    outs = []
    for _ in range(3):
        C = c0.clone()
        K.gemm(dy, x, C, M, N, T, K.GEMM_TN, M, N, N, accumulate=True, ksplit_max=split, variant=variant)
        outs.append(C)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    assert (outs[0] - ref).abs().max().item() < 2e-3 * T ** 0.5
    Ca = c0.clone()
    K.gemm(dy, x, Ca, M, N, T, K.GEMM_TN, M, N, N, accumulate=True, ksplit_max=split, variant=variant, split_ws=False)
    torch.testing.assert_close(outs[0], Ca, atol=1e-3 * T ** 0.5, rtol=1e-5)
    # non-accumulating: C is written, not added to (no pre-zeroing needed on the reduction path)
    Cz = torch.full((M, N), float("nan"), device=dev)
    K.gemm(dy, x, Cz, M, N, T, K.GEMM_TN, M, N, N, ksplit_max=split, variant=variant)
    torch.testing.assert_close(Cz, ref - c0, atol=2e-3 * T ** 0.5, rtol=1e-4)
    # pair launch
    dy2 = torch.randn(T, 256, device=dev, generator=g).bfloat16()
    x2 = torch.randn(T, 1024, device=dev, generator=g).bfloat16()
    p1, p2 = [], []
    for _ in range(2):
        C1, C2 = c0.clone(), torch.zeros(256, 1024, device=dev)
        K.mm_pair((dy, x, C1), (dy2, x2, C2), ksplit_max=split, variant=variant)
        p1.append(C1)
        p2.append(C2)
    torch.cuda.synchronize()
    assert torch.equal(p1[0], p1[1]) and torch.equal(p2[0], p2[1])
    assert (p1[0] - ref).abs().max().item() < 2e-3 * T ** 0.5
    assert (p2[0] - dy2.float().t() @ x2.float()).abs().max().item() < 2e-3 * T ** 0.5


@pytest.mark.parametrize("shapes", [((1024, 4096), (4096, 1024)),   # InternViT fc2.w + fc1.w: 128 tiles x 2 splits
                                    ((3072, 1024), (1024, 1024))])  # qkv.w + proj.w: 64 tiles x 4 splits
def test_gemm_pair_xcd_split_full_shape(dev, shapes):
    """The InternViT weight-gradient pairs at their real shapes (K = 16 x 1025 tokens): tiles x splits = 256, so the
    pair launches as one 1-D round with XCD x taking K split x % S of a contiguous tile range (SLX_PAIR_XCD_SPLIT);
    each gradient vs torch fp32 on the same bf16 operands, accumulating into a nonzero C, twice (counters reset)."""
    T = 16400
    g = torch.Generator(device=dev).manual_seed(sum(a * b for a, b in shapes))
    ops, refs = [], []
    for (N, Kd) in shapes:
        dy = torch.randn(T, N, device=dev, generator=g).bfloat16()
        x = torch.randn(T, Kd, device=dev, generator=g).bfloat16()
        C = torch.randn(N, Kd, device=dev, generator=g)
        refs.append(C + 2 * (dy.float().t() @ x.float()))
        ops.append((dy, x, C))
    for _ in range(2):
        K.mm_pair(ops[0], ops[1])
    torch.cuda.synchronize()
    for (_, _, C), ref in zip(ops, refs):
        err = (C - ref).abs().max().item()
        assert err < 4e-3 * T ** 0.5, err


@pytest.mark.parametrize("M,v", [(8208, 11), (8208, 8), (1000, 0), (77, 1)])
def test_gelu_aux_grad(dev, M, v):
    """aux_grad: the GELU / QGELU forward epilogue stores bf16(act'(h)) at the bf16-rounded pre-activation h as its aux
    (output unchanged), and the GELU_BWD / QGELU_BWD epilogue multiplies that aux in directly: against torch on the
    same bf16 h, for the FE (11), LDS-staged v3 (8), automatic and scalar (1) epilogues."""
    N, Kd = 2304, 512
    g = torch.Generator(device=dev).manual_seed(M + v)
    x = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    w = (torch.randn(N, Kd, device=dev, generator=g) * (2.0 / Kd ** 0.5)).bfloat16()
    bias = torch.randn(N, device=dev, generator=g)
    wt = w.t().contiguous()
    dy = torch.randn(M, Kd, device=dev, generator=g).bfloat16()
    for epi, bepi in ((K.EPI_GELU, K.EPI_GELU_BWD), (K.EPI_QGELU, K.EPI_QGELU_BWD)):
        h0, hpre = (torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2))
        K.gemm(x, w, h0, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=epi, bias=bias, aux_out=hpre, ldaux_out=N, variant=v)
        h1, gpre = (torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2))
        K.gemm(x, w, h1, M, N, Kd, K.GEMM_NT, Kd, Kd, N, epi=epi, bias=bias, aux_out=gpre, ldaux_out=N, variant=v,
               aux_grad=True)
        torch.cuda.synchronize()
        assert torch.equal(h0, h1)  # the activation output does not change
        hp = hpre.float().requires_grad_(True)
        act = torch.nn.functional.gelu(hp) if epi == K.EPI_GELU else hp * torch.sigmoid(1.702 * hp)
        (ref_g,) = torch.autograd.grad(act.sum(), hp)
        torch.testing.assert_close(gpre.float(), ref_g, atol=2e-3, rtol=8e-3)
        d0, d1 = (torch.empty(M, N, device=dev, dtype=torch.bfloat16) for _ in range(2))
        K.gemm(dy, wt, d0, M, N, Kd, K.GEMM_NN, Kd, N, N, epi=bepi, aux=hpre, ldaux=N, variant=v)
        K.gemm(dy, wt, d1, M, N, Kd, K.GEMM_NN, Kd, N, N, epi=bepi, aux=gpre, ldaux=N, variant=v, aux_grad=True)
        torch.cuda.synchronize()
        dv = dy.float() @ wt.float()
        torch.testing.assert_close(d1.float(), dv * gpre.float(), atol=3e-2, rtol=2e-2)
        # against the h-aux path: the only difference is the bf16 rounding of act'(h)
        torch.testing.assert_close(d1.float(), d0.float(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,N,Kd,f32,beta", [(6384, 960, 9728, True, 0.0), (6384, 896, 4928, True, 1.0),
                                             (6384, 896, 960, True, 1.0), (777, 200, 136, False, 0.0),
                                             (130, 64, 64, True, 1.0)])
def test_gemm_lt_vs_torch(dev, M, N, Kd, f32, beta):
    """slx_gemm_lt (hipBLASLt) on the step's plain Qwen2 shapes (gate/up data gradient; o / down projections with the
    f32 residual as C, beta = 1) and ragged ones, on strided row views, against a float64 reference."""
    gen = torch.Generator(device=dev).manual_seed(M + N)
    Ab = torch.randn(M, Kd + 8, device=dev, generator=gen).bfloat16()
    Bb = torch.randn(N, Kd + 16, device=dev, generator=gen).bfloat16()
    A, B = Ab[:, :Kd], Bb[:, :Kd]
    dt = torch.float32 if f32 else torch.bfloat16
    Dfull = torch.full((M, N + 24), 7.0, device=dev, dtype=dt)
    D = Dfull[:, :N]
    C = torch.randn(M, N, device=dev, generator=gen).to(dt) if beta else None
    K.mm_lt(A, B, D, C=C, beta=beta)
    torch.cuda.synchronize()
    ref = A.double() @ B.double().t() + (beta * C.double() if beta else 0)
    tol = 2e-5 * Kd ** 0.5 * 4 if f32 else 2e-2
    err = ((D.double() - ref).abs().max() / ref.abs().max()).item()
    assert err < tol, err
    assert torch.all(Dfull[:, N:] == 7.0)  # nothing written past N


def test_gemm_lt_in_place_residual(dev):
    """C == D (the residual updated in place) and a second call with the same shape reusing the cached plan."""
    gen = torch.Generator(device=dev).manual_seed(3)
    A = torch.randn(640, 256, device=dev, generator=gen).bfloat16()
    B = torch.randn(128, 256, device=dev, generator=gen).bfloat16()
    X = torch.randn(640, 128, device=dev, generator=gen)
    ref = X.double() + A.double() @ B.double().t()
    K.mm_lt(A, B, X, C=X, beta=1.0)
    torch.cuda.synchronize()
    assert ((X.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5
    Y = torch.zeros(640, 128, device=dev)
    K.mm_lt(A, B, Y, C=Y, beta=1.0)
    torch.cuda.synchronize()
    assert ((Y.double() - A.double() @ B.double().t()).abs().max()).item() < 1e-2
