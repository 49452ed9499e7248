"""LoRA dropout: the hash mask applied while loading A (down-projection), while loading B (dA GEMM) and
in the DROPMASK epilogue (dx) is one function of (seed, row*ldmask + col); checked against a PyTorch
fp32 reference that applies the host mirror of the mask (simlingo_amd/dropmask.py)."""
import numpy as np
import pytest
import torch

from simlingo_amd import kernels as K
from simlingo_amd.dropmask import keep_scale

pytestmark = pytest.mark.gpu


def test_dropout_mask_consistency(dev):
    M, kin, r, p, seed = 300, 256, 32, 0.1, 987654321
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(M, kin, device=dev, generator=g).bfloat16()
    A = (torch.randn(r, kin, device=dev, generator=g) * 0.1).bfloat16()
    mask = torch.from_numpy(keep_scale(seed, M, kin, kin, p)).to(dev)
    assert 0.85 < (mask > 0).float().mean().item() < 0.95
    xd = (x.float() * mask).bfloat16().float()  # the kernels round the scaled, masked input to bf16
    # forward: t = drop(x) A^T  (mask on the A operand)
    t = torch.empty(M, r, device=dev, dtype=torch.float32)
    K.mm(x, A, t, drop_operand=1, seed=seed, drop_p=p, ldmask=kin)
    torch.testing.assert_close(t, xd @ A.float().t(), atol=2e-2, rtol=2e-2)
    # dA = dt^T drop(x)  (mask on the B operand, TN layout)
    dt = torch.randn(M, r, device=dev, generator=g).bfloat16()
    dA = torch.zeros(r, kin, device=dev)
    K.mm(dt, x, dA, ta=True, tb=False, drop_operand=2, seed=seed, drop_p=p, ldmask=kin, accumulate=True)
    torch.testing.assert_close(dA, dt.float().t() @ xd, atol=2e-2, rtol=1e-2)
    # dx += mask * (dt A)  (epilogue)
    dx = torch.ones(M, kin, device=dev)
    K.mm(dt, A, dx, tb=False, epi=K.EPI_DROPMASK, accumulate=True, seed=seed, drop_p=p, ldmask=kin)
    torch.testing.assert_close(dx, 1 + mask * (dt.float() @ A.float()), atol=2e-2, rtol=2e-2)
    # standalone dropout kernel agrees too
    y = torch.empty_like(x)
    K.call("slx_dropout", K.P(x), kin, K.P(y), kin, M, kin, seed, p, kin, K.stream_ptr())
    torch.testing.assert_close(y.float(), (x.float() * mask).bfloat16().float())


@pytest.mark.parametrize("M,kin,nsites,p", [(300, 256, 3, 0.1), (6384 // 8 + 5, 896, 2, 0.1), (77, 1280, 1, 0.0),
                                            (1, 128, 4, 0.1), (6384, 4864, 1, 0.1)])
def test_lora_down_grouped(dev, M, kin, nsites, p):
    """slx_dropout_bits writes the keep masks as bits (bit c&31 of word c>>5) exactly as the host mirror computes
    them; slx_lora_down: t[:, 32j:32j+32] = drop_j(x) A_j^T from those bits, one launch for the sites sharing x."""
    from simlingo_amd.dropmask import keep_bits
    g = torch.Generator(device=dev).manual_seed(11)
    xfull = torch.randn(M, kin + 64, device=dev, generator=g).bfloat16()
    x = xfull[:, :kin]  # strided view: ldx != kin, ldmask = kin
    As = [(torch.randn(32, kin, device=dev, generator=g) * 0.1).bfloat16() for _ in range(nsites)]
    seeds = [1234567 + 7919 * j for j in range(nsites)]
    t = torch.full((M, 32 * nsites + 16), 7.0, device=dev).bfloat16()
    bits = [torch.zeros(M, kin // 32, device=dev, dtype=torch.int32) for _ in range(nsites)]
    if p > 0:
        K.dropout_bits([(seeds[j], bits[j], kin, kin) for j in range(nsites)], M, p)
    K.lora_down(x, As, t, seeds, p=p, bits=bits if p > 0 else None)
    for j in range(nsites):
        mask = torch.from_numpy(keep_scale(seeds[j], M, kin, kin, p)).to(dev) if p > 0 else 1.0
        xd = (x.float() * mask).bfloat16().float()
        torch.testing.assert_close(t[:, 32 * j:32 * (j + 1)].float(), xd @ As[j].float().t(), atol=3e-2, rtol=2e-2)
        if p > 0:
            want = torch.from_numpy(keep_bits(seeds[j], M, kin, kin, p).view("int32")).to(dev)
            assert torch.equal(bits[j], want), j
    assert (t[:, 32 * nsites:].float() == 7.0).all()  # columns past the sites untouched


def test_dropmask_dgrad_padded_k64(dev):
    """dx += mask * (dT_j A_j) as a K=64 GEMM: the A operand is a 64-column window of the group's dT buffer and
    B is A_j zero-padded to 64 rows (engine._lora_bwd), so the columns past site j contribute exactly 0."""
    M, kin, p, seed = 500, 896, 0.1, 424242
    g = torch.Generator(device=dev).manual_seed(5)
    dT = torch.randn(M, 96, device=dev, generator=g).bfloat16()
    A = (torch.randn(32, kin, device=dev, generator=g) * 0.1).bfloat16()
    Ap = torch.zeros(64, kin, device=dev, dtype=torch.bfloat16)
    Ap[:32] = A
    mask = torch.from_numpy(keep_scale(seed, M, kin, kin, p)).to(dev)
    for j in (0, 1):
        dx = torch.ones(M, kin, device=dev)
        K.mm(dT[:, 32 * j:32 * j + 64], Ap, dx, tb=False, epi=K.EPI_DROPMASK, accumulate=True, seed=seed, drop_p=p,
             ldmask=kin)
        ref = 1 + mask * (dT[:, 32 * j:32 * (j + 1)].float() @ A.float())
        torch.testing.assert_close(dx, ref, atol=2e-2, rtol=2e-2)


@pytest.mark.parametrize("M,kin,nsites,p,mode", [(300, 256, 3, 0.1, "f32"), (1000, 896, 2, 0.1, "f32"),
                                                 (130, 640, 1, 0.0, "f32"), (64, 128, 4, 0.1, "bf16"),
                                                 (6384, 896, 3, 0.1, "f32"), (6384, 896, 1, 0.1, "bf16"),
                                                 (6384, 4864, 1, 0.1, "none"), (798, 128, 3, 0.0, "f32"),
                                                 (798, 896, 2, 0.0, "bf16")])
@pytest.mark.parametrize("dt_bf16", [False, True])
@pytest.mark.parametrize("slab", [False, True])
def test_lora_bwd_grouped(dev, M, kin, nsites, p, mode, dt_bf16, slab, monkeypatch):
    """slx_lora_bwd: dA_j += dT_j^T drop_j(x) and dx += sum_j drop_j'(dT_j A_j) (f32 in place / bf16 out / none),
    masks read from the keep bits of slx_lora_down, dT read as f32 from a strided view (the dgrad GEMM's extra
    columns). slab: dA through slx_lora_bwd_ws's per-row-chunk partials and in-order sum instead of f32 atomics."""
    from simlingo_amd.dropmask import keep_bits
    monkeypatch.setattr(K, "LORA_DA_SLAB", slab)
    g = torch.Generator(device=dev).manual_seed(13)
    x = torch.randn(M, kin, device=dev, generator=g).bfloat16()
    dtfull = torch.randn(M, 32 * nsites + 64, device=dev, generator=g)
    if dt_bf16:  # slx_lora_bwd_desc.dt_bf16: dT as the bf16 dgrad output columns (16-B aligned rows)
        dtfull = dtfull.bfloat16()
    dt = dtfull[:, 16:16 + 32 * nsites]
    As = [(torch.randn(32, kin, device=dev, generator=g) * 0.1).bfloat16() for _ in range(nsites)]
    seeds = [777 + 31 * j for j in range(nsites)]
    bits = [torch.from_numpy(keep_bits(sd, M, kin, kin, p).view("int32")).to(dev) if p > 0 else None for sd in seeds]
    dAs = [torch.full((32, kin), 0.5, device=dev) for _ in range(nsites)]
    dx0 = torch.randn(M, kin, device=dev, generator=g)
    dx = dx0.clone()
    dxb = torch.empty(M, kin, device=dev, dtype=torch.bfloat16) if mode == "bf16" else None
    # the dx kernel's bf16 dT side output (slx_lora_grad's operand), a strided view as the engine passes it
    dto = torch.full((M, 32 * nsites + 16), -7.0, device=dev, dtype=torch.bfloat16) if mode != "none" else None
    K.lora_bwd(x, dt, As, bits, dAs, dx=None if mode == "none" else dx, dx_bf16=dxb, p=p,
               dt_out=None if dto is None else dto[:, 8:8 + 32 * nsites])
    dtb = dt.bfloat16().float()
    ref_dx = dx0.clone()
    for j in range(nsites):
        mask = torch.from_numpy(keep_scale(seeds[j], M, kin, kin, p)).to(dev) if p > 0 else 1.0
        xd = (x.float() * mask).bfloat16().float()
        torch.testing.assert_close(dAs[j], 0.5 + dtb[:, 32 * j:32 * (j + 1)].t() @ xd, atol=5e-2 * (M / 300) ** 0.5,
                                   rtol=1e-2)
        ref_dx += mask * (dtb[:, 32 * j:32 * (j + 1)] @ As[j].float())
    if dto is not None:  # every row (M % 32 != 0 too) and column tile of both column groups, exact
        assert torch.equal(dto[:, 8:8 + 32 * nsites], dt.bfloat16())
        assert bool((dto[:, :8] == -7.0).all()) and bool((dto[:, 8 + 32 * nsites:] == -7.0).all())
    lora_term = (ref_dx - dx0).abs().max().item()
    if mode == "f32":  # the kernel sums the same bf16 operands in f32: relative to the LoRA term, ~1e-7
        assert (dx - ref_dx).abs().max().item() <= 1e-5 * lora_term
    elif mode == "bf16":
        torch.testing.assert_close(dxb.float(), ref_dx, atol=3e-2, rtol=2e-2)
        assert (dxb.float() - ref_dx).abs().max().item() <= 1e-5 * lora_term + (ref_dx.abs().max().item() / 128)
        assert torch.equal(dx, dx0)  # the f32 base gradient is only read
    else:
        assert torch.equal(dx, dx0)


@pytest.mark.parametrize("M,kin,nsites", [(6384, 896, 3), (16400, 1024, 1)])
def test_lora_da_slab_deterministic(dev, M, kin, nsites, monkeypatch):
    """SLX_LORA_DA_SLAB: the slab-reduced dA is bit-identical run to run (fixed chunking and summation order) and
    agrees with the atomics path to f32 summation-order rounding."""
    monkeypatch.setattr(K, "LORA_DA_SLAB", True)
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(M, kin, device=dev, generator=g).bfloat16()
    dt = torch.randn(M, 32 * nsites, device=dev, generator=g)
    As = [(torch.randn(32, kin, device=dev, generator=g) * 0.1).bfloat16() for _ in range(nsites)]
    outs = []
    for _ in range(2):
        dAs = [torch.zeros(32, kin, device=dev) for _ in range(nsites)]
        K.lora_bwd(x, dt, As, [None] * nsites, dAs)
        outs.append(dAs)
    monkeypatch.setattr(K, "LORA_DA_SLAB", False)
    dAt = [torch.zeros(32, kin, device=dev) for _ in range(nsites)]
    K.lora_bwd(x, dt, As, [None] * nsites, dAt)
    for a, b, c in zip(*outs, dAt):
        assert torch.equal(a, b)
        assert ((a - c).norm() / c.norm()).item() < 1e-5


@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("M,p", [(6384, 0.1), (1000, 0.0), (77, 0.1)])
def test_lora_grad_jobs(dev, M, p, det):
    """slx_lora_grad: a B-gradient job (out [n][32] += s dy^T t) and an A-gradient job of 3 sites sharing x with keep
    bits (out_j [32][n] += dT_j^T bf16(x/(1-p)) & keep_j), against torch fp32 on the same bf16 operands.
    det: the deterministic-reduction mode (per-row-chunk partials + ordered sum instead of f32 atomics) - the same
    values, and two launches bitwise equal."""
    from simlingo_amd.dropmask import keep_bits
    g = torch.Generator(device=dev).manual_seed(21)
    s = 2.0
    dy = torch.randn(M, 4864, device=dev, generator=g).bfloat16()
    t = torch.randn(M, 96, device=dev, generator=g).bfloat16()
    x = torch.randn(M, 896, device=dev, generator=g).bfloat16()
    dT = torch.randn(M, 96, device=dev, generator=g).bfloat16()
    seeds = [5, 6, 7]
    bits = [torch.from_numpy(keep_bits(sd, M, 896, 896, p).view("int32")).to(dev) for sd in seeds] if p > 0 else None
    dB = torch.full((4864, 32), 0.25, device=dev)
    dA = [torch.full((32, 896), -0.5, device=dev) for _ in range(3)]
    jobs = [dict(x=dy, t=t[:, 32:64], outs=[dB], out_nr=True, alpha=s),
            dict(x=x, t=dT, outs=dA, out_nr=False, alpha=1.0, p=p, bits=bits)]
    if det:
        K.set_deterministic(True, dev)
    try:
        K.lora_grad(jobs, M)
        if det:
            dB2 = torch.full((4864, 32), 0.25, device=dev)
            dA2 = [torch.full((32, 896), -0.5, device=dev) for _ in range(3)]
            K.lora_grad([dict(jobs[0], outs=[dB2]), dict(jobs[1], outs=dA2)], M)
        torch.cuda.synchronize()
    finally:
        K.set_deterministic(False)
    if det:
        assert torch.equal(dB, dB2) and all(torch.equal(a, b) for a, b in zip(dA, dA2))
    refB = 0.25 + s * dy.float().t() @ t[:, 32:64].float()
    torch.testing.assert_close(dB, refB, atol=2e-3 * refB.abs().max().item(), rtol=1e-4)
    for j in range(3):
        mask = torch.from_numpy(keep_scale(seeds[j], M, 896, 896, p)).to(dev) if p > 0 else 1.0
        xd = (x.float() * mask).bfloat16().float()
        refA = -0.5 + dT[:, 32 * j:32 * (j + 1)].float().t() @ xd
        torch.testing.assert_close(dA[j], refA, atol=2e-3 * refA.abs().max().item(), rtol=1e-4)


@pytest.mark.parametrize("M,F,p", [(6384, 4864, 0.1), (77, 256, 0.1), (300, 512, 0.0)])
def test_lora_swiglu_bwd(dev, M, F, p):
    """slx_lora_swiglu_bwd (the down site's LoRA dgrad fused with the SwiGLU backward) against torch fp32 on the same
    bf16 operands and against the K = 64 GEMM form it replaces (DROPMASK_SWIGLU epilogue over the zero-padded A):
    both round the same f32 values to bf16, so they agree to one bf16 ulp."""
    from simlingo_amd.dropmask import keep_bits
    import torch.nn.functional as Fn
    g = torch.Generator(device=dev).manual_seed(31)
    dtfull = (torch.randn(M, 64, device=dev, generator=g) * 0.5).bfloat16()
    dtfull[:, 32:] = 0  # the W_cat padding columns are exactly zero
    A = (torch.randn(32, F, device=dev, generator=g) * 0.1).bfloat16()
    resid = torch.randn(M, F, device=dev, generator=g).bfloat16()
    gu = torch.randn(M, 2 * F, device=dev, generator=g).bfloat16()
    bits = torch.from_numpy(keep_bits(99, M, F, F, p).view("int32")).to(dev) if p > 0 else None
    dgu = torch.empty(M, 2 * F, device=dev, dtype=torch.bfloat16)
    K.lora_swiglu_bwd(dtfull, A.t().contiguous(), resid, gu, dgu, bits, p)
    mask = torch.from_numpy(keep_scale(99, M, F, F, p)).to(dev) if p > 0 else 1.0
    d = resid.float() + mask * (dtfull[:, :32].float() @ A.float())
    gg, uu = gu[:, :F].float(), gu[:, F:].float()
    sg = torch.sigmoid(gg)
    ref = torch.cat([d * uu * sg * (1 + gg * (1 - sg)), d * Fn.silu(gg)], 1)
    torch.testing.assert_close(dgu.float(), ref, atol=1e-2, rtol=1e-2)
    # the GEMM form it replaces
    apad = torch.zeros(64, F, device=dev, dtype=torch.bfloat16)
    apad[:32] = A
    dg2 = torch.empty_like(dgu)
    K.gemm(dtfull, apad, dg2, M, F, 64, K.GEMM_NN, 64, F, 2 * F, epi=K.EPI_DROPMASK_SWIGLU, resid=resid, ldr=F,
           aux=gu, ldaux=2 * F, seed=0, drop_p=p, ldmask=F, maskbits=bits)
    diff = (dgu.float() - dg2.float()).abs()
    assert (diff <= dg2.float().abs() * 2 ** -7 + 1e-6).all(), diff.max().item()


@pytest.mark.parametrize("M,F,p", [(6384, 4864, 0.1), (77, 256, 0.1), (300, 512, 0.0), (130, 384, 0.1)])
def test_lora_swiglu_bwd_grads(dev, M, F, p):
    """slx_lora_swiglu_bwd_grads: dgu bitwise equal to slx_lora_swiglu_bwd's; dA_down = dT^T drop(act) with act the
    forward's activation (slx_swiglu_fwd, bit-exact) and dB_gate / dB_up = s dgu^T t against float64 products of the same
    bf16 operands, accumulated onto non-zero gradients; two calls give bitwise-equal results (ordered partial sums)."""
    from simlingo_amd.dropmask import keep_bits
    g = torch.Generator(device=dev).manual_seed(53)
    dtfull = (torch.randn(M, 64, device=dev, generator=g) * 0.5).bfloat16()
    dtfull[:, 32:] = 0
    A = (torch.randn(32, F, device=dev, generator=g) * 0.1).bfloat16()
    AT = A.t().contiguous()
    resid = torch.randn(M, F, device=dev, generator=g).bfloat16()
    gu = torch.randn(M, 2 * F, device=dev, generator=g).bfloat16()
    tx = (torch.randn(M, 80, device=dev, generator=g) * 0.3).bfloat16()  # t_gate | t_up at columns 8.., 40..
    tg, tu = tx[:, 8:40], tx[:, 40:72]
    bits = torch.from_numpy(keep_bits(77, M, F, F, p).view("int32")).to(dev) if p > 0 else None
    s = 2.0
    outs = []
    for _ in range(2):
        dgu = torch.empty(M, 2 * F, device=dev, dtype=torch.bfloat16)
        dA = torch.full((32, F), 0.5, device=dev)
        dBg, dBu = torch.full((F, 32), -0.25, device=dev), torch.full((F, 32), 0.125, device=dev)
        K.lora_swiglu_bwd_grads(dtfull, AT, resid, gu, dgu, bits, p, tg, tu, dA, dBg, dBu, s)
        outs.append((dgu, dA, dBg, dBu))
    torch.cuda.synchronize()
    for a_, b_ in zip(*outs):
        assert torch.equal(a_, b_)
    dgu, dA, dBg, dBu = outs[0]
    if F % 256 == 0:
        ref_dgu = torch.empty_like(dgu)
        K.lora_swiglu_bwd(dtfull, AT, resid, gu, ref_dgu, bits, p)
        assert torch.equal(dgu, ref_dgu)
    act = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    K.call("slx_swiglu_fwd", K.P(gu), 2 * F, K.P(act), F, M, F, K.stream_ptr())
    mask = torch.from_numpy(keep_scale(77, M, F, F, p)).to(dev) if p > 0 else 1.0
    xd = (act.float() * mask).bfloat16().double()
    refA = 0.5 + dtfull[:, :32].double().t() @ xd
    refG = -0.25 + s * dgu[:, :F].double().t() @ tg.double()
    refU = 0.125 + s * dgu[:, F:].double().t() @ tu.double()
    for got, ref in ((dA, refA), (dBg, refG), (dBu, refU)):
        torch.testing.assert_close(got.double(), ref, atol=1e-4 * ref.abs().max().item(), rtol=1e-5)


@pytest.mark.parametrize("M,F,p", [(6384, 4864, 0.1), (77, 256, 0.1), (300, 512, 0.0)])
def test_swiglu_lora_down(dev, M, F, p):
    """slx_swiglu_lora_down (SwiGLU forward + the down site's LoRA down-projection in one pass) against the two launches
    it replaces: act bit-identical to slx_swiglu_fwd, t equal to slx_lora_down's up to f32 summation order (one bf16
    ulp), both against torch fp32; two calls on the same workspace agree bitwise."""
    from simlingo_amd.dropmask import keep_bits
    import torch.nn.functional as Fn
    g = torch.Generator(device=dev).manual_seed(41)
    gu = torch.randn(M, 2 * F, device=dev, generator=g).bfloat16()
    A = (torch.randn(32, F, device=dev, generator=g) * 0.05).bfloat16()
    bits = torch.from_numpy(keep_bits(123, M, F, F, p).view("int32")).to(dev) if p > 0 else None
    ws = torch.zeros(K.lib().slx_swiglu_lora_down_ws_floats(M, F), device=dev)
    outs = []
    for _ in range(2):
        act = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
        t = torch.full((M, 48), 7.0, device=dev, dtype=torch.bfloat16)
        K.swiglu_lora_down(gu, act, A, t[:, 8:40], bits, p, ws)
        outs.append((act, t))
    torch.cuda.synchronize()
    (act, t), (act2, t2) = outs
    assert torch.equal(act, act2) and torch.equal(t, t2)
    assert bool((t[:, :8] == 7.0).all()) and bool((t[:, 40:] == 7.0).all())
    ref_act = torch.empty_like(act)
    K.call("slx_swiglu_fwd", K.P(gu), 2 * F, K.P(ref_act), F, M, F, K.stream_ptr())
    assert torch.equal(act, ref_act)
    torch.testing.assert_close(act.float(), (Fn.silu(gu[:, :F].float()) * gu[:, F:].float()), atol=2e-2, rtol=1e-2)
    tl = torch.empty(M, 32, device=dev, dtype=torch.bfloat16)
    K.lora_down(act, [A], tl, [0], p=p, bits=[bits])
    diff = (t[:, 8:40].float() - tl.float()).abs()
    assert (diff <= tl.float().abs() * 2 ** -7 + 1e-4).all(), diff.max().item()
    mask = torch.from_numpy(keep_scale(123, M, F, F, p)).to(dev) if p > 0 else 1.0
    xd = (act.float() * mask).bfloat16().float()
    torch.testing.assert_close(t[:, 8:40].float(), xd @ A.float().t(), atol=3e-2, rtol=2e-2)


@pytest.mark.parametrize("M,kin,nsites", [(300, 256, 3), (6384 // 8 + 5, 896, 2), (1, 128, 4), (6384, 4864, 1)])
def test_lora_down_generates_keep_bits(dev, M, kin, nsites):
    """gen_bits (round 6, the engine's default): slx_lora_down hashes each site's keep mask itself while it reads x and
    writes the bits for the backward - bit-identical to slx_dropout_bits / the host mirror, and t bit-identical to the
    read-the-bits launch (the same masked operand, the same MFMAs)."""
    from simlingo_amd.dropmask import keep_bits
    g = torch.Generator(device=dev).manual_seed(12)
    x = torch.randn(M, kin + 64, device=dev, generator=g).bfloat16()[:, :kin]
    As = [(torch.randn(32, kin, device=dev, generator=g) * 0.1).bfloat16() for _ in range(nsites)]
    seeds = [987654 + 31 * j for j in range(nsites)]
    p = 0.1
    ref_bits = [torch.zeros(M, kin // 32, device=dev, dtype=torch.int32) for _ in range(nsites)]
    K.dropout_bits([(seeds[j], ref_bits[j], kin, kin) for j in range(nsites)], M, p)
    t_ref = torch.zeros(M, 32 * nsites, device=dev).bfloat16()
    K.lora_down(x, As, t_ref, seeds, p=p, bits=ref_bits)
    bits = [torch.full((M, kin // 32), -1, device=dev, dtype=torch.int32) for _ in range(nsites)]
    t = torch.zeros(M, 32 * nsites, device=dev).bfloat16()
    K.lora_down(x, As, t, seeds, p=p, bits=bits, gen=True)
    torch.cuda.synchronize()
    for j in range(nsites):
        assert torch.equal(bits[j], ref_bits[j]), j
        want = torch.from_numpy(keep_bits(seeds[j], M, kin, kin, p).view("int32")).to(dev)
        assert torch.equal(bits[j], want), j
    assert torch.equal(t, t_ref)


@pytest.mark.parametrize("M,F", [(6384, 4864), (77, 256)])
def test_swiglu_lora_down_generates_keep_bits(dev, M, F):
    """slx_swiglu_lora_down with a seed: the down site's keep bits hashed in the pass (mask index m * F + n) and stored
    bytewise - equal to the host mirror - and act / t bit-identical to the launch that reads those bits."""
    from simlingo_amd.dropmask import keep_bits
    g = torch.Generator(device=dev).manual_seed(43)
    gu = torch.randn(M, 2 * F, device=dev, generator=g).bfloat16()
    A = (torch.randn(32, F, device=dev, generator=g) * 0.05).bfloat16()
    p, seed = 0.1, 4242
    want = torch.from_numpy(keep_bits(seed, M, F, F, p).view("int32")).to(dev)
    ws = torch.zeros(K.lib().slx_swiglu_lora_down_ws_floats(M, F), device=dev)
    act_r, t_r = torch.empty(M, F, device=dev, dtype=torch.bfloat16), torch.zeros(M, 32, device=dev, dtype=torch.bfloat16)
    K.swiglu_lora_down(gu, act_r, A, t_r, want.clone(), p, ws)
    bits = torch.full((M, F // 32), -1, device=dev, dtype=torch.int32)
    act, t = torch.empty(M, F, device=dev, dtype=torch.bfloat16), torch.zeros(M, 32, device=dev, dtype=torch.bfloat16)
    K.swiglu_lora_down(gu, act, A, t, bits, p, ws, seed=seed)
    torch.cuda.synchronize()
    assert torch.equal(bits, want)
    assert torch.equal(act, act_r) and torch.equal(t, t_r)
