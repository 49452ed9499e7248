"""LayerNorm / RMSNorm (+ pixel-shuffle gather) parity vs PyTorch fp32."""
import pytest
import torch

from simlingo_amd import kernels as K

pytestmark = pytest.mark.gpu


def pixel_shuffle_v2(x, scale=0.5):
    # InternVL extract_feature pixel_shuffle (ps_version v2), x: [n, w, h, c]
    n, w, h, c = x.size()
    x = x.view(n, w, int(h * scale), int(c / scale))
    x = x.permute(0, 2, 1, 3).contiguous()
    x = x.view(n, int(h * scale), int(w * scale), int(c / (scale * scale)))
    return x.permute(0, 2, 1, 3).contiguous()


@pytest.mark.parametrize("D,rms", [(1024, False), (896, True), (4096, False), (512, True)])
def test_norm(dev, D, rms):
    torch.manual_seed(D)
    rows = 777
    x = torch.randn(rows, D, device=dev) * 2 + 0.5
    g = torch.rand(D, device=dev) + 0.5
    b = torch.randn(D, device=dev)
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    d = K.norm_desc(x, g, None if rms else b, y, None if rms else mean, rstd, rows, D, 1e-6, rms=rms)
    K.norm_fwd(d)
    xr = x.clone().requires_grad_()
    gr = g.clone().requires_grad_()
    br = b.clone().requires_grad_()
    if rms:
        xh = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6)
        # Qwen2RMSNorm: weight * hs.to(input_dtype) -> the weight sees the bf16-rounded xhat
        ref = gr * (xh + (xh.bfloat16().float() - xh).detach())
    else:
        ref = torch.nn.functional.layer_norm(xr, (D,), gr, br, 1e-6)
    assert (y.float() - ref).abs().max().item() < 3e-2
    dy = torch.randn(rows, D, device=dev)
    ref.backward(dy)
    dx = torch.ones(rows, D, device=dev)
    dg = torch.empty(D, device=dev)
    db = torch.empty(D, device=dev)
    ws = torch.empty(K.norm_ws_floats(D), device=dev)
    K.norm_bwd(d, dy, dx, dx_accumulate=True, dgamma=dg, dbeta=None if rms else db, ws=ws)
    torch.testing.assert_close(dx - 1, xr.grad, atol=2e-3, rtol=2e-3)
    torch.testing.assert_close(dg, gr.grad, atol=5e-2, rtol=1e-2)
    if not rms:
        torch.testing.assert_close(db, br.grad, atol=2e-3, rtol=1e-3)


def test_layernorm_pixel_shuffle_gather(dev):
    torch.manual_seed(1)
    n, G, C = 3, 8, 64
    T = 1 + G * G
    xv = torch.randn(n * T, C, device=dev)
    D = 4 * C
    rows = n * (G // 2) ** 2
    g = torch.rand(D, device=dev) + 0.5
    b = torch.randn(D, device=dev)
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    mean = torch.empty(rows, device=dev)
    rstd = torch.empty(rows, device=dev)
    d = K.norm_desc(xv, g, b, y, mean, rstd, rows, D, 1e-5, ps_grid=G, tok_per_img=T)
    K.norm_fwd(d)
    xr = xv.clone().requires_grad_()
    sh = pixel_shuffle_v2(xr.view(n, T, C)[:, 1:].reshape(n, G, G, C)).reshape(rows, D)
    ref = torch.nn.functional.layer_norm(sh, (D,), g, b, 1e-5)
    assert (y.float() - ref).abs().max().item() < 3e-2
    dy = torch.randn(rows, D, device=dev)
    ref.backward(dy)
    dx = torch.zeros(n * T, C, device=dev)
    K.norm_bwd(d, dy, dx, lddx=C)
    torch.testing.assert_close(dx, xr.grad, atol=2e-3, rtol=2e-3)


@pytest.mark.parametrize("rms", [False, True])
def test_norm_bwd_bf16_copy(dev, rms):
    """dx_bf16: the norm backward writes a bf16 copy of the accumulated f32 dx in the same pass."""
    M, D = 777, 896
    g = torch.Generator(device=dev).manual_seed(17)
    x = torch.randn(M, D, device=dev, generator=g)
    gamma = torch.rand(D, device=dev, generator=g) + 0.5
    beta = None if rms else torch.randn(D, device=dev, generator=g)
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    mean = None if rms else torch.empty(M, device=dev)
    rstd = torch.empty(M, device=dev)
    d = K.norm_desc(x, gamma, beta, y, mean, rstd, M, D, 1e-6, rms=rms)
    K.norm_fwd(d)
    dy = torch.randn(M, D, device=dev, generator=g)
    dx = torch.randn(M, D, device=dev, generator=g)
    dxb = torch.empty(M, D + 64, device=dev, dtype=torch.bfloat16)[:, :D]
    K.norm_bwd(d, dy, dx, dx_accumulate=True, dx_bf16=dxb)
    torch.cuda.synchronize()
    assert torch.equal(dxb, dx.bfloat16())


@pytest.mark.parametrize("M", [1025 * 3, 16400])
def test_layernorm_bwd_fused_ls_branch(dev, M):
    """slx_norm_desc.ls*: the InternViT layer-scale branch backward (g = bf16(dx * ls), dls += sum dx * y,
    dbias += sum dx * ls) fused onto the rows the LayerNorm backward just updated, against the separate
    norm backward + slx_ls_branch_bwd of the same inputs (3075 rows: one row per wave at a time; 16400 rows, the
    InternViT step's: two rows in flight per wave)."""
    D = 1024
    gen = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(M, D, device=dev, generator=gen)
    gamma, beta = torch.rand(D, device=dev, generator=gen) + 0.5, torch.randn(D, device=dev, generator=gen)
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    d = K.norm_desc(x, gamma, beta, y, mean, rstd, M, D, 1e-6)
    K.norm_fwd(d)
    dy = torch.randn(M, D, device=dev, generator=gen)
    dx0 = torch.randn(M, D, device=dev, generator=gen)
    ls = torch.rand(D, device=dev, generator=gen) * 0.2
    yb = torch.randn(M, D, device=dev, generator=gen).bfloat16()
    outs = []
    for fused in (False, True):
        dx = dx0.clone()
        dgm, dbt = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        g = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
        dls, dbias = torch.full((D,), 0.5, device=dev), torch.full((D,), -0.25, device=dev)  # accumulate onto these
        ws = torch.empty(K.norm_ws_floats(D), device=dev)
        if fused:
            K.norm_bwd(d, dy, dx, dx_accumulate=True, dgamma=dgm, dbeta=dbt, ws=ws, param_accumulate=True,
                       ls_branch=(ls, yb, g, dls, dbias))
        else:
            K.norm_bwd(d, dy, dx, dx_accumulate=True, dgamma=dgm, dbeta=dbt, ws=ws, param_accumulate=True)
            K.call("slx_ls_branch_bwd", K.P(dx), D, K.P(ls), K.P(yb), D, K.P(g), D, M, D, K.P(dls), K.P(dbias), 1,
                   K.P(torch.empty(2 * 256 * D, device=dev)), K.stream_ptr())
        torch.cuda.synchronize()
        outs.append((dx, g, dls, dbias, dgm, dbt))
    (dx_s, g_s, dls_s, db_s, gm_s, bt_s), (dx_f, g_f, dls_f, db_f, gm_f, bt_f) = outs
    assert torch.equal(dx_s, dx_f) and torch.equal(g_s, g_f)
    ref_dls = 0.5 + (dx_s.double() * yb.double()).sum(0)
    ref_db = -0.25 + (dx_s.double() * ls.double()).sum(0)
    for got in (dls_s, dls_f):
        torch.testing.assert_close(got.double(), ref_dls, rtol=1e-4, atol=1e-3)
    for got in (db_s, db_f):
        torch.testing.assert_close(got.double(), ref_db, rtol=1e-4, atol=1e-3)
    # (column sums over M rows accumulated by f32 atomics in a run-dependent order: the bound scales with M)
    tol = 1e-4 * M / 3075
    torch.testing.assert_close(gm_f, gm_s, rtol=1e-5, atol=tol)
    torch.testing.assert_close(bt_f, bt_s, rtol=1e-5, atol=tol)


@pytest.mark.parametrize("rms,fused_ls", [(False, True), (False, False), (True, False)])
def test_norm_bwd_bf16_dy(dev, rms, fused_ls):
    """slx_norm_desc.dy_bf16: a bf16 dy (what the InternViT fc1 / qkv dgrad GEMMs now hand LayerNorm) gives exactly the
    result of the f32 dy holding the same values, for the wave kernel with and without the fused ls branch."""
    M, D = 1025 * 2 + 7, 1024
    gen = torch.Generator(device=dev).manual_seed(9)
    x = torch.randn(M, D, device=dev, generator=gen)
    gamma, beta = torch.rand(D, device=dev, generator=gen) + 0.5, torch.randn(D, device=dev, generator=gen)
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    d = K.norm_desc(x, gamma, None if rms else beta, y, mean, rstd, M, D, 1e-6, rms=rms)
    K.norm_fwd(d)
    dyb = torch.randn(M, D, device=dev, generator=gen).bfloat16()
    dx0 = torch.randn(M, D, device=dev, generator=gen)
    ls = torch.rand(D, device=dev, generator=gen) * 0.2
    yb = torch.randn(M, D, device=dev, generator=gen).bfloat16()
    outs = []
    for dy in (dyb.float(), dyb):
        dx = dx0.clone()
        dgm, dbt = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        g = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
        dls, dbias = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
        K.norm_bwd(d, dy, dx, dx_accumulate=True, dgamma=dgm, dbeta=None if rms else dbt,
                   ws=torch.empty(K.norm_ws_floats(D), device=dev), param_accumulate=True,
                   ls_branch=(ls, yb, g, dls, dbias) if fused_ls else None)
        torch.cuda.synchronize()
        outs.append((dx, dgm, dbt, g, dls, dbias))
    (dx_f, gm_f, bt_f, g_f, dls_f, db_f), (dx_b, gm_b, bt_b, g_b, dls_b, db_b) = outs
    assert torch.equal(dx_f, dx_b) and torch.equal(g_f, g_b)
    for a, b in ((gm_f, gm_b), (bt_f, bt_b), (dls_f, dls_b), (db_f, db_b)):  # cross-block sums: order may differ
        torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("dy_bf16,fused_ls", [(True, True), (False, True), (True, False)])
def test_layernorm_bwd_1024_many_rows_vs_torch(dev, dy_bf16, fused_ls):
    """The InternViT / CLIP LayerNorm backward at the step's row count (16400 rows of 1024: the branch-free
    norm_bwd_wave1024_kernel, two rows in flight per wave, odd rows per wave included) against a float64 reference of
    the same inputs: dx accumulated onto its input, dgamma / dbeta, and the fused layer-scale branch (g = bf16(dx * ls),
    dls = sum dx * y, dbias = sum dx * ls)."""
    M, D = 16400, 1024
    gen = torch.Generator(device=dev).manual_seed(13)
    x = torch.randn(M, D, device=dev, generator=gen) * 1.5 + 0.25
    gamma, beta = torch.rand(D, device=dev, generator=gen) + 0.5, torch.randn(D, device=dev, generator=gen)
    y = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(M, device=dev), torch.empty(M, device=dev)
    d = K.norm_desc(x, gamma, beta, y, mean, rstd, M, D, 1e-6)
    K.norm_fwd(d)
    dy = torch.randn(M, D, device=dev, generator=gen)
    if dy_bf16:
        dy = dy.bfloat16()
    dx0 = torch.randn(M, D, device=dev, generator=gen)
    ls = torch.rand(D, device=dev, generator=gen) * 0.2
    yb = torch.randn(M, D, device=dev, generator=gen).bfloat16()
    dx = dx0.clone()
    dgm, dbt = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    g = torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    dls, dbias = torch.zeros(D, device=dev), torch.zeros(D, device=dev)
    K.norm_bwd(d, dy, dx, dx_accumulate=True, dgamma=dgm, dbeta=dbt, ws=torch.empty(K.norm_ws_floats(D), device=dev),
               param_accumulate=True, ls_branch=(ls, yb, g, dls, dbias) if fused_ls else None)
    torch.cuda.synchronize()
    xd, dyd = x.double(), dy.double()
    xh = (xd - mean.double()[:, None]) * rstd.double()[:, None]
    gd = dyd * gamma.double()
    ref = rstd.double()[:, None] * (gd - gd.mean(1, keepdim=True) - xh * (gd * xh).mean(1, keepdim=True)) + dx0.double()
    torch.testing.assert_close(dx.double(), ref, rtol=1e-5, atol=2e-5)
    torch.testing.assert_close(dgm.double(), (dyd * xh).sum(0), rtol=1e-4, atol=5e-3)
    torch.testing.assert_close(dbt.double(), dyd.sum(0), rtol=1e-4, atol=5e-3)
    if fused_ls:
        assert torch.equal(g, (dx * ls).bfloat16())
        torch.testing.assert_close(dls.double(), (dx.double() * yb.double()).sum(0), rtol=1e-4, atol=5e-3)
        torch.testing.assert_close(dbias.double(), (dx.double() * ls.double()).sum(0), rtol=1e-4, atol=5e-3)


@pytest.mark.parametrize("rows,D,rms", [(16401, 1024, False), (6384, 896, True), (4097, 512, False)])
def test_norm_fwd_many_rows(dev, rows, D, rms):
    """The norm forward on the step's long row streams (one row per wave, every load unconditional) against a
    float64 reference: bf16 y within its rounding, mean / rstd within f32 rounding."""
    gen = torch.Generator(device=dev).manual_seed(rows)
    x = torch.randn(rows, D, device=dev, generator=gen) * 2 + 0.5
    g = torch.rand(D, device=dev, generator=gen) + 0.5
    b = torch.randn(D, device=dev, generator=gen)
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    d = K.norm_desc(x, g, None if rms else b, y, None if rms else mean, rstd, rows, D, 1e-6, rms=rms)
    K.norm_fwd(d)
    torch.cuda.synchronize()
    xd = x.double()
    mu = torch.zeros(rows, 1, device=dev, dtype=torch.float64) if rms else xd.mean(1, keepdim=True)
    rs = torch.rsqrt(((xd - mu) ** 2).mean(1, keepdim=True) + 1e-6)
    xh = (xd - mu) * rs
    ref = g.double() * (xh.float().bfloat16().double() if rms else xh) + (0 if rms else b.double())
    torch.testing.assert_close(rstd.double(), rs[:, 0], rtol=2e-6, atol=0)
    if not rms:
        torch.testing.assert_close(mean.double(), mu[:, 0], rtol=0, atol=2e-6)
    torch.testing.assert_close(y.double(), ref, rtol=8e-3, atol=8e-3)
