"""Data-gradient GEMMs over transposed weight copies (engine.NT_DGRAD): the batched bf16 transpose
(slx_transpose_bf16), slx_pack_scaled's transposed mode, and the VLA step with the NT data-gradient path against
the same step run NN over the weights themselves (identical operands and K order, so the gradients agree up
to f32 atomic-accumulation order: split-K weight gradients and column sums add partials in arrival order), across an
optimizer step (the copies are refreshed from the updated bf16 weights)."""
import ctypes

import numpy as np
import pytest
import torch

from golden_util import load_case
from simlingo_amd import kernels as K

pytestmark = pytest.mark.gpu


def _transpose(pairs):
    rows = [[w.data_ptr(), w.stride(0), wt.data_ptr(), wt.stride(0), w.shape[0], w.shape[1]] for w, wt in pairs]
    tiles = max(((w.shape[0] + 63) // 64) * ((w.shape[1] + 63) // 64) for w, _ in pairs)
    tab = torch.tensor(rows, dtype=torch.int64, device=pairs[0][0].device)
    K.call("slx_transpose_bf16", K.P(tab), len(pairs), tiles, K.stream_ptr())
    torch.cuda.synchronize()


def test_transpose_bf16(dev):
    g = torch.Generator(device=dev).manual_seed(3)
    shapes = [(4096, 1024), (1024, 3072), (896, 1152), (1, 1), (70, 130), (64, 8), (200, 72)]
    srcs, dsts = [], []
    for r, c in shapes:
        base = torch.randn(r, c + 8, device=dev, generator=g).bfloat16()
        srcs.append(base[:, :c])  # row stride c + 8: strided source
        dsts.append(torch.full((c, r + 16), 7.0, device=dev, dtype=torch.bfloat16)[:, :r])
    _transpose(list(zip(srcs, dsts)))
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.t()), s.shape
    # the padding columns of the strided destinations are untouched
    for d in dsts:
        full = torch.as_strided(d, (d.shape[0], d.stride(0)), (d.stride(0), 1))
        assert bool((full[:, d.shape[1]:] == 7.0).all())
    # an odd (2-byte aligned) source takes the element-wise path
    raw = torch.randn(129 * 65 + 1, device=dev, generator=g).bfloat16()
    s = raw[1:].view(129, 65)
    d = torch.empty(65, 129, device=dev, dtype=torch.bfloat16)
    _transpose([(s, d)])
    assert torch.equal(d, s.t())
    with pytest.raises(RuntimeError, match="slx_transpose_bf16"):
        K.call("slx_transpose_bf16", ctypes.c_void_p(0), -1, 1, K.stream_ptr())


def test_pack_scaled_transposed(dev):
    g = torch.Generator(device=dev).manual_seed(4)
    b = torch.randn(96, 32, device=dev, generator=g)
    dst = torch.zeros(40, 200, device=dev, dtype=torch.bfloat16)
    view = dst[4:36, 10:106]  # [32, 96] window, row stride 200
    s = 0.25
    tab = torch.tensor([[b.data_ptr(), b.stride(0), view.data_ptr(), view.stride(0), 96, 32,
                         int(np.float32(s).view(np.int32)), 4]], dtype=torch.int64, device=dev)
    K.call("slx_pack_scaled", K.P(tab), 1, K.stream_ptr())
    torch.cuda.synchronize()
    want = torch.zeros_like(dst)
    want[4:36, 10:106] = (b * s).bfloat16().t()
    assert torch.equal(dst, want)


def _step(monkeypatch, nt, case):
    import simlingo_amd.engine as E
    from simlingo_amd.plan import plan_from_example
    monkeypatch.setattr(E, "NT_DGRAD", nt)
    monkeypatch.setattr(E, "GEMM_LT", False)  # slx_gemm_bf16 on both sides: the NT / NN main loops are the subject
    cfg, P, ex, _ = load_case(case)
    dev = torch.device("cuda")
    eng = E.VLAEngine(cfg, dev, P)
    assert bool(eng.WT) == nt
    plan = plan_from_example(cfg, ex)
    lab = ex.driving_label
    eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev),
                lab.waypoints.to(dev))
    eng.backward(None)
    torch.cuda.synchronize()
    return eng


def _check_copies(eng):
    """Every transposed copy equals the transpose of the operand the NN path would read."""
    for n, wt in eng.WT.items():
        assert torch.equal(wt, eng.W[n].t()), n
    for cats in eng.cat:
        for g in ("qkv", "o", "gu", "down"):
            assert torch.equal(cats["T." + g], cats[g].t()), g


@pytest.mark.parametrize("case", ["nopad", "leftpad"])
def test_nt_dgrad_step_matches_nn(dev, monkeypatch, case):
    e_nt = _step(monkeypatch, True, case)
    e_nn = _step(monkeypatch, False, case)
    a, b = e_nt.grad, e_nn.grad
    err = (a - b).abs().max().item()
    assert err <= 1e-5 * a.abs().max().item(), err
    _check_copies(e_nt)
    # after an optimizer step the copies follow the updated weights (and the LoRA B columns of the concatenated
    # Qwen2 operands, packed transposed by slx_pack_scaled)
    e_nt.adamw_step(1e-2, 1)
    torch.cuda.synchronize()
    _check_copies(e_nt)


def test_base_engine_copies_follow_optimizer(dev):
    """SimLingo-Base: every weight is trainable, so every transposed copy is refreshed after each AdamW step."""
    from base_golden_util import load_base_case
    from simlingo_amd.base_engine import BaseEngine
    cfg, P, ex, _ = load_base_case("tiny")
    eng = BaseEngine(cfg, dev, P)
    assert eng.WT
    eng.grad.normal_()
    eng.adamw_step(1e-2, 1e-2, 1)
    torch.cuda.synchronize()
    for n, wt in eng.WT.items():
        assert torch.equal(wt, eng.W[n].t()), n


def test_pack_scaled_flat_equals_per_entry_grid(dev):
    """slx_pack_scaled_flat (one block per 2048 elements through a block map) writes exactly what slx_pack_scaled
    (32 blocks per entry) writes, for every mode: 0 / 1 row-major bf16 / f32, 2 / 3 the LoRA fragment orders (32 rows),
    4 transposed; entries from a few elements to more than one chunk per thread."""
    g = torch.Generator(device=dev).manual_seed(8)
    specs = [(0, 96, 32), (1, 40, 32), (2, 32, 896), (3, 32, 4864), (4, 4864, 32), (0, 3, 5), (4, 130, 7), (2, 32, 64)]
    srcs, outs = [], {True: [], False: []}
    for mode, r, c in specs:
        srcs.append(torch.randn(r, c + 3, device=dev, generator=g)[:, :c])
    for flat in (False, True):
        rows = []
        for (mode, r, c), src in zip(specs, srcs):
            if mode in (2, 3):
                dst = torch.zeros(r * c, device=dev, dtype=torch.bfloat16)
                ld = 0
            elif mode == 4:
                dst = torch.zeros(c, r + 6, device=dev, dtype=torch.bfloat16)
                ld = dst.stride(0)
            else:
                dst = torch.zeros(r, c + 6, device=dev, dtype=torch.float32 if mode == 1 else torch.bfloat16)
                ld = dst.stride(0)
            outs[flat].append(dst)
            rows.append([src.data_ptr(), src.stride(0), dst.data_ptr(), ld, r, c,
                         int(np.float32(0.75).view(np.int32)), mode])
        tab = torch.tensor(rows, dtype=torch.int64, device=dev)
        if flat:
            bmap = [e | (k << 16) for e, row in enumerate(rows) for k in range((row[4] * row[5] + 2047) // 2048)]
            bm = torch.tensor(bmap, dtype=torch.int32, device=dev)
            K.call("slx_pack_scaled_flat", K.P(tab), len(rows), K.P(bm), len(bmap), K.stream_ptr())
        else:
            K.call("slx_pack_scaled", K.P(tab), len(rows), K.stream_ptr())
        torch.cuda.synchronize()
    for a, b in zip(outs[False], outs[True]):
        assert torch.equal(a, b)
    assert bool((outs[True][4][:, 4864:] == 0).all())  # nothing past the transposed rows
