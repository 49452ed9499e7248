"""Full VLA training step on the MI355X (HIP engine, bf16 MFMA) vs the CPU fp32 oracle.

Tolerances (bf16 operands, f32 accumulation, 2+2 tiny layers, weights N(0, 0.05)) = SURVEY.md §8d's bf16
gate: losses rel <= 1e-2; waypoint predictions (cumsum of 20 / 10 head outputs) max |diff| <= 5e-2 m; every
trainable gradient cosine >= 0.98 and relative L2 error <= 0.2 (tiny widths: a 128-wide bf16 dot product
carries relatively more rounding than the real 896/1024 widths, which tests/test_fullgeom_parity_gpu.py holds to
cosine >= 0.99 / rel <= 0.1). The north-star 1e-4 m bound is held by the fp32 parity mode below, on the forward
and on a whole training step (forward + backward + clip + AdamW, then the updated model's predictions).
"""
import numpy as np
import pytest
import torch

from golden_util import CASES, load_case
from oracle import vla_oracle as O

pytestmark = pytest.mark.gpu


def run_engine(cfg, P, ex, dev):
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    eng = VLAEngine(cfg, dev, P)
    plan = plan_from_example(cfg, ex)
    dplan = plan.to_device(dev)
    lab = ex.driving_label
    out4, rp, sp = eng.forward(ex.driving_input.camera_images.to(dev), plan, dplan, lab.path.to(dev),
                               lab.waypoints.to(dev))
    eng.backward(None)
    torch.cuda.synchronize()
    return eng, out4.cpu(), rp.cpu(), sp.cpu()


def engine_precision_params(eng, P):
    """The parameters as the bf16 engine computes with them: every tensor it reads as a GEMM operand (eng.W: the
    2-D weights, frozen LLM, embeddings, LoRA A/B) is held in bf16, the rest (biases, norms, layer scales,
    position / query embeddings, the f32 heads and wp_encoder) in f32."""
    return {k: (v.bfloat16().float() if k in eng.W else v) for k, v in P.items()}


@pytest.mark.parametrize("case", CASES)
def test_engine_vs_oracle(dev, case):
    """At the tiny widths (128) with N(0, 0.05) weights, rounding the weights to bf16 alone moves the oracle's route
    points by up to 0.065 m (a systematic shift shared by the 20 query rows, which the cumsum adds up), so the
    arithmetic is judged against the oracle evaluated on the engine's own parameter precision; the losses are
    also held to 1e-2 against the f32-parameter oracle."""
    cfg, P, ex, z = load_case(case)
    eng, out4, rp, sp = run_engine(cfg, P, ex, dev)
    ref32, _ = O.loss_and_grads(P, cfg, ex)
    want32 = [ref32["loss"].item(), ref32["language_loss"].item(), ref32["route_loss"].item(),
              ref32["speed_wps_loss"].item()]
    np.testing.assert_allclose(out4.numpy(), want32, rtol=1e-2, atol=1e-4)
    # a looser bound against the f32-parameter oracle too, so a systematic shift cannot hide behind the bf16-param
    # comparison (0.065 m is the bf16 weight-rounding shift alone; SURVEY's bf16 gate is 0.1 m)
    dr32 = (rp - ref32["route_pred"]).abs().max().item()
    ds32 = (sp - ref32["speed_pred"]).abs().max().item()
    assert dr32 <= 0.1 and ds32 <= 0.1, (dr32, ds32)
    ref, grads = O.loss_and_grads(engine_precision_params(eng, P), cfg, ex)
    want = [ref["loss"].item(), ref["language_loss"].item(), ref["route_loss"].item(), ref["speed_wps_loss"].item()]
    dr, ds = (rp - ref["route_pred"]).abs().max().item(), (sp - ref["speed_pred"]).abs().max().item()
    print(f"[{case}] loss {out4.tolist()} vs {want}; route max {dr:.4g} speed max {ds:.4g}")
    np.testing.assert_allclose(out4.numpy(), want, rtol=1e-2, atol=1e-4)
    assert dr <= 5e-2 and ds <= 5e-2, (dr, ds)
    bad = []
    for name, g in grads.items():
        e = eng.G[name].detach().float().cpu().reshape(-1)
        r = g.reshape(-1)
        if r.norm() < 1e-12:
            continue
        cos = torch.nn.functional.cosine_similarity(e, r, dim=0).item()
        rel = ((e - r).norm() / r.norm()).item()
        if cos < 0.98 or rel > 0.2:
            bad.append((name, round(cos, 4), round(rel, 4)))
    assert not bad, bad


@pytest.mark.parametrize("case", CASES)
def test_precise_forward_north_star(dev, case):
    """fp32 parity mode (csrc/precise.hip): the engine's own launch sequence with f32 operands, held to the
    north-star tolerance against the fp32 oracle — waypoint / route points max |diff| <= 1e-4 m, LM
    cross-entropy |diff| <= 1e-4 (BASELINE.json north_star)."""
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    cfg, P, ex, z = load_case(case)
    ref, _ = O.loss_and_grads(P, cfg, ex)
    eng = VLAEngine(cfg, dev, P, precise=True)
    plan = plan_from_example(cfg, ex)
    lab = ex.driving_label
    out4, rp, sp = eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev),
                               lab.waypoints.to(dev), training=False)
    torch.cuda.synchronize()
    out4, rp, sp = out4.cpu(), rp.cpu(), sp.cpu()
    want = torch.tensor([ref["loss"].item(), ref["language_loss"].item(), ref["route_loss"].item(),
                         ref["speed_wps_loss"].item()])
    d_loss = (out4 - want).abs()
    d_route = (rp - ref["route_pred"]).abs().max().item()
    d_speed = (sp - ref["speed_pred"]).abs().max().item()
    msg = f"loss diffs {d_loss.tolist()} route {d_route:.3g} speed {d_speed:.3g}"
    print(msg)
    assert d_loss[1].item() <= 1e-4 and d_route <= 1e-4 and d_speed <= 1e-4, msg
    assert torch.allclose(out4, want, rtol=1e-4, atol=1e-5), msg


@pytest.mark.parametrize("case", CASES)
def test_precise_train_step_north_star(dev, case):
    """VERDICT r4 missing #1: the TRAINED path at the north-star tolerance. fp32 parity mode forward + backward +
    global-norm clip 0.3 + AdamW (driving.py:718-732, train.py:206) against the oracle's autograd gradients and
    torch.optim.AdamW over the same trainable set: every gradient within 1e-4 relative L2, the parameter update within
    1e-3 relative L2 (and each element within Adam's step size), and the waypoints / route points the updated
    model predicts within 1e-4 m of the oracle's updated model (losses 1e-4 relative)."""
    cfg, P, ex, _ = load_case(case)
    _precise_step(dev, cfg, P, ex, case)


def test_precise_train_step_north_star_full_width(dev):
    """The same north-star step at the REAL InternVL2-1B widths (2 InternViT + 2 Qwen2 layers, T = 1025, GQA 14/2,
    V = 151655, LoRA r32 on the 7 sites, S_text 256 with 16 loss tokens): fp32 parity mode vs the fp32 oracle through
    forward, backward, clip and one AdamW update, then the updated model's route / waypoints within 1e-4 m."""
    from simlingo_amd.config import full_config
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    torch.set_num_threads(16)
    cfg = full_config(vit_layers=2, llm_layers=2, lora_dropout=0.0)
    P = init_params(cfg, seed=7, lora_b_std=0.02)
    ex = make_batch(cfg, B=1, s_text=256, n_loss=16, seed=100)
    _precise_step(dev, cfg, P, ex, "full-width")


def _precise_step(dev, cfg, P, ex, case):
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    assert cfg.lora_dropout == 0.0
    ref, grads = O.loss_and_grads(P, cfg, ex)
    eng = VLAEngine(cfg, dev, P, precise=True)
    plan = plan_from_example(cfg, ex)
    lab = ex.driving_label
    args = (ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev), lab.waypoints.to(dev))
    out4, _, _ = eng.forward(*args, training=True)
    eng.backward(None)
    torch.cuda.synchronize()
    assert abs(out4[0].item() - ref["loss"].item()) <= 1e-4 * abs(ref["loss"].item())
    worst, bad = 0.0, []
    for name, g in grads.items():
        e = eng.G[name].detach().float().cpu().reshape(-1)
        r = g.reshape(-1)
        if r.norm() < 1e-10:
            assert e.norm() < 1e-6, name
            continue
        rel = ((e - r).norm() / r.norm()).item()
        worst = max(worst, rel)
        if rel > 1e-4:
            bad.append((name, rel))
    print(f"[{case}] worst gradient rel L2 {worst:.3g}")
    assert not bad, bad
    # one optimizer step each side
    lr = 1e-4
    Pt = {k: v.detach().clone().float() for k, v in P.items()}
    tr = [k for k in grads]
    for k in tr:
        Pt[k].requires_grad_(True)
        Pt[k].grad = grads[k].clone().float()
    torch.nn.utils.clip_grad_norm_([Pt[k] for k in tr], cfg.grad_clip)
    opt = torch.optim.AdamW([Pt[k] for k in tr], lr=lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay)
    opt.step()
    eng.adamw_step(lr, 1, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay, max_norm=cfg.grad_clip)
    torch.cuda.synchronize()
    # Adam's first step moves every element by ~lr * g / (|g| + eps): an element whose gradient is at the f32 noise
    # floor can land on either side, so the per-element bound is the update size 2 lr; the update as a whole agrees
    # to 1e-3 relative
    dmax = max((eng.P[k].detach().cpu() - Pt[k].detach()).abs().max().item() for k in tr)
    du = torch.cat([(eng.P[k].detach().cpu() - Pt[k].detach()).reshape(-1) for k in tr])
    upd = torch.cat([(Pt[k].detach() - P[k].float()).reshape(-1) for k in tr])
    rel_upd = (du.norm() / upd.norm()).item()
    print(f"[{case}] parameters after the step: max |diff| {dmax:.3g}, update rel L2 {rel_upd:.3g}")
    assert dmax <= 2 * lr and rel_upd <= 1e-3, (dmax, rel_upd)
    Pu = {k: v.detach() for k, v in Pt.items()}
    with torch.no_grad():
        ref2 = O.forward_loss(Pu, cfg, ex)
    out4, rp, sp = eng.forward(*args, training=True)
    torch.cuda.synchronize()
    d_route = (rp.cpu() - ref2["route_pred"]).abs().max().item()
    d_speed = (sp.cpu() - ref2["speed_pred"]).abs().max().item()
    msg = f"after the update: route {d_route:.3g} speed {d_speed:.3g} params {dmax:.3g}"
    print(f"[{case}] {msg}")
    assert d_route <= 1e-4 and d_speed <= 1e-4, msg
    assert abs(out4[0].item() - ref2["loss"].item()) <= 1e-4 * abs(ref2["loss"].item()), msg


def test_engine_vocab_not_multiple_of_128(dev):
    """the fused CE gradient epilogue writes whole 128-column tiles of dlogits, so the engine pads the LM
    head and dlog to a multiple of 128 rows. V = 1030 (64-padding 1088 is not a multiple of 128): the training step
    runs and matches the oracle at the bf16 gate of test_engine_vs_oracle (losses 1e-2 rel, waypoints 5e-2 m)."""
    from simlingo_amd.config import tiny_config
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    cfg = tiny_config(vocab=1030, first_added_id=1030, target_point_id=1037)
    P = init_params(cfg, seed=3, lora_b_std=0.02, std=0.05)
    ex = make_batch(cfg, B=2, s_text=24, n_loss=6, seed=3, pad=[0, 3])
    eng, out4, rp, sp = run_engine(cfg, P, ex, dev)
    assert eng.Vp % 128 == 0 and eng.Vp >= cfg.vocab
    ref, grads = O.loss_and_grads(engine_precision_params(eng, P), cfg, ex)
    want = [ref["loss"].item(), ref["language_loss"].item(), ref["route_loss"].item(), ref["speed_wps_loss"].item()]
    np.testing.assert_allclose(out4.numpy(), want, rtol=1e-2, atol=1e-4)
    assert (rp - ref["route_pred"]).abs().max().item() <= 5e-2
    assert (sp - ref["speed_pred"]).abs().max().item() <= 5e-2
    for name in ("llm.0.lora.q.a", "vit.0.fc1.w", "route.0.w"):
        if name in grads and grads[name].norm() > 1e-12:
            e = eng.G[name].detach().float().cpu().reshape(-1)
            assert torch.nn.functional.cosine_similarity(e, grads[name].reshape(-1), dim=0).item() >= 0.98, name
