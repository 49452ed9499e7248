"""Parity at the REAL depth (VERDICT r5 "do this" #1): the whole model the reference trains, not a 2 + 2 slice.

  * config 3: InternViT 24 layers + mlp1 + Qwen2 24 layers + LoRA r32 on the 7 sites, V = 151655, B = 2 with sample 1
    left-padded by 37 tokens (S = 798), 16 loss tokens per sample — DrivingModel.forward_model / forward_loss
    (/root/reference/simlingo_training/models/driving.py:190-261, extract_feature internvl2_model.py:114, the LLM
    llm.py:88-119);
      - the bf16 engine step (forward + backward) against the fp32 oracle: SURVEY §8d's gates (losses 1e-2 relative,
        route / speed points 5e-2 m, every trainable gradient cosine >= 0.99) AND regression gates at ~3x the maxima
        observed on the round-6 build (REGRESSION below), so a numerics change that loses an order of magnitude fails
        even while it stays inside §8d;
      - the fp32 parity mode's step (forward + backward + clip 0.3 + AdamW, configure_optimizers driving.py:718-732,
        gradient_clip_val train.py:206) against the oracle's autograd + torch.optim.AdamW, then the UPDATED model's
        route / waypoints within the north-star 1e-4 m of the oracle's updated model;
  * config 2 (SimLingo-Base): 24 CLIP layers (23 used, hidden_states[-2]) + the 4096 projector + 12 Llama layers,
    B = 2 — the bf16 step at §8d's gates + regression gates, and the fp32 parity forward at 1e-4 m.

The oracle runs on the box's host cores (~10 s per VLA sample forward + backward on 16 threads); one oracle pass per
model is shared by the tests of that model (module fixtures). Observed maxima are printed (pytest -s / -v -rA).
"""
import numpy as np
import pytest
import torch

from oracle import vla_oracle as O

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

# §8d's bf16 gates
LOSS_REL_8D, WP_8D, COS_8D = 1e-2, 5e-2, 0.99
# regression gates: ~3x the maxima the round-6 build showed on these exact inputs (printed by the tests). Observed
# (gpurun_out/r6a_tests.log -> DESIGN.md): VLA loss rel 7.3e-4, route 9.2e-3 m, speed 1.06e-2 m, worst gradient cosine
# 0.99965 (llm.4.lora.k.a); SimLingo-Base loss rel 1.25e-3, route 1.48e-2 m, speed 5.5e-3 m, worst cosine 0.99994
REGRESSION = dict(loss_rel=2.5e-3, wp=3e-2, cos=0.999)
BASE_REGRESSION = dict(loss_rel=4e-3, wp=4.5e-2, cos=0.9998)


def _grad_stats(eng_G, grads):
    worst_cos, worst_rel, worst_name, rows = 1.0, 0.0, None, []
    for name, g in grads.items():
        e = eng_G[name].detach().float().cpu().reshape(-1)
        r = g.reshape(-1)
        if r.norm() < 1e-12:
            continue
        cos = torch.nn.functional.cosine_similarity(e, r, dim=0).item()
        rel = ((e - r).norm() / r.norm()).item()
        rows.append((name, cos, rel))
        if cos < worst_cos:
            worst_cos, worst_name = cos, name
        worst_rel = max(worst_rel, rel)
    return worst_cos, worst_rel, worst_name, rows


# ------------------------------------------------------------------------------------------------------------------
# config 3: the full VLA


@pytest.fixture(scope="module")
def vla_case():
    from simlingo_amd.config import full_config
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    torch.set_num_threads(16)
    cfg = full_config(lora_dropout=0.0)
    assert cfg.vit_layers == 24 and cfg.llm_layers == 24
    P = init_params(cfg, seed=7, lora_b_std=0.02)
    ex = make_batch(cfg, B=2, s_text=256, n_loss=16, seed=11, pad=[0, 37])
    ref, grads = O.loss_and_grads(P, cfg, ex)
    return cfg, P, ex, ref, grads


def _vla_args(ex, plan, dev):
    lab = ex.driving_label
    return (ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev), lab.waypoints.to(dev))


def test_fulldepth_vla_bf16_step(dev, vla_case, record_property):
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    cfg, P, ex, ref, grads = vla_case
    eng = VLAEngine(cfg, dev, P)
    plan = plan_from_example(cfg, ex)
    assert plan.S == 798
    out4, rp, sp = eng.forward(*_vla_args(ex, plan, dev), training=True)
    eng.backward(None)
    torch.cuda.synchronize()
    out4, rp, sp = out4.cpu(), rp.cpu(), sp.cpu()
    want = torch.tensor([ref[k].item() for k in ("loss", "language_loss", "route_loss", "speed_wps_loss")])
    rel_loss = ((out4 - want).abs() / want.abs().clamp_min(1e-6)).max().item()
    d_route = (rp - ref["route_pred"]).abs().max().item()
    d_speed = (sp - ref["speed_pred"]).abs().max().item()
    worst_cos, worst_rel, worst_name, rows = _grad_stats(eng.G, grads)
    obs = dict(loss=out4.tolist(), oracle=want.tolist(), loss_rel_max=rel_loss, route_max=d_route, speed_max=d_speed,
               worst_grad_cos=worst_cos, worst_grad_cos_name=worst_name, worst_grad_rel=worst_rel, n_grads=len(rows))
    print(f"[fulldepth vla bf16] {obs}")
    for k, v in obs.items():
        record_property(k, v)
    del eng
    torch.cuda.empty_cache()
    # SURVEY §8d
    assert rel_loss <= LOSS_REL_8D and d_route <= WP_8D and d_speed <= WP_8D, obs
    bad = [(n, round(c, 5), round(r, 4)) for n, c, r in rows if c < COS_8D]
    assert not bad, bad
    # regression gates
    assert rel_loss <= REGRESSION["loss_rel"], obs
    assert max(d_route, d_speed) <= REGRESSION["wp"], obs
    assert worst_cos >= REGRESSION["cos"], obs


def test_fulldepth_vla_precise_step_north_star(dev, vla_case, record_property):
    """fp32 parity mode at 24 + 24 layers: gradients within 1e-4 relative L2 of the oracle's autograd, one clip 0.3 +
    AdamW step each side, then the updated model's route / waypoints within 1e-4 m and its loss within 1e-4 relative
    of the oracle's updated model."""
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    cfg, P, ex, ref, grads = vla_case
    eng = VLAEngine(cfg, dev, P, precise=True)
    plan = plan_from_example(cfg, ex)
    args = _vla_args(ex, plan, dev)
    out4, _, _ = eng.forward(*args, training=True)
    eng.backward(None)
    torch.cuda.synchronize()
    loss_rel = abs(out4[0].item() - ref["loss"].item()) / abs(ref["loss"].item())
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
    print(f"[fulldepth vla precise] loss rel {loss_rel:.3g}, worst gradient rel L2 {worst:.3g}")
    assert loss_rel <= 1e-4
    assert not bad, bad[:10]
    lr = 1e-4
    tr = list(grads)
    Pt = {k: P[k].detach().clone().float() for k in tr}
    for k in tr:
        Pt[k].requires_grad_(True)
        Pt[k].grad = grads[k].clone().float()
    torch.nn.utils.clip_grad_norm_([Pt[k] for k in tr], cfg.grad_clip)
    opt = torch.optim.AdamW([Pt[k] for k in tr], lr=lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay)
    opt.step()
    eng.adamw_step(lr, 1, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay, max_norm=cfg.grad_clip)
    torch.cuda.synchronize()
    du = torch.cat([(eng.P[k].detach().cpu() - Pt[k].detach()).reshape(-1) for k in tr])
    upd = torch.cat([(Pt[k].detach() - P[k].float()).reshape(-1) for k in tr])
    rel_upd = (du.norm() / upd.norm()).item()
    dmax = du.abs().max().item()
    del du, upd
    Pu = dict(P)
    Pu.update({k: v.detach() for k, v in Pt.items()})
    with torch.no_grad():
        ref2 = O.forward_loss(Pu, cfg, ex)
    out4, rp, sp = eng.forward(*args, training=True)
    torch.cuda.synchronize()
    d_route = (rp.cpu() - ref2["route_pred"]).abs().max().item()
    d_speed = (sp.cpu() - ref2["speed_pred"]).abs().max().item()
    loss2_rel = abs(out4[0].item() - ref2["loss"].item()) / abs(ref2["loss"].item())
    obs = dict(loss_rel=loss_rel, worst_grad_rel=worst, update_rel=rel_upd, param_max=dmax, route_after=d_route,
               speed_after=d_speed, loss_after_rel=loss2_rel)
    print(f"[fulldepth vla precise] {obs}")
    for k, v in obs.items():
        record_property(k, v)
    eng.saved = None
    del eng
    torch.cuda.empty_cache()
    assert dmax <= 2 * lr and rel_upd <= 1e-3, obs
    assert d_route <= 1e-4 and d_speed <= 1e-4, obs
    assert loss2_rel <= 1e-4, obs


# ------------------------------------------------------------------------------------------------------------------
# config 2: SimLingo-Base at its real depth


@pytest.fixture(scope="module")
def base_case():
    from oracle import base_oracle as BO
    from simlingo_amd.base_config import base_config
    from simlingo_amd.base_params import init_base_params
    from simlingo_amd.base_types import make_base_batch
    torch.set_num_threads(16)
    cfg = base_config()
    assert cfg.vit_layers == 24 and cfg.vit_used == 23 and cfg.llm_layers == 12
    P = init_base_params(cfg, seed=9, std=0.02)
    ex = make_base_batch(cfg, B=2, seed=10)
    ref, grads = BO.loss_and_grads(P, cfg, ex)
    return cfg, P, ex, ref, grads


def _base_run(cfg, P, ex, dev, precise=False, backward=True):
    from simlingo_amd.base_engine import BaseEngine
    eng = BaseEngine(cfg, dev, P, precise=precise)
    di, dl = ex.driving_input, ex.driving_label
    out4, rp, sp = eng.forward(di.camera_images.to(dev), di.vehicle_speed.to(dev), di.map_route.to(dev),
                               dl.route_adjusted.to(dev), dl.waypoints.to(dev),
                               image_size=tuple(di.image_sizes[0].tolist()))
    if backward:
        eng.backward(None)
    torch.cuda.synchronize()
    return eng, out4.cpu(), rp.cpu(), sp.cpu()


def test_fulldepth_base_bf16_step(dev, base_case, record_property):
    cfg, P, ex, ref, grads = base_case
    eng, out4, rp, sp = _base_run(cfg, P, ex, dev)
    rels = {k: abs(out4[i].item() - ref[k].item()) / abs(ref[k].item())
            for i, k in ((0, "loss"), (2, "route_loss"), (3, "speed_wps_loss"))}
    d_route = (rp - ref["route_pred"]).abs().max().item()
    d_speed = (sp - ref["speed_pred"]).abs().max().item()
    worst_cos, worst_rel, worst_name, rows = _grad_stats(eng.G, grads)
    obs = dict(loss_rel=rels, route_max=d_route, speed_max=d_speed, worst_grad_cos=worst_cos,
               worst_grad_cos_name=worst_name, worst_grad_rel=worst_rel, n_grads=len(rows))
    print(f"[fulldepth base bf16] {obs}")
    for k, v in obs.items():
        record_property(k, v)
    del eng
    torch.cuda.empty_cache()
    assert max(rels.values()) <= LOSS_REL_8D and max(d_route, d_speed) <= WP_8D, obs
    bad = [(n, round(c, 5), round(r, 4)) for n, c, r in rows if c < 0.98]
    assert not bad, bad
    assert max(rels.values()) <= BASE_REGRESSION["loss_rel"], obs
    assert max(d_route, d_speed) <= BASE_REGRESSION["wp"], obs
    assert worst_cos >= BASE_REGRESSION["cos"], obs


def test_fulldepth_base_precise_forward_north_star(dev, base_case):
    cfg, P, ex, ref, _ = base_case
    eng, out4, rp, sp = _base_run(cfg, P, ex, dev, precise=True, backward=False)
    d_route = (rp - ref["route_pred"]).abs().max().item()
    d_speed = (sp - ref["speed_pred"]).abs().max().item()
    d_loss = {k: abs(out4[i].item() - ref[k].item()) / abs(ref[k].item())
              for i, k in ((0, "loss"), (2, "route_loss"), (3, "speed_wps_loss"))}
    print(f"[fulldepth base precise] route {d_route:.3g} speed {d_speed:.3g} loss rel {d_loss}")
    del eng
    torch.cuda.empty_cache()
    assert d_route <= 1e-4 and d_speed <= 1e-4, (d_route, d_speed)
    assert max(d_loss.values()) <= 1e-4, d_loss
