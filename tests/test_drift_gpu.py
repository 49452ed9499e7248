"""Multi-step drift bound (VERDICT r3 "do this" #7): 20 optimizer steps at the REAL InternVL2-1B widths
(2 + 2 layers, as tests/test_fullgeom_parity_gpu.py) on a stream of fresh seeded batches (B = 1, S_text 256, 16 loss
tokens), the reference's training step each time (driving.py:236-261 forward_loss, backward, clip_grad_norm 0.3 from
train.py:206, AdamW(wd 0.1 on all, driving.py:718-732)), lr = 1e-4 (above the reference's 3e-5, so 20 steps move the
trainable weights by ~10 % of their init scale and drift has room to show).

Four trajectories from the same initial parameters:
  E  the bf16 engine (the product path),
  X  the engine's fp32 parity mode (VLAEngine(precise=True): the same launch sequence on f32 operands),
  O  the CPU fp32 oracle with torch's clip + AdamW,
  Q  the oracle computing every step with its GEMM-operand weights rounded to bf16 (the engine's bf16 working copy
     of the f32 master), i.e. bf16 rounding injected into the oracle alone.
Gates, written here:
  * every step's total loss and LM CE of E within 2e-2 relative of O's (the bf16 gate), of X within 1e-4;
  * X vs O after 20 steps: the held-out predictions within 1e-3 m (f32 against f32: only summation order differs,
    which Adam's per-element normalisation turns into +-lr flips of near-zero-gradient elements);
  * E vs the oracle evaluated at E's own final parameters: 5e-2 m (SURVEY.md §8d bf16 gate at the trained point);
  * E vs O: the drift is the mechanism Q isolates - bf16 rounding amplified by Adam's normalised steps - so E's
    distance to O is bounded by 2x Q's distance to O (+ 1e-2 m), not by a fixed number;
  * every tensor whose init dominates its update (init > 20x update): E's parameters within cosine 0.995 of O's; every
    trainable tensor's 20-step update direction within cosine 0.9 of O's (the floor on worst_upd).
"""
import pytest
import torch

from oracle import vla_oracle as O

pytestmark = pytest.mark.gpu

STEPS = 20
LR = 1e-4


def _oracle_trajectory(P0, cfg, names, batches, bf16_names=None):
    ref = {k: v.clone() for k, v in P0.items()}
    for k in names:
        ref[k].requires_grad_(True)
    opt = torch.optim.AdamW([ref[k] for k in names], lr=LR, betas=cfg.betas, eps=cfg.eps,
                            weight_decay=cfg.weight_decay)
    losses = []
    for ex in batches:
        Pe = {k: v.detach() for k, v in ref.items()}
        if bf16_names is not None:
            Pe = {k: (v.bfloat16().float() if k in bf16_names else v) for k, v in Pe.items()}
        r, grads = O.loss_and_grads(Pe, cfg, ex)
        for k in names:
            ref[k].grad = grads[k].clone()
        torch.nn.utils.clip_grad_norm_([ref[k] for k in names], cfg.grad_clip)
        opt.step()
        opt.zero_grad(set_to_none=True)
        losses.append(torch.tensor([r["loss"].item(), r["language_loss"].item()]))
    return {k: v.detach() for k, v in ref.items()}, losses


def _engine_trajectory(eng, cfg, batches, dev):
    from simlingo_amd.plan import plan_from_example
    losses = []
    for i, ex in enumerate(batches):
        plan = plan_from_example(cfg, ex)
        lab = ex.driving_label
        out4, _, _ = eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev),
                                 lab.waypoints.to(dev), training=True)
        eng.backward(None)
        eng.adamw_step(LR, i + 1, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay, max_norm=cfg.grad_clip)
        losses.append(out4[:2].cpu())
    torch.cuda.synchronize()
    return losses


def _engine_predict(eng, cfg, ex, dev):
    from simlingo_amd.plan import plan_from_example
    plan = plan_from_example(cfg, ex)
    lab = ex.driving_label
    _, rp, sp = eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev),
                            lab.waypoints.to(dev), training=False)
    torch.cuda.synchronize()
    return rp.cpu(), sp.cpu()


def _dist(a, b):
    return max((a[0] - b["route_pred"]).abs().max().item(), (a[1] - b["speed_pred"]).abs().max().item())


def test_twenty_step_drift(dev):
    from simlingo_amd.config import full_config
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    torch.set_num_threads(16)
    cfg = full_config(vit_layers=2, llm_layers=2, lora_dropout=0.0)
    P0 = init_params(cfg, seed=7, lora_b_std=0.02)
    names = O.trainable_names(cfg, P0)
    batches = [make_batch(cfg, B=1, s_text=256, n_loss=16, seed=100 + i) for i in range(STEPS)]
    held = make_batch(cfg, B=1, s_text=256, n_loss=16, seed=999)

    eng = VLAEngine(cfg, dev, P0)
    le = _engine_trajectory(eng, cfg, batches, dev)
    bf16_names = set(eng.W)
    pe = _engine_predict(eng, cfg, held, dev)
    Pe = {k: (eng.P[k].detach().float().cpu() if k in names else P0[k]) for k in P0}
    del eng
    engx = VLAEngine(cfg, dev, P0, precise=True)
    lx = _engine_trajectory(engx, cfg, batches, dev)
    px = _engine_predict(engx, cfg, held, dev)
    del engx

    ref, lo = _oracle_trajectory(P0, cfg, names, batches)
    refq, _lq = _oracle_trajectory(P0, cfg, names, batches, bf16_names=bf16_names)
    bad = []
    for i in range(STEPS):
        re_ = ((le[i] - lo[i]).abs() / lo[i].abs()).max().item()
        rx = ((lx[i] - lo[i]).abs() / lo[i].abs()).max().item()
        print(f"step {i}: bf16 {le[i].tolist()} fp32-mode {lx[i].tolist()} oracle {lo[i].tolist()} "
              f"rel {re_:.3g} / {rx:.3g}")
        if re_ > 2e-2 or rx > 1e-4:
            bad.append((i, re_, rx))

    ro, _g = O.loss_and_grads(ref, cfg, held)
    rq, _g = O.loss_and_grads(refq, cfg, held)
    Pe_b = {k: (v.bfloat16().float() if k in bf16_names else v) for k, v in Pe.items()}
    rpe, _g = O.loss_and_grads(Pe_b, cfg, held)
    d_x = _dist(px, ro)          # fp32 parity mode vs the f32 oracle trajectory
    d_e_own = _dist(pe, rpe)     # bf16 engine vs the oracle at the engine's own parameters
    d_e = _dist(pe, ro)          # bf16 engine vs the f32 oracle trajectory
    d_q = max((rq["route_pred"] - ro["route_pred"]).abs().max().item(),
              (rq["speed_pred"] - ro["speed_pred"]).abs().max().item())  # bf16-weight oracle vs f32 oracle
    print(f"final (held-out batch, max |diff| over route + speed points): fp32 mode vs O {d_x:.4g} m; bf16 engine vs "
          f"O at its own parameters {d_e_own:.4g} m; bf16 engine vs O {d_e:.4g} m; bf16-weight oracle Q vs O "
          f"{d_q:.4g} m")
    worst_p, worst_upd = 1.0, 1.0
    for k in names:
        e = Pe[k].reshape(-1)
        o = ref[k].reshape(-1)
        p0 = P0[k].reshape(-1)
        if (o - p0).norm() > 0:
            worst_upd = min(worst_upd, torch.nn.functional.cosine_similarity(e - p0, o - p0, dim=0).item())
        if p0.norm() > 20 * (o - p0).norm():  # tensors whose init dominates their 20-step update
            worst_p = min(worst_p, torch.nn.functional.cosine_similarity(e, o, dim=0).item())
    print(f"worst parameter cosine {worst_p:.6f}, worst update-direction cosine {worst_upd:.4f}")
    assert not bad, bad
    assert d_x <= 1e-3, d_x
    assert d_e_own <= 5e-2, d_e_own
    assert d_e <= 2 * d_q + 1e-2, (d_e, d_q)
    assert worst_p >= 0.995, worst_p
    assert worst_upd >= 0.9, worst_upd
