"""The VLA drop-in surface on the MI355X: DrivingModel.training_step -> loss.backward() -> configure_optimizers()
["optimizer"].step() + OneCycleLR (simlingo_training/models/driving.py:263-271, 718-732; train.py:206 clip 0.3), and
checkpoint loading in the reference layout (train.py:104-111, agent_simlingo.py:223).

Optimizer check: after each engine backward, the engine's gradients are replaced by the fp32 oracle's gradients of
the same step, so FusedAdamW (one HIP kernel over the flat master buffer, global-norm clip inside) and
torch.optim.AdamW(wd 0.1 on every parameter, betas cycled by OneCycleLR) + clip_grad_norm_(0.3) see identical inputs:
master weights must agree to 1e-6. The engine's own gradients are held to cosine >= 0.98 (the tiny-geometry gate) against the oracle first.
"""
import os

import numpy as np
import pytest
import torch

from golden_util import GOLDEN, load_case
from oracle import vla_oracle as O

pytestmark = pytest.mark.gpu


def _model(P, **kw):
    from simlingo_amd.driving import DrivingModel
    m = DrivingModel(vision_model={"variant": "tiny", "freeze": False},
                     language_model={"variant": "tiny", "lora": True, "lora_dropout": 0.0}, init_params=P, **kw)
    m.max_steps = 10
    return m


def test_training_step_backward_optimizer_vs_torch_adamw(dev):
    cfg, P, ex, _ = load_case("nopad")
    model = _model(P)
    conf = model.configure_optimizers()
    opt, sched = conf["optimizer"], conf["lr_scheduler"]["scheduler"]
    assert conf["lr_scheduler"]["interval"] == "step"
    eng = model.engine
    names = [s.name for s in eng.specs if s.trainable]
    ref = {k: P[k].clone().double().requires_grad_(True) for k in names}
    ropt = torch.optim.AdamW(list(ref.values()), lr=cfg.lr, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay)
    rsched = torch.optim.lr_scheduler.OneCycleLR(ropt, max_lr=cfg.lr, total_steps=10, pct_start=cfg.pct_start)
    for step in range(2):
        out = model.training_step(ex, step)
        assert set(out) == {"loss", "outputs"}
        out["loss"].backward()
        torch.cuda.synchronize()
        Pcur = dict(P)
        Pcur.update({k: v.detach().float() for k, v in ref.items()})
        oref, grads = O.loss_and_grads(Pcur, cfg, ex)
        assert abs(out["loss"].item() - oref["loss"].item()) <= 1e-2 * abs(oref["loss"].item())
        for k in ("vit.0.qkv.w", "proj.fc1.w", "llm.1.lora.q.b", "route.0.w"):
            g = eng.G[k].float().cpu().reshape(-1)
            cos = torch.nn.functional.cosine_similarity(g, grads[k].reshape(-1), dim=0).item()
            assert cos >= 0.98, (step, k, cos)  # the tiny-geometry gradient gate of test_vla_parity_gpu.py
        # identical gradients for both optimizers
        for k in names:
            eng.G[k].copy_(grads[k].to(dev))
            ref[k].grad = grads[k].double()
        opt.step()
        sched.step()
        torch.nn.utils.clip_grad_norm_(list(ref.values()), cfg.grad_clip)
        ropt.step()
        rsched.step()
        ropt.zero_grad()
        assert opt.param_groups[0]["betas"] == pytest.approx(ropt.param_groups[0]["betas"])
        assert opt.param_groups[0]["lr"] == pytest.approx(ropt.param_groups[0]["lr"])
        torch.cuda.synchronize()
        worst = max((eng.P[k].double().cpu() - ref[k].detach()).abs().max().item() for k in names)
        assert worst <= 1e-6, (step, worst)
    # per-sample loss values, as summarise_losses receives them (models/utils.py:28-31)
    o = out["outputs"]
    B, L = ex.driving_input.prompt.phrase_ids.shape
    assert o.loss_values["route_loss"].shape == (B, cfg.n_route)
    lv, lc = o.loss_values["language_loss"], o.loss_counts["language_loss"]
    assert lv.shape == lc.shape == (B, L - 1)
    torch.testing.assert_close(lv.sum() / lc.sum(), o.loss_averages["language_loss"], rtol=1e-5, atol=1e-6)


def test_reference_checkpoint_reproduces_golden_losses(dev):
    """The reference-layout state dict of the golden parameters (tests/golden/vla_tiny_refsd.safetensors, written
    from the reference module tree by oracle/gen_golden_ckpt.py) loaded into a fresh DrivingModel reproduces the
    golden fixture's losses (which the reference code computed); state_dict() gives it back."""
    from safetensors.torch import load_file
    from simlingo_amd.driving import DrivingModel
    cfg, P, ex, z = load_case("nopad")
    sd = load_file(os.path.join(GOLDEN, "vla_tiny_refsd.safetensors"))
    m = DrivingModel(vision_model={"variant": "tiny"}, language_model={"variant": "tiny", "lora_dropout": 0.0},
                     seed=123)  # different init: everything must come from the checkpoint
    m.build_engine(dev)
    res = m.load_state_dict(sd)
    assert not res.missing_keys and not res.unexpected_keys
    m.eval()
    out, _ = m.forward_loss(ex)
    got = [out.loss.item(), out.loss_averages["language_loss"].item(), out.loss_averages["route_loss"].item(),
           out.loss_averages["speed_wps_loss"].item()]
    want = [float(z["out.loss"]), float(z["out.language_loss"]), float(z["out.route_loss"]),
            float(z["out.speed_wps_loss"])]
    np.testing.assert_allclose(got, want, rtol=1e-2, atol=1e-4)
    back = m.state_dict()
    for k, v in sd.items():
        tol = 0 if v.dim() == 1 or "lora" in k or "adaptors.driving" in k or "wp_encoder" in k else 4e-3
        assert (back[k].float() - v).abs().max().item() <= tol * max(1.0, v.abs().max().item()), k


def test_frozen_vision_model(dev):
    """vision_model.freeze=True (encoder/vlm.py:35-44): InternViT takes no gradient and no optimizer update, mlp1
    (proj.*) still trains. The engine skips the whole InternViT backward; the step's losses and every remaining
    gradient match the oracle (gradients of the frozen set do not exist), and the ViT weights survive optimizer
    steps bit-identical."""
    from simlingo_amd.driving import DrivingModel
    cfg, P, ex, _ = load_case("nopad")
    m = DrivingModel(vision_model={"variant": "tiny", "freeze": True},
                     language_model={"variant": "tiny", "lora_dropout": 0.0}, init_params=P)
    m.max_steps = 10
    assert m.vla_cfg.vit_freeze
    eng = m.build_engine(dev)
    names = [s.name for s in eng.specs if s.trainable]
    assert not any(n.startswith("vit.") for n in names) and "proj.fc1.w" in names
    vit_before = {k: v.clone() for k, v in eng.W.items() if k.startswith("vit.")}
    vit_before["vit.pos"] = eng.P["vit.pos"].clone()
    opt = m.configure_optimizers()["optimizer"]
    for step in range(2):
        out = m.training_step(ex, step)
        out["loss"].backward()
        torch.cuda.synchronize()
        if step == 0:
            from test_vla_parity_gpu import engine_precision_params
            ref, grads = O.loss_and_grads(engine_precision_params(eng, P), m.vla_cfg, ex)
            assert set(grads) == set(names)
            assert abs(out["loss"].item() - ref["loss"].item()) <= 1e-2 * abs(ref["loss"].item())
            for k in names:
                g, r = eng.G[k].float().cpu().reshape(-1), grads[k].reshape(-1)
                if r.norm() > 1e-12:
                    cos = torch.nn.functional.cosine_similarity(g, r, dim=0).item()
                    assert cos >= 0.98, (k, cos)
        opt.step()
    torch.cuda.synchronize()
    for k, v in vit_before.items():
        cur = eng.P[k] if k == "vit.pos" else eng.W[k]
        assert torch.equal(cur, v), k
