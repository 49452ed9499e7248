"""bf16 training step at the REAL InternVL2-1B widths vs the CPU fp32 oracle (VERDICT r1 "do this" #1).

Geometry: InternViT D=1024, T=1025, 16 heads, FFN 4096 (2 tiles per frame); mlp1 4096->896; Qwen2 d=896,
GQA 14/2, FFN 4864, V=151655 (full-vocab LM head + CE), LoRA r32 on all 7 linears; 2 + 2 layers (depth is
the only reduction, so the oracle finishes in seconds). Cases:
  * config 3: B=2, S_text=256 (S=798), 16 loss tokens per sample, sample 1 left-padded by 37 tokens;
  * config 4: B=1, S_text=512 (S=1054), 128 loss tokens;
  * config 3 with LoRA dropout 0.1 ON: the oracle applies the engine's own hash masks (simlingo_amd.dropmask,
    the same counter-based mask the kernels regenerate), so the dropout step is compared end to end.
HF-default init (weights N(0, 0.02)), LoRA B N(0, 0.02) so the LoRA path carries signal.

Gates (SURVEY.md §8d bf16 target, written here): waypoint / route points max |diff| <= 5e-2 m; LM CE and the
two driving losses rel <= 1e-2; every trainable gradient cosine >= 0.99 and rel-L2 <= 0.1. The observed
maxima are printed (pytest -s) and recorded as user properties.
"""
import numpy as np
import pytest
import torch

from oracle import vla_oracle as O

pytestmark = pytest.mark.gpu

CASES = {
    "cfg3_pad": dict(B=2, s_text=256, n_loss=16, pad=[0, 37], drop=0.0),
    "cfg4": dict(B=1, s_text=512, n_loss=128, pad=None, drop=0.0),
    "cfg3_dropout": dict(B=1, s_text=256, n_loss=16, pad=None, drop=0.1),
}


def _setup(case):
    from simlingo_amd.config import full_config
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    c = CASES[case]
    cfg = full_config(vit_layers=2, llm_layers=2, lora_dropout=c["drop"])
    P = init_params(cfg, seed=7, lora_b_std=0.02)
    ex = make_batch(cfg, B=c["B"], s_text=c["s_text"], n_loss=c["n_loss"], seed=11, pad=c["pad"])
    return cfg, P, ex


def compare(case, dev, record=None):
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    cfg, P, ex = _setup(case)
    eng = VLAEngine(cfg, dev, P)
    plan = plan_from_example(cfg, ex)
    lab = ex.driving_label
    eng.step_seed = 41
    masks = None
    if cfg.lora_dropout > 0:
        from simlingo_amd.dropmask import lora_masks
        masks = lora_masks(cfg, plan.B * plan.S, step_seed=eng.step_seed + 1)  # forward() increments step_seed
    out4, rp, sp = eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev),
                               lab.waypoints.to(dev), training=True)
    eng.backward(None)
    torch.cuda.synchronize()
    torch.set_num_threads(16)
    ref, grads = O.loss_and_grads(P, cfg, ex, dropout_masks=masks)
    out4, rp, sp = out4.cpu(), rp.cpu(), sp.cpu()
    want = torch.tensor([ref["loss"].item(), ref["language_loss"].item(), ref["route_loss"].item(),
                         ref["speed_wps_loss"].item()])
    rel_loss = ((out4 - want).abs() / want.abs().clamp_min(1e-6))
    d_route = (rp - ref["route_pred"]).abs().max().item()
    d_speed = (sp - ref["speed_pred"]).abs().max().item()
    worst_cos, worst_rel, bad = 1.0, 0.0, []
    for name, g in grads.items():
        e = eng.G[name].detach().float().cpu().reshape(-1)
        r = g.reshape(-1)
        if r.norm() < 1e-12:
            continue
        cos = torch.nn.functional.cosine_similarity(e, r, dim=0).item()
        rel = ((e - r).norm() / r.norm()).item()
        worst_cos, worst_rel = min(worst_cos, cos), max(worst_rel, rel)
        if cos < 0.99 or rel > 0.1:
            bad.append((name, round(cos, 5), round(rel, 4)))
    obs = dict(loss=out4.tolist(), oracle=want.tolist(), rel_loss=rel_loss.tolist(), route_max=d_route,
               speed_max=d_speed, worst_grad_cos=worst_cos, worst_grad_rel=worst_rel, S=plan.S, R=int(plan.loss_pos.size))
    print(f"[{case}] {obs} bad={bad}")
    if record is not None:
        for k, v in obs.items():
            record(k, v)
    return obs, bad


@pytest.mark.parametrize("case", list(CASES))
def test_full_geometry_step(dev, case, record_property):
    obs, bad = compare(case, dev, record_property)
    assert max(obs["rel_loss"]) <= 1e-2, obs
    assert obs["route_max"] <= 5e-2 and obs["speed_max"] <= 5e-2, obs
    assert not bad, bad
    # regression gates at ~3x the maxima observed over these cases (loss rel 3.7e-4, points 3e-3 m, cosine 0.9999)
    assert max(obs["rel_loss"]) <= 1.2e-3, obs
    assert max(obs["route_max"], obs["speed_max"]) <= 1e-2, obs
    assert obs["worst_grad_cos"] >= 0.9997, obs


def test_engine_vs_reference_full1_fixture(dev):
    """The bf16 step against the REFERENCE-generated full-width fixture directly (tests/golden/vla_full1.npz,
    oracle/gen_golden.py: the reference's AdaptorList / replace_placeholder_tokens / summarise_losses on the
    transformers InternViT / mlp1 / Qwen2 mirrors; 1 + 1 layers, GQA 14/2, V = 151655, left-padded B = 2, S = 798).
    Same bf16 gates as above: losses rel <= 1e-2, route / speed points <= 5e-2 m; the stored gradient samples of
    every trainable tensor cosine >= 0.99 against the engine's."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from golden_util import grad_entries, load_full_case
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    cfg, P, ex, z = load_full_case("full1")
    eng = VLAEngine(cfg, dev, P)
    plan = plan_from_example(cfg, ex)
    lab = ex.driving_label
    out4, rp, sp = eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev),
                               lab.waypoints.to(dev), training=True)
    eng.backward(None)
    torch.cuda.synchronize()
    want = np.asarray([float(z["out.loss"]), float(z["out.language_loss"]), float(z["out.route_loss"]),
                       float(z["out.speed_wps_loss"])])
    got = out4.cpu().numpy()
    assert np.all(np.abs(got - want) <= 1e-2 * np.abs(want)), (got, want)
    assert np.abs(rp.cpu().numpy() - z["out.route_pred"]).max() <= 5e-2
    assert np.abs(sp.cpu().numpy() - z["out.speed_pred"]).max() <= 5e-2
    bad = []
    for name in eng.G:
        if "gs." + name not in z:
            continue
        idx, ref = grad_entries(z, name)
        e = eng.G[name].detach().float().cpu().reshape(-1)[torch.from_numpy(np.asarray(idx))]
        r = torch.from_numpy(np.asarray(ref)).float()
        if r.norm() < 1e-12:
            continue
        cos = torch.nn.functional.cosine_similarity(e, r, dim=0).item()
        if cos < 0.99:
            bad.append((name, round(cos, 4)))
    assert not bad, bad
