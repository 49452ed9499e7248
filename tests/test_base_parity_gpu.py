"""SimLingo-Base training step on the MI355X (BaseEngine, bf16 MFMA / f32 accumulation) vs the CPU fp32
oracle (oracle/base_oracle.py, itself pinned to the reference fixture tests/golden/base_tiny.npz).

Tolerances (bf16 operands, 2 CLIP + 2 Llama tiny layers): SURVEY.md §8d's bf16 gate - losses rel 1e-2, the
cumulated waypoints within 5e-2 m (3e-2 / 0.1 m before); every trainable
gradient cosine >= 0.98 and relative L2 error <= 0.2. Plus one optimizer step against torch.optim.AdamW with
the reference's param groups (decay only on Linear/Conv weights, no decay on route_head) and clip 1.0."""
import pytest
import torch

from base_golden_util import load_base_case
from oracle import base_oracle as O

pytestmark = pytest.mark.gpu


def run(cfg, P, ex, dev):
    from simlingo_amd.base_engine import BaseEngine
    eng = BaseEngine(cfg, dev, P)
    di, dl = ex.driving_input, ex.driving_label
    out4, rp, sp = eng.forward(di.camera_images.to(dev), di.vehicle_speed.to(dev), di.map_route.to(dev),
                               dl.route_adjusted.to(dev), dl.waypoints.to(dev), image_size=tuple(di.image_sizes[0].tolist()))
    eng.backward(None)
    torch.cuda.synchronize()
    return eng, out4.cpu(), rp.cpu(), sp.cpu()


@pytest.mark.parametrize("case", ["tiny", "full1"])
def test_base_engine_vs_oracle(dev, case):
    """tiny widths, and full1: CLIP-L/14-336 width (1024 x 16 heads, 577-token tiles), the 4096-wide projector,
    the 2-tile anyres merge of the 359 x 1024 frame, Llama-tiny width (1 used CLIP layer, 1 Llama layer)."""
    cfg, P, ex, _ = load_base_case(case)
    ref, grads = O.loss_and_grads(P, cfg, ex)
    eng, out4, rp, sp = run(cfg, P, ex, dev)
    rels = {k: abs(got.item() - ref[k].item()) / abs(ref[k].item())
            for got, k in ((out4[0], "loss"), (out4[2], "route_loss"), (out4[3], "speed_wps_loss"))}
    dists = [(got - want).abs().max().item() for got, want in ((rp, ref["route_pred"]), (sp, ref["speed_pred"]))]
    print(f"[{case}] loss rel {rels}, waypoints max |diff| route {dists[0]:.4g} m speed {dists[1]:.4g} m")
    # SURVEY.md §8d's bf16 gate: losses 1e-2 relative, waypoints 5e-2 m
    for k, r in rels.items():
        assert r <= 1e-2, (k, r)
    assert max(dists) <= 5e-2, dists
    bad = []
    for name, r in grads.items():
        e = eng.G[name].detach().float().cpu().reshape(-1)
        r = r.reshape(-1)
        if r.norm() < 1e-12:
            continue
        cos = torch.nn.functional.cosine_similarity(e, r, dim=0).item()
        rel = ((e - r).norm() / r.norm()).item()
        if cos < 0.98 or rel > 0.2:
            bad.append((name, round(cos, 4), round(rel, 4)))
    assert not bad, bad


def test_base_adamw_groups_match_torch(dev):
    """One step of the 4-segment fused AdamW == torch.optim.AdamW over the same gradients and groups."""
    from simlingo_amd.base_params import base_specs
    cfg, P, ex, _ = load_base_case()
    eng, _, _, _ = run(cfg, P, ex, dev)
    lr, vlr, wd = 1e-3, 2e-3, 0.1
    params = {s.name: eng.P[s.name].detach().clone().requires_grad_(True) for s in base_specs(cfg)}
    for s in base_specs(cfg):
        params[s.name].grad = eng.G[s.name].detach().clone()
    groups = []
    for vis in (False, True):
        for dec in (True, False):
            ps = [params[s.name] for s in base_specs(cfg) if s.vision == vis and s.decay == dec]
            groups.append({"params": ps, "lr": vlr if vis else lr, "weight_decay": wd if dec else 0.0})
    torch.nn.utils.clip_grad_norm_(list(params.values()), 1.0)
    opt = torch.optim.AdamW(groups, betas=(0.9, 0.999), eps=1e-8)
    opt.step()
    eng.adamw_step(lr, vlr, 1, weight_decay=wd, max_norm=1.0)
    torch.cuda.synchronize()
    for n, p in params.items():
        torch.testing.assert_close(eng.P[n], p.detach(), rtol=1e-5, atol=1e-6, msg=n)


def test_base_precise_forward_north_star(dev):
    """fp32 parity mode (csrc/precise.hip): BaseEngine's own launch sequence with f32 operands vs the fp32 oracle,
    held to the north-star tolerance — route / speed waypoints max |diff| <= 1e-4 m, losses rel 1e-4."""
    from simlingo_amd.base_engine import BaseEngine
    cfg, P, ex, _ = load_base_case()
    ref = O.forward_loss(P, cfg, ex)
    eng = BaseEngine(cfg, dev, P, precise=True)
    di, dl = ex.driving_input, ex.driving_label
    out4, rp, sp = eng.forward(di.camera_images.to(dev), di.vehicle_speed.to(dev), di.map_route.to(dev),
                               dl.route_adjusted.to(dev), dl.waypoints.to(dev),
                               image_size=tuple(di.image_sizes[0].tolist()))
    torch.cuda.synchronize()
    out4, rp, sp = out4.cpu(), rp.cpu(), sp.cpu()
    d_route = (rp - ref["route_pred"]).abs().max().item()
    d_speed = (sp - ref["speed_pred"]).abs().max().item()
    d_loss = [abs(out4[i].item() - ref[k].item()) for i, k in ((0, "loss"), (2, "route_loss"), (3, "speed_wps_loss"))]
    msg = f"loss diffs {d_loss} route {d_route:.3g} speed {d_speed:.3g}"
    print(msg)
    assert d_route <= 1e-4 and d_speed <= 1e-4, msg
    for i, k in ((0, "loss"), (2, "route_loss"), (3, "speed_wps_loss")):
        assert abs(out4[i].item() - ref[k].item()) <= 1e-4 * abs(ref[k].item()) + 1e-6, msg
    with pytest.raises(RuntimeError):
        eng.backward(None)
