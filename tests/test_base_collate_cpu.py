"""SimLingo-Base collate (LLaVA-NeXT anyres, pinpoints [[336, 672]]) and the config-1 CPU step.

- anyres_patches is pinned against tests/golden/base_collate.npz, made by transformers' LlavaNextImageProcessor
  (oracle/gen_golden_base_collate.py) on the same seeded 1024 x 512 frames cut to 359 rows (dataset_base.py:445).
  The fixture keeps the global patch first (index 0); the collate drops it (datamodule.py:236-239), so
  use_global=True is compared patch by patch and base_collate is checked to hold patches 1..2.
- config 1 (BASELINE.json configs[0]: simlingo_base, bs=1): one 1024 x 512 frame through base_collate into the
  CPU fp32 step the reference runs (oracle/base_oracle.py forward/backward, torch AdamW over the four parameter
  groups of driving.py:382-400, grad clip 1.0) - full CLIP-L / Llama-tiny geometry.
"""
import os

import numpy as np
import pytest
import torch

from simlingo_amd.base_collate import anyres_patches, base_collate, cut_bottom, select_best_resolution, \
    synthetic_samples
from simlingo_amd.base_config import base_config

GOLD = os.path.join(os.path.dirname(__file__), "golden", "base_collate.npz")


def _frame(seed, H=512, W=1024):
    return np.random.default_rng(seed).integers(0, 256, size=(H, W, 3), dtype=np.uint8)


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_select_best_resolution():
    assert select_best_resolution((359, 1024), [(336, 672)]) == (336, 672)
    # wider frames pick the wider pinpoint; ties go to the least padding
    assert select_best_resolution((359, 1024), [(672, 672), (336, 1008)]) == (336, 1008)
    assert select_best_resolution((500, 500), [(336, 336), (672, 672)]) == (672, 672)


@pytest.mark.parametrize("b", [0, 1])
def test_anyres_matches_llava_next_processor(gold, b):
    f = cut_bottom(_frame(int(gold["seeds"][b])))
    assert list(f.shape[:2]) == gold["image_sizes"][b].tolist() == [359, 1024]
    np.testing.assert_allclose([f.astype(np.float64).sum(), (f.astype(np.float64) ** 2).sum()], gold[f"frame_cs.{b}"])
    pix = anyres_patches(f, pinpoints=((336, 672),), patch=336, use_global=True)
    assert pix.shape == tuple(gold["shape"][1:]) and pix.dtype == np.float32
    idx = gold["idx"]
    for p in range(pix.shape[0]):
        t = pix[p]
        # same Pillow bicubic resize and f32 normalisation as the processor -> equal to f32 rounding
        np.testing.assert_allclose(t.reshape(-1)[idx], gold[f"v.{b}.{p}"], rtol=0, atol=1e-6)
        np.testing.assert_allclose(t[:, [0, 50, 167, 285, 335], :], gold[f"rows.{b}.{p}"], rtol=0, atol=1e-6)
        t64 = t.astype(np.float64)
        np.testing.assert_allclose([t64.sum(), np.abs(t64).sum(), (t64 * t64).sum()], gold[f"cs.{b}.{p}"], rtol=1e-6)


def test_base_collate_layout(gold):
    cfg = base_config()
    samples = synthetic_samples(cfg, 2, seed=1)
    for s, seed in zip(samples, gold["seeds"]):
        s["rgb"] = _frame(int(seed))
    ex = base_collate(samples, cfg)
    di = ex.driving_input
    assert di.camera_images.shape == (2, 1, 1, 2, 3, 336, 336)      # global patch dropped
    assert di.image_sizes.tolist() == gold["image_sizes"].tolist()
    idx = gold["idx"]
    for b in range(2):
        for p in range(2):
            got = di.camera_images[b, 0, 0, p].numpy().reshape(-1)[idx]
            np.testing.assert_allclose(got, gold[f"v.{b}.{p + 1}"], rtol=0, atol=1e-6)
    assert di.map_route.shape == (2, cfg.n_tp, 2) and di.vehicle_speed.shape == (2, 1)
    assert ex.driving_label.route_adjusted.shape == (2, cfg.n_route, 2)
    assert ex.driving_label.waypoints.shape == (2, 11, 2)


def test_config1_cpu_step():
    """BASELINE configs[0]: simlingo_base at full geometry, bs=1, one 1024 x 512 frame -> collate -> the CPU fp32
    forward / backward / AdamW step; three steps on the same sample (overfit) lower the loss."""
    import oracle.base_oracle as BO
    from simlingo_amd.base_params import base_specs, init_base_params

    torch.manual_seed(0)
    cfg = base_config()
    ex = base_collate(synthetic_samples(cfg, 1, seed=7), cfg)
    assert ex.driving_input.camera_images.shape == (1, 1, 1, 2, 3, 336, 336)
    assert ex.driving_input.image_sizes.tolist() == [[cfg.frame_h, cfg.frame_w]]
    P = {k: v.float().requires_grad_() for k, v in init_base_params(cfg, seed=0).items()}
    specs = {s.name: s for s in base_specs(cfg)}
    groups = {}
    for k, v in P.items():  # driving.py:382-400 - (vision?, decay?) -> lr / weight decay
        s = specs.get(k)
        vision, decay = (s.vision, s.decay) if s is not None else (False, False)
        groups.setdefault((vision, decay), []).append(v)
    opt = torch.optim.AdamW([{"params": ps, "lr": cfg.vision_lr if vis else cfg.lr,
                              "weight_decay": cfg.weight_decay if dec else 0.0}
                             for (vis, dec), ps in groups.items()], betas=cfg.betas, eps=cfg.eps)
    losses = []
    with torch.inference_mode(False):
        for _ in range(3):
            out = BO.forward_loss(P, cfg, ex)
            opt.zero_grad(set_to_none=True)
            out["loss"].backward()
            torch.nn.utils.clip_grad_norm_(list(P.values()), cfg.grad_clip)
            opt.step()
            losses.append(float(out["loss"].detach()))
            assert out["route_pred"].shape == (1, cfg.n_route, 2)
            assert out["speed_pred"].shape == (1, cfg.n_speed, 2)
    assert all(np.isfinite(losses)), losses
    assert losses[-1] < losses[0], losses
