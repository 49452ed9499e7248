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


LABELS = os.path.join(os.path.dirname(__file__), "golden", "base_labels.npz")


def test_base_labels_match_reference_definitions():
    """VERDICT r3 missing #6, pinned by tests/golden/base_labels.npz (oracle/gen_golden_base_labels.py runs the
    reference's own get_camera_intrinsics / get_camera_extrinsics, encode_uint8 and BaseDataset.load_waypoints):
    the camera matrices, waypoints / waypoints_1d from the ego-frame list, and the uint8 run_id rows."""
    from simlingo_amd.base_collate import waypoints_from_ego
    from simlingo_amd.collate import camera_extrinsics, camera_intrinsics, encode_uint8
    z = np.load(LABELS, allow_pickle=False)
    for i, (w, h) in enumerate(z["cam.sizes"].tolist()):
        np.testing.assert_array_equal(camera_intrinsics(w, h, 110).numpy(), z[f"cam.K.{i}"])
    np.testing.assert_array_equal(camera_extrinsics().numpy(), z["cam.E"])
    for s in z["wp.seeds"].tolist():
        wps, wp1d = waypoints_from_ego(z[f"wp.full.{s}"])
        np.testing.assert_allclose(wps, z[f"wp.waypoints.{s}"], rtol=0, atol=1e-12)
        np.testing.assert_allclose(wp1d, z[f"wp.waypoints_1d.{s}"], rtol=0, atol=1e-12)
    np.testing.assert_array_equal(encode_uint8([str(p) for p in z["run.paths"]], 1000).numpy(), z["run.enc"])


def test_base_collate_carries_reference_labels():
    """base_collate puts the reference's fields in the batch: intrinsics of the collated (cut) frame size at fov 110,
    the fixed extrinsics, the sample's own waypoints_1d (not a copy of the 2-d waypoints) and run_id as uint8
    [B, 1000] (datamodule.py:252-264)."""
    from simlingo_amd.base_collate import waypoints_from_ego
    from simlingo_amd.collate import camera_extrinsics, camera_intrinsics
    cfg = base_config()
    z = np.load(LABELS, allow_pickle=False)
    samples = synthetic_samples(cfg, 2, seed=4)
    wps, wp1d = waypoints_from_ego(z["wp.full.12"])
    samples[1]["waypoints"], samples[1]["waypoints_1d"] = wps, wp1d
    samples[1]["measurement_path"] = str(z["run.paths"][0])
    ex = base_collate(samples, cfg)
    di, dl = ex.driving_input, ex.driving_label
    assert di.camera_intrinsics.shape == (2, 1, 3, 3) and di.camera_extrinsics.shape == (2, 1, 4, 4)
    np.testing.assert_array_equal(di.camera_intrinsics[1, 0].numpy(), z["cam.K.0"])  # 1024 x 359 after the cut
    torch.testing.assert_close(di.camera_intrinsics[0, 0], camera_intrinsics(1024, 359, 110))
    torch.testing.assert_close(di.camera_extrinsics[0, 0], camera_extrinsics())
    np.testing.assert_allclose(dl.waypoints_1d[1].numpy(), z["wp.waypoints_1d.12"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(dl.waypoints[1].numpy(), z["wp.waypoints.12"], rtol=1e-6, atol=1e-6)
    assert not torch.equal(dl.waypoints_1d, dl.waypoints)
    assert torch.all(dl.waypoints_1d[..., 1] == 0) and torch.all(dl.waypoints_1d[:, 1:, 0] >= dl.waypoints_1d[:, :-1, 0])
    assert ex.run_id.dtype == torch.uint8 and ex.run_id.shape == (2, 1000)
    np.testing.assert_array_equal(ex.run_id[1].numpy(), z["run.enc"][0])
