"""SimLingo-Base collate: camera frames -> LLaVA-NeXT anyres patches -> the base DrivingExample (SURVEY.md §8f row 1
for the base model; VERDICT r2 missing #3).

Reference path (simlingo_base_training):
  dataset_base.py:433-445   cv2 RGB frame; `cut_bottom_quarter` / `img_shift_augmentation` keep the top
                            int(H - (H * 4.8) // 16) rows (1024 x 512 -> 1024 x 359)
  datamodule.py:220-239     dl_collate_fn: frames [B*T*N, C, H, W] uint8 -> self.processor.image_processor(...,
                            image_grid_pinpoints=[[336, 672]]) -> pixel_values [B*T*N, 1 + npatch, 3, 336, 336];
                            the global (first) patch dropped unless use_global_img (:236-239); image_sizes kept
  datamodule.py:241-266     DrivingExample(DrivingInput(camera_images, image_sizes, intrinsics, extrinsics,
                            vehicle_speed, map_route, target_point), DrivingLabel(...), run_id, timestamp)

The image processor is transformers' LlavaNextImageProcessor [third-party; llava-hf/llava-v1.6-mistral-7b-hf's
published preprocessor config: size.shortest_edge 336, crop 336 x 336, bicubic, CLIP mean / std; the hub file itself
is unavailable offline]. Its anyres patch path is restated here (get_image_patches): select_best_resolution over the
pinpoints, an aspect-preserving Pillow BICUBIC resize (the processor's own resize primitive: PIL.Image.resize),
zero padding centred to the pinpoint, 336 x 336 patches row-major, then per patch rescale 1/255 and normalise in f32
(the 336 -> 336 resize and centre crop are identities). Pinned against the installed transformers processor by
tests/golden/base_collate.npz (oracle/gen_golden_base_collate.py). Host-side numpy + Pillow, like the reference's
CPU DataLoader workers; the CLIP tower consumes the patches on the GPU.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .base_config import BaseConfig
from .base_types import CLIP_MEAN, CLIP_STD, DrivingExample, DrivingInput, DrivingLabel
from .collate import camera_extrinsics, camera_intrinsics, encode_uint8


def cut_bottom(frame: np.ndarray) -> np.ndarray:
    """dataset_base.py:445: keep the top int(H - (H * 4.8) // 16) rows of an [H, W, C] frame."""
    H = frame.shape[0]
    return frame[: int(H - (H * 4.8) // 16)]


def select_best_resolution(hw, pinpoints):
    """LLaVA-NeXT select_best_resolution: the pinpoint (h, w) with the largest effective resolution after an
    aspect-preserving downscale, ties broken by the least wasted area."""
    oh, ow = hw
    best, best_eff, best_waste = None, -1, float("inf")
    for h, w in pinpoints:
        scale = min(w / ow, h / oh)
        dw, dh = int(ow * scale), int(oh * scale)
        eff = min(dw * dh, ow * oh)
        waste = w * h - eff
        if eff > best_eff or (eff == best_eff and waste < best_waste):
            best, best_eff, best_waste = (h, w), eff, waste
    return best


def patch_output_size(hw, target):
    """get_patch_output_size: the aspect-preserving size inside the target resolution."""
    oh, ow = hw
    th, tw = target
    sw, sh = tw / ow, th / oh
    if sw < sh:
        return min(math.ceil(oh * sw), th), tw
    return th, min(math.ceil(ow * sh), tw)


def anyres_patches(frame: np.ndarray, pinpoints=((336, 672),), patch: int = 336, use_global: bool = False,
                   mean=CLIP_MEAN, std=CLIP_STD) -> np.ndarray:
    """One uint8 [H, W, 3] frame -> [npatch (+1), 3, patch, patch] f32 (LlavaNextImageProcessor.get_image_patches +
    _preprocess). The global patch (a plain resize to patch x patch) leads when use_global."""
    from PIL import Image
    H, W = frame.shape[:2]
    th, tw = select_best_resolution((H, W), pinpoints)
    nh, nw = patch_output_size((H, W), (th, tw))
    img = Image.fromarray(np.ascontiguousarray(frame))
    resized = np.asarray(img.resize((nw, nh), resample=Image.BICUBIC))
    py, px = (th - nh) // 2, (tw - nw) // 2
    padded = np.zeros((th, tw, 3), dtype=np.uint8)
    padded[py:py + nh, px:px + nw] = resized
    tiles = [padded[r:r + patch, c:c + patch] for r in range(0, th, patch) for c in range(0, tw, patch)]
    if use_global:
        tiles = [np.asarray(img.resize((patch, patch), resample=Image.BICUBIC))] + tiles
    m = np.asarray(mean, dtype=np.float32).reshape(1, 1, 3)
    s = np.asarray(std, dtype=np.float32).reshape(1, 1, 3)
    out = [((t.astype(np.float32) * np.float32(1 / 255)) - m) / s for t in tiles]
    return np.stack([o.transpose(2, 0, 1) for o in out]).astype(np.float32)


def waypoints_from_ego(full: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """dataset_base.py:368-385 (BaseDataset.load_waypoints, no augmentation): `full` = get_waypoints' ego-frame
    positions [n, 2], current frame first. waypoints = full[1:-1]; waypoints_1d = the cumulative path length to each
    of full[1..n-2] as (distance, 0) pairs (the 1-d speed target of speed_wps_mode '1d', adaptors.py:213)."""
    full = np.asarray(full, dtype=np.float64)
    arc = np.cumsum(np.linalg.norm(full[1:] - full[:-1], axis=1))
    wp1d = np.stack([arc, np.zeros_like(arc)], 1)[:-1]
    return full[1:-1], wp1d


def base_collate(samples: list[dict], cfg: BaseConfig, cut: bool = True) -> DrivingExample:
    """datamodule.py:213-266 for the llavanext encoder. Each sample: 'rgb' uint8 [H, W, 3] (one view, one frame),
    'speed' float, 'target_point' [2], 'map_route' [n_tp, 2] (target points), 'waypoints' [11, 2],
    'waypoints_1d' [11, 2], 'route_adjusted' [n_route, 2], 'measurement_path' str.
    camera_intrinsics / extrinsics are the fixed CARLA camera of :252-253 (get_camera_intrinsics(W, H, 110) of the
    collated frame size, repeated [B, N=1, 3, 3] / [B, 1, 4, 4]); run_id = encode_uint8(measurement paths, 1000)
    (:264)."""
    frames = [cut_bottom(s["rgb"]) if cut else s["rgb"] for s in samples]
    pix = np.stack([anyres_patches(f, pinpoints=((cfg.img_size * cfg.npatch_h, cfg.img_size * cfg.npatch_w),),
                                   patch=cfg.img_size) for f in frames])
    B = len(samples)
    H, W = frames[0].shape[:2]
    sizes = torch.tensor([list(f.shape[:2]) for f in frames])
    wps = torch.tensor(np.stack([s["waypoints"] for s in samples])).float()
    wp1d = torch.tensor(np.stack([s["waypoints_1d"] for s in samples])).float()
    di = DrivingInput(camera_images=torch.from_numpy(pix).view(B, 1, 1, *pix.shape[1:]), image_sizes=sizes,
                      camera_intrinsics=camera_intrinsics(W, H, 110).expand(B, 1, 3, 3).contiguous(),
                      camera_extrinsics=camera_extrinsics().expand(B, 1, 4, 4).contiguous(),
                      vehicle_speed=torch.tensor([[float(s["speed"])] for s in samples]),
                      map_route=torch.tensor(np.stack([s["map_route"] for s in samples])).float(),
                      target_point=torch.tensor(np.stack([s["target_point"] for s in samples])).float())
    dl = DrivingLabel(time_delta_sec=torch.tensor([0.2 * i for i in range(11)]).repeat(B, 1).float(), waypoints=wps,
                      waypoints_1d=wp1d,
                      route_adjusted=torch.tensor(np.stack([s["route_adjusted"] for s in samples])).float())
    return DrivingExample(driving_input=di, driving_label=dl,
                          run_id=encode_uint8([s["measurement_path"] for s in samples], 1000),
                          timestamp=torch.zeros(B, dtype=torch.int64))


def synthetic_samples(cfg: BaseConfig, B: int, seed: int = 0, H: int = 512, W: int = 1024) -> list[dict]:
    """B seeded samples of the dataset's shape: a uniform uint8 1024 x 512 RGB frame, speed, target points, labels."""
    rng = np.random.default_rng(seed)
    out = []
    for b in range(B):
        tp = rng.normal(0.0, 10.0, size=(cfg.n_tp, 2)).astype(np.float32)
        ego = np.concatenate([np.zeros((1, 2)), np.cumsum(np.array([0.8, 0.0]) + 0.3 * rng.normal(size=(12, 2)), 0)])
        wps, wp1d = waypoints_from_ego(ego)
        out.append({"rgb": rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8), "speed": float(rng.uniform(0, 15)),
                    "target_point": tp[0], "map_route": tp,
                    "waypoints": wps.astype(np.float32), "waypoints_1d": wp1d.astype(np.float32),
                    "route_adjusted": np.cumsum(np.array([1.0, 0.0]) + 0.1 * rng.normal(size=(cfg.n_route, 2)),
                                                0).astype(np.float32),
                    "measurement_path": f"synthetic/seed{seed}/Town00_route{b}/measurements"})
    return out
