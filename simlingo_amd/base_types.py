"""SimLingo-Base batch schema (field-for-field mirror of simlingo_base_training/utils/custom_types.py:57-118)
and seeded synthetic batches of its shape (no dataset offline)."""
from __future__ import annotations

from typing import NamedTuple

import numpy as np
import torch
from torch import Tensor

from .base_config import BaseConfig

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)   # LLaVA-NeXT image processor (CLIP statistics)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


class DrivingInput(NamedTuple):   # custom_types.py:68-86
    camera_images: Tensor         # [B, T=1, N=1, npatch, 3, 336, 336] f32 (processor output)
    image_sizes: Tensor           # [B*T*N, 2] original (height, width)
    camera_intrinsics: Tensor
    camera_extrinsics: Tensor
    vehicle_speed: Tensor         # [B, 1] m/s
    map_route: Tensor             # [B, 2, 2] target_point, next_target_point (route_as 'target_point')
    target_point: Tensor          # [B, 2]


class DrivingLabel(NamedTuple):   # custom_types.py:88-103
    time_delta_sec: Tensor
    waypoints: Tensor             # [B, 11, 2]
    waypoints_1d: Tensor
    route_adjusted: Tensor        # [B, 20, 2]


class DrivingExample(NamedTuple):  # custom_types.py:105-118
    driving_input: DrivingInput
    driving_label: DrivingLabel
    run_id: Tensor                # [B, 1000] uint8 (encode_uint8 of the measurement paths, datamodule.py:264)
    timestamp: Tensor


def _waypoints_1d(wps: Tensor) -> Tensor:
    """dataset_base.py:381-385 on the ego-frame list [origin, wps...]: cumulative path length as (distance, 0)."""
    full = torch.cat([torch.zeros(wps.shape[0], 1, 2), wps], 1)
    arc = torch.cumsum((full[:, 1:] - full[:, :-1]).norm(dim=-1), 1)
    return torch.stack([arc, torch.zeros_like(arc)], -1)


def make_base_batch(cfg: BaseConfig, B: int, seed: int = 0) -> DrivingExample:
    """Anyres patches drawn in the CLIP-normalised distribution of uint8 frames; speed U(0, 15) m/s; target
    points N(0, 10) m; labels: route = cumsum((1,0) + N(0, 0.1)), waypoints = cumsum(N((0.8,0), 0.3))."""
    g = torch.Generator().manual_seed(seed)
    H = cfg.img_size
    u = torch.rand((B, 1, 1, cfg.npatch, 3, H, H), generator=g)
    mean = torch.tensor(CLIP_MEAN).view(1, 1, 1, 1, 3, 1, 1)
    std = torch.tensor(CLIP_STD).view(1, 1, 1, 1, 3, 1, 1)
    pix = ((u - mean) / std).float()
    speed = torch.rand((B, 1), generator=g) * 15.0
    tp = torch.randn((B, cfg.n_tp, 2), generator=g) * 10.0
    route = torch.cumsum(torch.tensor([1.0, 0.0]) + 0.1 * torch.randn((B, cfg.n_route, 2), generator=g), 1)
    wps = torch.cumsum(torch.tensor([0.8, 0.0]) + 0.3 * torch.randn((B, 11, 2), generator=g), 1)
    from .collate import camera_extrinsics, camera_intrinsics, encode_uint8
    di = DrivingInput(camera_images=pix, image_sizes=torch.tensor([[cfg.frame_h, cfg.frame_w]] * B),
                      camera_intrinsics=camera_intrinsics(cfg.frame_w, cfg.frame_h, 110).expand(B, 1, 3, 3).contiguous(),
                      camera_extrinsics=camera_extrinsics().expand(B, 1, 4, 4).contiguous(),
                      vehicle_speed=speed, map_route=tp, target_point=tp[:, 0].clone())
    dl = DrivingLabel(time_delta_sec=torch.linspace(0.2, 2.2, 11).repeat(B, 1), waypoints=wps,
                      waypoints_1d=_waypoints_1d(wps), route_adjusted=route)
    return DrivingExample(driving_input=di, driving_label=dl,
                          run_id=encode_uint8([f"synthetic-{seed}-{b}" for b in range(B)], 1000),
                          timestamp=torch.zeros(B))
