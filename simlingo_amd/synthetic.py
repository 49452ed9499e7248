"""Seeded synthetic batches of the reference's shape (SURVEY.md §8d "Synthetic inputs").

There is no dataset or tokenizer offline; token ids are drawn around the fixed InternVL2 prompt
skeleton: text, <img>, img_tokens x <IMG_CONTEXT>, </img>, text with two consecutive <TARGET_POINT>
placeholders (coords N(0, 10) m, shape [2, 2]), text. The tokenizer is left-padded
(datamodule.py:138), so padded samples carry invalid tokens at the front.
"""
from __future__ import annotations

import numpy as np
import torch

from .config import VLAConfig
from .types import DrivingExample, DrivingInput, DrivingLabel, LanguageLabel

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def make_batch(cfg: VLAConfig, B: int, s_text: int, n_loss: int, seed: int = 0, pad: list[int] | None = None,
               device: str | torch.device = "cpu") -> DrivingExample:
    """B samples; each language sequence has L = s_text + img_tokens positions; the last `n_loss`
    tokens of every sample take part in the LM loss; pad[b] leading positions of sample b are padding."""
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    nimg = cfg.img_tokens
    L = s_text + nimg
    pad = pad or [0] * B
    text_hi = min(cfg.pad_id, cfg.vocab)  # ordinary text ids stay below the special tokens
    ids = np.zeros((B, L), dtype=np.int64)
    valid = np.ones((B, L), dtype=bool)
    loss_mask = np.zeros((B, L), dtype=bool)
    placeholders = []
    for b in range(B):
        p = pad[b]
        seq = list(rng.integers(0, text_hi, size=4))
        seq += [cfg.img_start_id] + [cfg.img_context_id] * nimg + [cfg.img_end_id]
        n_rest = L - p - len(seq)
        assert n_rest >= 8, "s_text too small for the prompt skeleton"
        tail = list(rng.integers(0, text_hi, size=n_rest))
        tp = max(0, min(3, n_rest - n_loss - 3))  # keep the placeholders out of the loss span
        tail[tp] = cfg.target_point_id
        tail[tp + 1] = cfg.target_point_id
        seq += tail
        ids[b, :p] = cfg.pad_id
        valid[b, :p] = False
        ids[b, p:] = np.asarray(seq)
        nl = min(n_loss, L - p - 1)
        loss_mask[b, L - nl:] = True
        placeholders.append({cfg.target_point_id: rng.normal(0.0, 10.0, size=(2, 2)).astype(np.float32)})
    prompt = LanguageLabel(
        phrase_ids=torch.from_numpy(ids), phrase_valid=torch.from_numpy(valid),
        phrase_mask=torch.from_numpy(valid.copy()), placeholder_values=placeholders,
        language_string=[""] * B, loss_masking=torch.from_numpy(loss_mask))
    # pixel tiles directly in the ImageNet-normalised distribution of uint8 uniform frames
    H = cfg.img_size
    u = torch.rand((B, 1, cfg.tiles, 3, H, H), generator=g)
    mean = torch.tensor(IMAGENET_MEAN).view(1, 1, 1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 1, 1, 3, 1, 1)
    pix = ((u - mean) / std).float()
    route = torch.cumsum(torch.tensor([1.0, 0.0]) + 0.1 * torch.randn((B, cfg.n_route, 2), generator=g), 1)
    speed = torch.cumsum(torch.tensor([0.8, 0.0]) + 0.3 * torch.randn((B, cfg.n_speed, cfg.speed_dims), generator=g), 1)
    di = DrivingInput(
        camera_images=pix.to(device), image_sizes=torch.tensor([[H * cfg.tiles, H]] * B),
        camera_intrinsics=torch.eye(3).repeat(B, 1, 1), camera_extrinsics=torch.eye(4).repeat(B, 1, 1),
        vehicle_speed=torch.zeros(B, 1), target_point=torch.zeros(B, 2), prompt=prompt, prompt_inference=prompt)
    dl = DrivingLabel(waypoints=speed.float().to(device), path=route.float().to(device), answer=None,
                      image_ff_org=torch.zeros(B, 2))
    return DrivingExample(driving_input=di, driving_label=dl, run_id=[f"synthetic-{seed}-{b}" for b in range(B)])
