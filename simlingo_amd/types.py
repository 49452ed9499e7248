"""Batch / output schema — field-for-field mirror of the reference's NamedTuples
(simlingo_training/utils/custom_types.py:5-64), the data contract of the drop-in surface."""
from __future__ import annotations

from typing import Dict, List, NamedTuple, Optional, Tuple

import torch
from torch import Tensor


class LanguageLabel(NamedTuple):  # custom_types.py:21-27
    phrase_ids: Tensor            # [B, L] int64
    phrase_valid: Tensor          # [B, L] bool, true => fed into the model
    phrase_mask: Tensor           # [B, L] bool
    placeholder_values: list      # per sample {token_id: ndarray[n, 2]}
    language_string: list
    loss_masking: Tensor          # [B, L] bool, true => takes part in the loss


class TrainingOutput(NamedTuple):  # custom_types.py:35-41
    loss: Tensor
    loss_averages: Dict[str, Tensor]
    loss_values: Dict[str, Tensor]
    loss_counts: Dict[str, Tensor]
    driving_output: Optional[object] = None


class DrivingInput(NamedTuple):  # custom_types.py:43-51
    camera_images: Tensor         # [B, T=1, N=2, 3, 448, 448] f32, normalised tiles
    image_sizes: Tensor
    camera_intrinsics: Tensor
    camera_extrinsics: Tensor
    vehicle_speed: Tensor
    target_point: Tensor
    prompt: LanguageLabel
    prompt_inference: LanguageLabel


class DrivingLabel(NamedTuple):  # custom_types.py:53-58
    waypoints: Tensor             # [B, F, 2] speed waypoints
    path: Tensor                  # [B, 20, 2] route
    answer: LanguageLabel
    image_ff_org: Tensor
    eval_infos: Optional[Dict] = None


class DrivingExample(NamedTuple):  # custom_types.py:60-64
    driving_input: DrivingInput
    driving_label: DrivingLabel
    run_id: List[str]
    qa_templates: Optional[Tuple[str, str]] = None
