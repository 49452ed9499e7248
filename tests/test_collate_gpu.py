"""Collate with the HIP frame kernel feeding the drop-in DrivingModel (tiny geometry): uint8 frames + conversations ->
DrivingExample (tiles from slx_frames_to_tiles) -> training_step on the engine, held to the oracle's loss on the same
collated batch (rel 1e-2, the tiny bf16 gate of test_vla_parity_gpu.py)."""
import numpy as np
import pytest
import torch

from chat_util import build_tokenizer
from oracle import vla_oracle as O
from test_collate_cpu import _samples
from test_vla_parity_gpu import engine_precision_params

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::UserWarning")]


def test_collate_frames_to_training_step(dev):
    from simlingo_amd.collate import Collate
    from simlingo_amd.config import tiny_config
    from simlingo_amd.driving import DrivingModel
    from simlingo_amd.params import init_params
    cfg = tiny_config()
    col = Collate(build_tokenizer(), num_image_tokens_per_patch=cfg.img_tokens_per_tile, num_image_patches=cfg.tiles,
                  device=dev, input_size=cfg.img_size)
    ex = col(_samples(cfg, 4))
    pix = ex.driving_input.camera_images
    assert pix.is_cuda and pix.shape == (4, 1, cfg.tiles, 3, cfg.img_size, cfg.img_size) and torch.isfinite(pix).all()
    P = init_params(cfg, seed=3, lora_b_std=0.05, std=0.05)
    m = DrivingModel(vision_model={"variant": "tiny"}, language_model={"variant": "tiny", "lora_dropout": 0.0},
                     init_params=P)
    m.build_engine(dev)
    out = m.training_step(ex, 0)
    exc = ex._replace(driving_input=ex.driving_input._replace(camera_images=pix.cpu()))
    ref, _ = O.loss_and_grads(engine_precision_params(m.engine, P), cfg, exc)
    np.testing.assert_allclose(out["loss"].item(), ref["loss"].item(), rtol=1e-2)
