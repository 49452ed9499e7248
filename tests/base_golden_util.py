"""Rebuild the SimLingo-Base golden case (tests/golden/base_tiny.npz, made by oracle/gen_golden_base.py)."""
import os

import numpy as np
import torch

from simlingo_amd.base_config import base_tiny_config
from simlingo_amd.base_params import init_base_params
from simlingo_amd.base_types import make_base_batch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_base_case():
    z = np.load(os.path.join(GOLDEN, "base_tiny.npz"), allow_pickle=False)
    cfg = base_tiny_config()
    seed, B = int(z["seed"]), int(z["B"])
    P = init_base_params(cfg, seed=seed, std=0.05)
    for k, v in P.items():
        t = v.double()
        got = np.asarray([t.sum().item(), t.abs().sum().item(), t.pow(2).sum().item()])
        assert np.allclose(got, z["pc." + k], rtol=1e-9, atol=1e-9), f"param init drifted: {k}"
    ex = make_base_batch(cfg, B=B, seed=seed + 1)
    assert np.allclose(ex.driving_input.camera_images.double().sum().item(), z["in.pixel_sum"][0], rtol=1e-9)
    return cfg, P, ex, z


def ref_grad(z, name, g):
    """(reference entries, our entries at the same positions) for a gradient stored full or sampled."""
    g = g.reshape(-1)
    if "g." + name in z:
        return torch.from_numpy(z["g." + name]).reshape(-1), g
    idx = torch.from_numpy(z["gi." + name])
    return torch.from_numpy(z["gv." + name]), g[idx]
