"""Rebuild the SimLingo-Base golden cases (tests/golden/base_tiny.npz, base_full1.npz, made by
oracle/gen_golden_base.py)."""
import os

import numpy as np
import torch

from simlingo_amd.base_config import base_config, base_tiny_config
from simlingo_amd.base_params import init_base_params
from simlingo_amd.base_types import make_base_batch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# the cases oracle/gen_golden_base.py writes: tiny widths, and full1 (CLIP-L / 4096 projector / Llama-tiny widths,
# 1 used CLIP layer + 1 Llama layer)
CASES = {"tiny": (base_tiny_config, {}, "base_tiny.npz"),
         "full1": (base_config, dict(vit_layers=2, llm_layers=1), "base_full1.npz")}


def load_base_case(name: str = "tiny"):
    mk, kw, fname = CASES[name]
    z = np.load(os.path.join(GOLDEN, fname), allow_pickle=False)
    cfg = mk(**kw)
    seed, B = int(z["seed"]), int(z["B"])
    std = float(z["std"]) if "std" in z else 0.05
    P = init_base_params(cfg, seed=seed, std=std)
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
