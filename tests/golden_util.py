"""Helpers to rebuild the golden cases (tests/golden/vla_tiny_*.npz, made by oracle/gen_golden.py)."""
import os

import numpy as np
import torch

from simlingo_amd.config import tiny_config
from simlingo_amd.params import init_params
from simlingo_amd.types import DrivingExample, DrivingInput, DrivingLabel, LanguageLabel

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["nopad", "leftpad"]


def load_case(name):
    z = np.load(os.path.join(GOLDEN, f"vla_tiny_{name}.npz"), allow_pickle=False)
    cfg = tiny_config()
    P = init_params(cfg, seed=int(z["seed"]), lora_b_std=0.05, std=0.05)
    for k, v in P.items():  # the regenerated parameters must be the ones the fixture was made with
        t = v.double()
        got = np.asarray([t.sum().item(), t.abs().sum().item(), t.pow(2).sum().item()])
        assert np.allclose(got, z["pc." + k], rtol=1e-9, atol=1e-9), f"param init drifted: {k}"
    ids = torch.from_numpy(z["in.ids"])
    B = ids.shape[0]
    pv = [{cfg.target_point_id: z["in.tp_coords"][b]} for b in range(B)]
    lab = LanguageLabel(phrase_ids=ids, phrase_valid=torch.from_numpy(z["in.valid"]),
                        phrase_mask=torch.from_numpy(z["in.valid"]), placeholder_values=pv,
                        language_string=[""] * B, loss_masking=torch.from_numpy(z["in.loss_mask"]))
    di = DrivingInput(camera_images=torch.from_numpy(z["in.pixel"]), image_sizes=None, camera_intrinsics=None,
                      camera_extrinsics=None, vehicle_speed=None, target_point=None, prompt=lab, prompt_inference=lab)
    dl = DrivingLabel(waypoints=torch.from_numpy(z["in.waypoints"]), path=torch.from_numpy(z["in.path"]),
                      answer=None, image_ff_org=None)
    return cfg, P, DrivingExample(driving_input=di, driving_label=dl, run_id=[""] * B), z


def grad_entries(z, name):
    """(indices, values) of the reference gradient stored for `name` (full or sampled)."""
    if "g." + name in z:
        v = z["g." + name]
        return np.arange(v.size), v
    return z["gi." + name], z["gv." + name]
