"""Shared helpers for the collate image-path tests (tests/golden/frames.npz, oracle/gen_golden_frames.py)."""
import hashlib
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.npz")
# name: (W0, H0, cut_bottom, max_num_grid, seed) — must match oracle/gen_golden_frames.py
CASES = {
    "carla_1024x512": (1024, 512, True, 2, 0),
    "uncropped_1024x512": (1024, 512, False, 2, 1),
    "small_300x200": (300, 200, False, 2, 2),
    "exact_896x448": (896, 448, False, 2, 3),
    "down_2000x900": (2000, 900, False, 2, 4),
    "tall_37x23_max4": (23, 37, False, 4, 5),
}


def golden():
    return np.load(GOLDEN, allow_pickle=False)


def frame(W, H, seed):
    return np.random.default_rng(seed).integers(0, 256, (H, W, 3), dtype=np.uint8)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
