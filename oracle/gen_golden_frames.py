"""Generate tests/golden/frames.npz: golden vectors of the collate image path.

Inputs are seeded uint8 frames (numpy default_rng(seed).integers(0, 256, (H, W, 3))), expected outputs come from
the reference chain with the real Pillow (oracle/frames_oracle.preprocess_image_batch): sha256 of the resized
uint8 image and of the f32 pixel tiles, 4096 sampled tile values, image_sizes, the tile grid, and Pillow's
coefficient tables for the production geometry (1024x359 -> 896x448). Test infrastructure only.

    python oracle/gen_golden_frames.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import frames_oracle as O  # noqa: E402

# name: (W0, H0, cut_bottom, max_num_grid, seed)
CASES = {
    "carla_1024x512": (1024, 512, True, 2, 0),     # the training frame: crop to 359 rows -> (2,1) grid
    "uncropped_1024x512": (1024, 512, False, 2, 1),
    "small_300x200": (300, 200, False, 2, 2),       # upsampling, (1,1) grid
    "exact_896x448": (896, 448, False, 2, 3),       # no resize pass at all
    "down_2000x900": (2000, 900, False, 2, 4),      # heavy downsampling (ksize 11)
    "tall_37x23_max4": (23, 37, False, 4, 5),       # portrait, (1,2) grid
}


def frame(W, H, seed):
    return np.random.default_rng(seed).integers(0, 256, (H, W, 3), dtype=np.uint8)


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out = {}
    for name, (W, H, cut, mx, seed) in CASES.items():
        f = frame(W, H, seed)
        r = O.preprocess_image_batch([f], 448, mx, cut)
        pv = r["pixel_values"][0].numpy()
        idx = np.random.default_rng(100 + seed).integers(0, pv.size, 4096)
        out[f"{name}.input_sha"] = np.array(sha(f))
        out[f"{name}.resized_sha"] = np.array(sha(r["resized"][0]))
        out[f"{name}.pixel_sha"] = np.array(sha(pv))
        out[f"{name}.pixel_shape"] = np.array(pv.shape)
        out[f"{name}.sample_idx"] = idx
        out[f"{name}.sample_val"] = pv.reshape(-1)[idx]
        out[f"{name}.image_sizes"] = r["image_sizes"].numpy()
        print(name, pv.shape, r["image_sizes"].tolist())
    for a, b in ((1024, 896), (359, 448)):
        bd, kk = O.pil_resample_coeffs(a, b)
        out[f"coeffs_{a}_{b}.bounds"] = bd
        out[f"coeffs_{a}_{b}.kk"] = kk
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "frames.npz"), **out)


if __name__ == "__main__":
    main()
