"""Fixture for the SimLingo-Base collate (tests/golden/base_collate.npz) from transformers' own LLaVA-NeXT image
processor - ORACLE TOOLING, test infrastructure only; runs where transformers is installed:
    python oracle/gen_golden_base_collate.py

The reference's collate (simlingo_base_training/dataloader/datamodule.py:220-239) calls
LlavaNextProcessor.from_pretrained("llava-hf/llava-v1.6-mistral-7b-hf").image_processor(frames,
image_grid_pinpoints=[[336, 672]]); the hub config is unavailable offline, so the processor is built with that
checkpoint's published preprocessor settings (shortest_edge 336, crop 336, bicubic, CLIP mean / std; the installed
transformers falls back to its Pillow backend, the reference's pinned 4.46.3 default). Frames: seeded uniform uint8
1024 x 512 RGB cut to 359 rows (dataset_base.py:445), fed as [C, H, W] tensors like the collate. Stored: the frame
seeds and checksums, image_sizes, and per output patch a digest (sum / |sum| / sumsq, 4096 sampled values, two
whole rows per channel).
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from transformers import LlavaNextImageProcessor  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "base_collate.npz")


def frame(seed, H=512, W=1024):
    return np.random.default_rng(seed).integers(0, 256, size=(H, W, 3), dtype=np.uint8)


def main():
    proc = LlavaNextImageProcessor(size={"shortest_edge": 336}, crop_size={"height": 336, "width": 336},
                                   image_grid_pinpoints=[[336, 672], [672, 336], [672, 672], [1008, 336], [336, 1008]],
                                   resample=3, do_center_crop=True, do_pad=True)
    seeds = [5, 6]
    frames = []
    for s in seeds:
        f = frame(s)
        f = f[: int(f.shape[0] - (f.shape[0] * 4.8) // 16)]  # dataset_base.py:445
        frames.append(torch.from_numpy(np.ascontiguousarray(f.transpose(2, 0, 1))))
    out = proc(frames, return_tensors="pt", image_grid_pinpoints=[[336, 672]])
    pix = out["pixel_values"].numpy().astype(np.float32)  # [B, 1 + 2, 3, 336, 336]
    arrays = {"seeds": np.asarray(seeds), "image_sizes": out["image_sizes"].numpy(), "shape": np.asarray(pix.shape)}
    idx = np.random.default_rng(0).choice(pix[0, 0].size, 4096, replace=False)
    for b in range(pix.shape[0]):
        arrays[f"frame_cs.{b}"] = np.asarray([float(frames[b].double().sum()), float(frames[b].double().pow(2).sum())])
        for p in range(pix.shape[1]):
            t = pix[b, p].astype(np.float64)
            arrays[f"cs.{b}.{p}"] = np.asarray([t.sum(), np.abs(t).sum(), (t * t).sum()])
            arrays[f"v.{b}.{p}"] = pix[b, p].reshape(-1)[idx]
            arrays[f"rows.{b}.{p}"] = pix[b, p][:, [0, 50, 167, 285, 335], :]
    arrays["idx"] = idx.astype(np.int64)
    np.savez_compressed(OUT, **arrays)
    print(f"wrote {OUT}: pixel_values {pix.shape}, image_sizes {arrays['image_sizes'].tolist()}")


if __name__ == "__main__":
    main()
