"""CPU oracle of the collate image path. TEST INFRASTRUCTURE ONLY — imported by tests/,
__graft_entry__.smoke() and tools/frame_bench.py's cpu_baseline leg, never by the product path.

Reference chain (simlingo_training):
  dataset_base.py:464-467      bottom crop: rows [0, int(H - (H*4.8)//16))
  internvl2_utils.py:179-203   preprocess_image_batch: uint8 HWC -> PIL image -> dynamic_preprocess -> transform
  internvl2_utils.py:231-266   dynamic_preprocess: grid choice, image.resize((tw, th)), 448-tile crops
  internvl2_utils.py:206-214   build_transform: Resize((448, 448), BICUBIC) [identity on a 448 tile], ToTensor,
                               Normalize(IMAGENET_MEAN, IMAGENET_STD)

The arithmetic lives in third-party code: Pillow's Image.resize (pinned pillow==10.2.0, environment.yaml:187;
Pillow 12.2.0 here — the Resample.c algorithm is the same) and torchvision's ToTensor/Normalize (pinned
torchvision==0.17.0, environment.yaml:259; absent here). `preprocess_image_batch` below runs the real Pillow
for the resize and restates ToTensor/Normalize with the same torch f32 ops torchvision uses
(`img.float().div(255)`, `sub_(mean).div_(std)`). `pil_resample_coeffs` / `pil_resize_bicubic` restate Pillow's
ImagingResample (precompute_coeffs, normalize_coeffs_8bpc, ImagingResampleHorizontal/Vertical_8bpc) in numpy and
are pinned against the installed Pillow bit for bit (tests/test_frames_cpu.py). The reference module itself
(internvl2_utils) cannot be imported here (torchvision is absent), so parity is anchored on the
restatement of its call sites + the real Pillow + the fixtures of tests/golden/frames.npz
(oracle/gen_golden_frames.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch

PRECISION_BITS = 32 - 8 - 2
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def bottom_crop(frame_hwc: np.ndarray) -> np.ndarray:  # dataset_base.py:466
    H = frame_hwc.shape[0]
    return frame_hwc[:int(H - (H * 4.8) // 16)]


# ---- Pillow Resample.c restatement (BICUBIC, box = whole image) ------------------------------------------------
def _bicubic(x: float) -> float:
    a = -0.5
    x = abs(x)
    if x < 1.0:
        return ((a + 2.0) * x - (a + 3.0)) * x * x + 1
    if x < 2.0:
        return (((x - 5) * x + 8) * x - 4) * a
    return 0.0


def pil_resample_coeffs(in_size: int, out_size: int):
    """precompute_coeffs + normalize_coeffs_8bpc -> (bounds [out, 2] int32, kk [out, ksize] int32)."""
    scale = in_size / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    bounds = np.zeros((out_size, 2), np.int32)
    kk = np.zeros((out_size, ksize), np.int32)
    for xx in range(out_size):
        center = 0.0 + (xx + 0.5) * scale
        ss = 1.0 / filterscale
        xmin = max(int(center - support + 0.5), 0)
        xmax = min(int(center + support + 0.5), in_size) - xmin
        k = [_bicubic((x + xmin - center + 0.5) * ss) for x in range(xmax)]
        ww = 0.0
        for w in k:
            ww += w
        if ww != 0.0:
            k = [w / ww for w in k]
        bounds[xx] = (xmin, xmax)
        for x, w in enumerate(k):
            kk[xx, x] = int(-0.5 + w * (1 << PRECISION_BITS)) if w < 0 else int(0.5 + w * (1 << PRECISION_BITS))
    return bounds, kk


def _pass(img: np.ndarray, bounds, kk, axis: int) -> np.ndarray:
    """One 8-bpc pass along `axis` (1 = horizontal over columns, 0 = vertical over rows), int32 math + clip8."""
    x = np.moveaxis(img.astype(np.int64), axis, 0)          # [in, other, 3]
    out = np.empty((bounds.shape[0],) + x.shape[1:], np.int64)
    for o in range(bounds.shape[0]):
        lo, n = int(bounds[o, 0]), int(bounds[o, 1])
        s = (1 << (PRECISION_BITS - 1)) + np.tensordot(kk[o, :n].astype(np.int64), x[lo:lo + n], axes=(0, 0))
        s = s.astype(np.int32).astype(np.int64)  # Pillow accumulates in a C int
        out[o] = np.where(s >= (1 << PRECISION_BITS << 8), 255, np.where(s <= 0, 0, s >> PRECISION_BITS))
    return np.moveaxis(out, 0, axis).astype(np.uint8)


def pil_resize_bicubic(img_hwc: np.ndarray, tw: int, th: int) -> np.ndarray:
    """ImagingResampleInner: horizontal pass (rows the vertical pass needs) then vertical; a pass whose axis keeps
    its size is skipped entirely (no rounding)."""
    H, W, _ = img_hwc.shape
    x = img_hwc
    if tw != W:
        b, k = pil_resample_coeffs(W, tw)
        x = _pass(x, b, k, 1)
    if th != H:
        b, k = pil_resample_coeffs(H, th)
        x = _pass(x, b, k, 0)
    return x


# ---- the reference chain with the real Pillow -------------------------------------------------------------------
def closest_grid(width, height, min_num=1, max_num=12, image_size=448):
    """find_closest_aspect_ratio + the candidate list of dynamic_preprocess (internvl2_utils.py:216-244)."""
    aspect = width / height
    ratios = set((i, j) for n in range(min_num, max_num + 1) for i in range(1, n + 1) for j in range(1, n + 1)
                 if i * j <= max_num and i * j >= min_num)
    ratios = sorted(ratios, key=lambda x: x[0] * x[1])
    best_diff, best = float("inf"), (1, 1)
    area = width * height
    for r in ratios:
        d = abs(aspect - r[0] / r[1])
        if d < best_diff:
            best_diff, best = d, r
        elif d == best_diff and area > 0.5 * image_size * image_size * r[0] * r[1]:
            best = r
    return best


def dynamic_preprocess_u8(img_hwc: np.ndarray, image_size=448, max_num=2, resize=None):
    """-> (resized uint8 [th, tw, 3], list of uint8 tiles). resize(img, tw, th) defaults to Pillow's Image.resize."""
    from PIL import Image
    H, W, _ = img_hwc.shape
    cols, rows = closest_grid(W, H, 1, max_num, image_size)
    tw, th = image_size * cols, image_size * rows
    if resize is None:
        resized = np.asarray(Image.fromarray(img_hwc).resize((tw, th)))
    else:
        resized = resize(img_hwc, tw, th)
    tiles = []
    for i in range(cols * rows):
        c, r = i % (tw // image_size), i // (tw // image_size)
        tiles.append(resized[r * image_size:(r + 1) * image_size, c * image_size:(c + 1) * image_size])
    return resized, tiles


def to_tensor_normalize(tile_u8: np.ndarray) -> torch.Tensor:
    """ToTensor + Normalize exactly as torchvision 0.17 computes them on a uint8 PIL image."""
    t = torch.from_numpy(np.array(tile_u8, copy=True)).permute(2, 0, 1).contiguous().to(torch.float32).div(255)
    mean = torch.as_tensor(IMAGENET_MEAN, dtype=torch.float32)[:, None, None]
    std = torch.as_tensor(IMAGENET_STD, dtype=torch.float32)[:, None, None]
    return t.sub_(mean).div_(std)


def preprocess_image_batch(frames_hwc, input_size=448, max_num_grid=2, cut_bottom=True, resize=None):
    """frames: iterable of uint8 [H, W, 3] -> {"pixel_values": [B, tiles, 3, s, s] f32, "image_sizes": [B, 2],
    "resized": list of uint8 [th, tw, 3]}."""
    pv, sizes, resized = [], [], []
    for f in frames_hwc:
        f = bottom_crop(np.asarray(f)) if cut_bottom else np.asarray(f)
        f = np.ascontiguousarray(f)
        r, tiles = dynamic_preprocess_u8(f, input_size, max_num_grid, resize)
        pv.append(torch.stack([to_tensor_normalize(t) for t in tiles]))
        sizes.append([f.shape[0], f.shape[1]])
        resized.append(r)
    return {"pixel_values": torch.stack(pv), "image_sizes": torch.tensor(sizes), "resized": resized}
