"""Collate image path on the MI355X: uint8 camera frames -> InternVL2 pixel tiles.

Mirrors `preprocess_image_batch` (simlingo_training/utils/internvl2_utils.py:179-203) and the bottom crop the
dataset applies before it (dataloader/dataset_base.py:464-467): same arguments (`input_size`, `max_num_grid`,
`use_global_img`), same outputs (`{"pixel_values": [B, tiles, 3, 448, 448] f32, "image_sizes": [B, 2]}`), but the
frames stay uint8 until they are on the GPU (1.1 MB per 1024x359 frame crosses PCIe instead of 4.8 MB of f32
tiles) and the Pillow resize + ToTensor + Normalize run as one HIP kernel (csrc/frames.hip) that reproduces
Pillow's bicubic resample bit for bit. The grid choice (dynamic_preprocess, internvl2_utils.py:231-266) is host
logic and is restated here.

`FramePipeline` adds the H2D half: pinned staging buffers, a copy stream and events, so batch i+1's frames
upload while batch i trains (SURVEY.md §8f row 1 "pinned double-buffering").
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from . import kernels as K

IMAGENET_MEAN = (0.485, 0.456, 0.406)   # internvl2_utils.py:17-18
IMAGENET_STD = (0.229, 0.224, 0.225)


class FrameDesc(ctypes.Structure):  # include/slx.h slx_frame_desc
    _fields_ = [("src", ctypes.c_void_p), ("sb", ctypes.c_int64), ("sy", ctypes.c_int64), ("sx", ctypes.c_int64),
                ("sc", ctypes.c_int64), ("B", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("tw", ctypes.c_int), ("th", ctypes.c_int), ("tile", ctypes.c_int),
                ("hbounds", ctypes.c_void_p), ("hcoeffs", ctypes.c_void_p), ("hksize", ctypes.c_int),
                ("vbounds", ctypes.c_void_p), ("vcoeffs", ctypes.c_void_p), ("vksize", ctypes.c_int),
                ("need_h", ctypes.c_int), ("need_v", ctypes.c_int), ("rows_per_block", ctypes.c_int),
                ("cols_per_block", ctypes.c_int), ("lds_rows", ctypes.c_int), ("lds_cols", ctypes.c_int), ("mean", ctypes.c_float * 3), ("std", ctypes.c_float * 3),
                ("out", ctypes.c_void_p)]


_i32p = ctypes.POINTER(ctypes.c_int32)
K.register("slx_frames_to_tiles", [ctypes.POINTER(FrameDesc), ctypes.c_void_p])
K.register("slx_resample_coeffs", [ctypes.c_int, ctypes.c_int, ctypes.c_int, _i32p, _i32p])
K.register("slx_resample_ksize", [ctypes.c_int, ctypes.c_int])


def bottom_crop_rows(H: int) -> int:
    """Rows kept by `cut_bottom_quarter` (dataset_base.py:466): H - (H * 4.8) // 16 (float floor division)."""
    return int(H - (H * 4.8) // 16)


def closest_grid(width: int, height: int, min_num: int = 1, max_num: int = 12, image_size: int = 448):
    """dynamic_preprocess's grid choice (internvl2_utils.py:231-249 with find_closest_aspect_ratio :216-229):
    candidate (cols, rows) with min_num <= cols*rows <= max_num, ordered by tile count; the closest aspect ratio
    wins, a tie goes to the later candidate when the image area exceeds half the candidate's pixel area."""
    aspect = width / height
    cands = set((i, j) for n in range(min_num, max_num + 1) for i in range(1, n + 1) for j in range(1, n + 1)
                if min_num <= i * j <= max_num)
    cands = sorted(cands, key=lambda r: r[0] * r[1])
    best, best_diff = (1, 1), float("inf")
    area = width * height
    for r in cands:
        diff = abs(aspect - r[0] / r[1])
        if diff < best_diff:
            best, best_diff = r, diff
        elif diff == best_diff and area > 0.5 * image_size * image_size * r[0] * r[1]:
            best = r
    return best


def resample_coeffs(in_size: int, out_size: int):
    """Pillow's bicubic coefficient tables for one axis via the C-ABI host function: (bounds [out, 2], kk [out, k])."""
    k = K.lib().slx_resample_ksize(in_size, out_size)
    if k <= 0:
        raise RuntimeError(f"slx_resample_ksize({in_size}, {out_size}) failed")
    bounds = np.zeros((out_size, 2), dtype=np.int32)
    kk = np.zeros((out_size, k), dtype=np.int32)
    rc = K.lib().slx_resample_coeffs(in_size, out_size, k, bounds.ctypes.data_as(_i32p), kk.ctypes.data_as(_i32p))
    if rc != k:
        K.check(rc if rc < 0 else -1, "slx_resample_coeffs")
    # the kernel derives each block's source window from its first and last output: both ends must be monotone
    if not (np.all(np.diff(bounds[:, 0]) >= 0) and np.all(np.diff(bounds[:, 0] + bounds[:, 1]) >= 0)):
        raise RuntimeError(f"resample bounds {in_size}->{out_size} are not monotone")
    return bounds, kk


class FramePreprocessor:
    """preprocess_image_batch for one frame geometry on the GPU.

    frames: uint8 [B, H0, W0, 3] (HWC, as cv2/PIL decode them) or [B, 3, H0, W0] (channels_first=True, the layout
    the reference collate hands to preprocess_image_batch), any element strides, on the device. H0 rows are cut to
    bottom_crop_rows(H0) when `cut_bottom` (the dataset's `cut_bottom_quarter`)."""

    def __init__(self, H0: int, W0: int, device, input_size: int = 448, max_num_grid: int = 2,
                 use_global_img: bool = False, cut_bottom: bool = True, rows_per_block: int = 16,
                 cols_per_block: int = 128):
        if use_global_img:
            raise NotImplementedError("use_global_img (thumbnail tile) is off in every simlingo config "
                                      "(datamodule.py:349 use_global_img=False)")
        self.device = torch.device(device)
        self.H0, self.W0 = H0, W0
        self.H = bottom_crop_rows(H0) if cut_bottom else H0
        self.W = W0
        self.tile = input_size
        cols, rows = closest_grid(self.W, self.H, 1, max_num_grid, input_size)
        self.grid = (cols, rows)
        self.tw, self.th = input_size * cols, input_size * rows
        self.tiles = cols * rows
        self.need_h = int(self.tw != self.W)
        self.need_v = int(self.th != self.H)
        dev = self.device
        z = torch.zeros(2, dtype=torch.int32, device=dev)
        if self.need_h:
            hb, hk = resample_coeffs(self.W, self.tw)
            self.hb, self.hk = torch.from_numpy(hb).to(dev), torch.from_numpy(hk).to(dev)
        else:
            hb = hk = None
            self.hb, self.hk = z, z
        if self.need_v:
            vb, vk = resample_coeffs(self.H, self.th)
            self.vb, self.vk = torch.from_numpy(vb).to(dev), torch.from_numpy(vk).to(dev)
        else:
            vb = vk = None
            self.vb, self.vk = z, z
        # block = rows_per_block x cols_per_block outputs; its source window = the largest row / column span any
        # block reads; halve the block until window + horizontal-pass buffer fit 64 KiB of LDS
        def span(bounds, n_out, step):
            if bounds is None:
                return min(step, n_out)
            return max(int((bounds[o:o + step, 0] + bounds[o:o + step, 1]).max() - bounds[o, 0])
                       for o in range(0, n_out, step))

        ry, cw = rows_per_block, cols_per_block
        while True:
            lr, lc = span(vb, self.th, ry), span(hb, self.tw, cw)
            lds = lr * (lc * 3 + 4) + lr * cw * 3 + 4 * (cw * (hk.shape[1] + 2 if hb is not None else 2)
                                                          + ry * (vk.shape[1] + 2 if vb is not None else 2))
            if lds <= 64 * 1024 or ry == 1:
                break
            ry //= 2  # the kernel fixes 128 output columns per block; only the row count shrinks
        if lds > 64 * 1024:
            raise ValueError(f"frame geometry {W0}x{H0} -> {self.tw}x{self.th} needs {lds} B of LDS per block")
        self.rows_per_block, self.cols_per_block, self.lds_rows, self.lds_cols = ry, cw, lr, lc
        self._desc_cache = {}
        self.mean = [float(np.float32(m)) for m in IMAGENET_MEAN]
        self.std = [float(np.float32(s)) for s in IMAGENET_STD]

    def image_sizes(self, B: int) -> torch.Tensor:
        """[B, 2] = (height, width) of the cropped frame (preprocess_image_batch :197)."""
        return torch.tensor([[self.H, self.W]] * B, dtype=torch.int64)

    def __call__(self, frames: torch.Tensor, out: torch.Tensor | None = None, channels_first: bool = False):
        """-> pixel_values [B, tiles, 3, tile, tile] f32 on the device (the caller views it as [B, T=1, ...])."""
        if frames.device != self.device or frames.dtype != torch.uint8:
            raise RuntimeError("FramePreprocessor expects uint8 frames already on its device")
        if channels_first:
            B, C, H0, W0 = frames.shape
            sb, sc, sy, sx = frames.stride()
        else:
            B, H0, W0, C = frames.shape
            sb, sy, sx, sc = frames.stride()
        if (H0, W0, C) != (self.H0, self.W0, 3):
            raise ValueError(f"frames {tuple(frames.shape)} do not match the configured {self.W0}x{self.H0} RGB")
        if out is None:
            out = torch.empty(B, self.tiles, 3, self.tile, self.tile, dtype=torch.float32, device=self.device)
        elif out.dtype != torch.float32 or not out.is_contiguous() or out.numel() != B * self.tiles * 3 * self.tile ** 2:
            raise ValueError("out must be a contiguous f32 [B, tiles, 3, tile, tile] buffer")
        key = (frames.data_ptr(), sb, sy, sx, sc, B, out.data_ptr())
        d = self._desc_cache.get(key)
        if d is None:  # the descriptor is rebuilt only when the buffers change (steady state: ctypes call only)
            d = FrameDesc()
            d.src, d.sb, d.sy, d.sx, d.sc = frames.data_ptr(), sb, sy, sx, sc
            d.B, d.H, d.W = B, self.H, self.W
            d.tw, d.th, d.tile = self.tw, self.th, self.tile
            d.hbounds, d.hcoeffs = self.hb.data_ptr(), self.hk.data_ptr()
            d.hksize = self.hk.shape[-1] if self.need_h else 0
            d.vbounds, d.vcoeffs = self.vb.data_ptr(), self.vk.data_ptr()
            d.vksize = self.vk.shape[-1] if self.need_v else 0
            d.need_h, d.need_v = self.need_h, self.need_v
            d.rows_per_block, d.cols_per_block = self.rows_per_block, self.cols_per_block
            d.lds_rows, d.lds_cols = self.lds_rows, self.lds_cols
            d.mean[:] = self.mean
            d.std[:] = self.std
            d.out = out.data_ptr()
            if len(self._desc_cache) > 16:
                self._desc_cache.clear()
            self._desc_cache[key] = d
        K.check(K.lib().slx_frames_to_tiles(ctypes.byref(d), K.stream_ptr()), "slx_frames_to_tiles")
        return out


def preprocess_image_batch(frames: torch.Tensor, input_size: int = 448, use_global_img: bool = False,
                           max_num_grid: int = 2, cut_bottom: bool = False, channels_first: bool = True):
    """Drop-in for internvl2_utils.preprocess_image_batch on a device tensor of uint8 frames [B, 3, H, W]
    (the reference passes a list of [3, H, W] tensors holding uint8 values, internvl2_utils.py:186-190).
    Returns {"pixel_values": [B, tiles, 3, s, s] f32 (device), "image_sizes": [B, 2]}."""
    if channels_first:
        B, _, H0, W0 = frames.shape
    else:
        B, H0, W0, _ = frames.shape
    pre = FramePreprocessor(H0, W0, frames.device, input_size, max_num_grid, use_global_img, cut_bottom)
    return {"pixel_values": pre(frames, channels_first=channels_first), "image_sizes": pre.image_sizes(B)}


class FramePipeline:
    """Double-buffered host -> HBM upload of uint8 frames + the tiling kernel.

    put(frames_np [B, H0, W0, 3] uint8) copies into a pinned slot and enqueues the H2D on a side stream; get()
    makes the current stream wait for that upload and returns the [B, 1, tiles, 3, 448, 448] pixel tiles. With
    depth 2, batch i+1 uploads while batch i computes."""

    def __init__(self, B: int, H0: int, W0: int, device, depth: int = 2, **kw):
        self.pre = FramePreprocessor(H0, W0, device, **kw)
        self.B, self.depth = B, depth
        dev = self.pre.device
        self.host = [torch.empty(B, H0, W0, 3, dtype=torch.uint8).pin_memory() for _ in range(depth)]
        self.dev = [torch.empty(B, H0, W0, 3, dtype=torch.uint8, device=dev) for _ in range(depth)]
        self.out = [torch.empty(B, 1, self.pre.tiles, 3, self.pre.tile, self.pre.tile, dtype=torch.float32,
                                device=dev) for _ in range(depth)]
        self.copy_stream = torch.cuda.Stream(device=dev)
        # the device slots come from the current stream's pool (possibly memory its queued kernels still use): the
        # copy stream's first writes wait for the work enqueued so far (see FrameUploader)
        self.copy_stream.wait_stream(torch.cuda.current_stream(dev))
        self.ready = [torch.cuda.Event() for _ in range(depth)]
        self.consumed = [torch.cuda.Event() for _ in range(depth)]
        self.put_i = self.get_i = 0

    def put(self, frames) -> None:
        s = self.put_i % self.depth
        if self.put_i - self.get_i >= self.depth:
            raise RuntimeError("FramePipeline: more batches in flight than buffers (call get() first)")
        self.consumed[s].synchronize()  # the kernel that last read this slot has finished
        src = torch.from_numpy(np.ascontiguousarray(frames)) if isinstance(frames, np.ndarray) else frames
        self.host[s].copy_(src)
        with torch.cuda.stream(self.copy_stream):
            self.dev[s].copy_(self.host[s], non_blocking=True)
            self.ready[s].record(self.copy_stream)
        self.put_i += 1

    def get(self):
        if self.get_i >= self.put_i:
            raise RuntimeError("FramePipeline: get() without a pending put()")
        s = self.get_i % self.depth
        cur = torch.cuda.current_stream(self.pre.device)
        cur.wait_event(self.ready[s])
        out = self.out[s]
        self.pre(self.dev[s], out=out.view(self.B, self.pre.tiles, 3, self.pre.tile, self.pre.tile))
        self.consumed[s].record(cur)
        self.get_i += 1
        return out, self.pre.image_sizes(self.B)


class FrameUploader:
    """uint8 frames host -> HBM through a ring of (pinned slot, device slot) pairs, the copy on a side stream.

    __call__(frames) copies the stacked uint8 frames into a pinned slot, enqueues the H2D on the copy
    stream and makes the current stream wait for it; `release(t)` (called by the consumer after the kernel that reads
    the device slot was enqueued) records when the slot may be overwritten. The host never waits on the GPU except when
    a slot is still in use `depth` batches later. Collate's default image path."""

    def __init__(self, device, depth: int = 3):
        self.device = torch.device(device)
        self.depth = depth
        self.slots = [None] * depth      # (shape, pinned, device)
        self.copied = [None] * depth     # event: the H2D that last read the pinned slot is done
        self.consumed = [None] * depth   # event: the kernel that last read the device slot is done
        self.i = 0
        self.copy_stream = torch.cuda.Stream(device=self.device)

    def __call__(self, frames) -> torch.Tensor:
        """frames: uint8 host tensor / array [B, ...] -> the device slot holding a copy (the current stream waits)."""
        frames = torch.as_tensor(frames)
        shape = tuple(frames.shape)
        s = self.i % self.depth
        self.i += 1
        for ev in (self.copied[s], self.consumed[s]):
            if ev is not None:
                ev.synchronize()
        cur = torch.cuda.current_stream(self.device)
        if self.slots[s] is None or self.slots[s][0] != shape:
            self.slots[s] = (shape, torch.empty(shape, dtype=torch.uint8).pin_memory(),
                             torch.empty(shape, dtype=torch.uint8, device=self.device))
            # the caching allocator hands out blocks in the CURRENT stream's order: the new device slot may be memory
            # the current stream freed while kernels still queued on it read or write it. The copy stream is not
            # ordered after those kernels, so its first write into the slot waits for everything enqueued so far.
            self.copy_stream.wait_stream(cur)
        _, host, dev = self.slots[s]
        host.copy_(frames)
        with torch.cuda.stream(self.copy_stream):
            dev.copy_(host, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.copy_stream)
        self.copied[s] = ev
        cur.wait_event(ev)
        self._last = s
        return dev

    def release(self):
        """The current stream's work enqueued so far (the tiling kernel) is the last reader of the newest slot."""
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        self.consumed[self._last] = ev


def algorithmic_bytes(pre: FramePreprocessor, B: int) -> int:
    """HBM bytes one launch must move: the cropped uint8 frames once + the f32 tiles once."""
    return B * (pre.H * pre.W * 3 + pre.tiles * 3 * pre.tile * pre.tile * 4)


__all__ = ["FramePreprocessor", "FramePipeline", "FrameUploader", "preprocess_image_batch", "bottom_crop_rows", "closest_grid",
           "resample_coeffs", "algorithmic_bytes"]
