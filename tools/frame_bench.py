"""Collate image path microbenchmark: B uint8 1024x512 frames resident in HBM ->
[B, 2, 3, 448, 448] f32 tiles (bottom crop, Pillow-exact bicubic 1024x359 -> 896x448, ToTensor, Normalize).

Prints one JSON line: kernel time with HIP events on the launch stream, algorithmic HBM bytes per launch
(cropped frames read once + tiles written once) and the fraction of the 8 TB/s HBM peak; the PCIe-inclusive
FramePipeline rate (pinned H2D of uint8 frames + kernel); and the CPU reference chain (real Pillow + torch
ToTensor/Normalize, oracle/frames_oracle.py) on one host thread per frame."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from simlingo_amd.frames import FramePipeline, FramePreprocessor, algorithmic_bytes  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--iters", type=int, default=50)
ap.add_argument("--cpu-frames", type=int, default=8)
a = ap.parse_args()
dev = torch.device("cuda:0")
B = a.batch
frames = np.random.default_rng(0).integers(0, 256, (B, 512, 1024, 3), dtype=np.uint8)
pre = FramePreprocessor(512, 1024, dev)
x = torch.from_numpy(frames).to(dev)
out = torch.empty(B, pre.tiles, 3, 448, 448, device=dev)
for _ in range(3):
    pre(x, out=out)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(a.iters):
    pre(x, out=out)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / a.iters
alg = algorithmic_bytes(pre, B)
gbs = alg / (ms * 1e-3) / 1e9
# PCIe-inclusive: pinned double-buffered pipeline, host frames -> tiles
pipe = FramePipeline(B, 512, 1024, dev, depth=2)
pipe.put(frames)
pipe.get()
torch.cuda.synchronize()
t0 = time.perf_counter()
n = 20
pipe.put(frames)
for i in range(n):
    if i + 1 < n:
        pipe.put(frames)
    pipe.get()
torch.cuda.synchronize()
pipe_fps = n * B / (time.perf_counter() - t0)
# CPU reference chain, 1 thread
from oracle import frames_oracle as O  # noqa: E402
torch.set_num_threads(1)
t0 = time.perf_counter()
O.preprocess_image_batch(list(frames[:a.cpu_frames]), 448, 2, True)
cpu_fps = a.cpu_frames / (time.perf_counter() - t0)
print(json.dumps({
    "workload": f"collate image path: {B} x 1024x512 uint8 frames -> [{B},2,3,448,448] f32 tiles",
    "kernel_ms": round(ms, 4), "frames_per_s": round(B / (ms * 1e-3), 1),
    "roofline": {"bound": "hbm", "achieved": round(gbs, 1), "peak": 8000.0, "unit": "GB/s",
                 "frac": round(gbs / 8000.0, 4), "algorithmic_bytes": alg},
    "pipeline_pcie_inclusive_frames_per_s": round(pipe_fps, 1),
    "cpu_baseline": {"value": round(cpu_fps, 2), "unit": "frames/s", "cores": 1, "kind": "port",
                     "sample": f"{a.cpu_frames} frames through Pillow resize + torch ToTensor/Normalize"},
}))
