"""Golden fixture for the SimLingo-Base collate's non-image fields (tests/golden/base_labels.npz).

Test infrastructure only. VERDICT r3 missing #6: the base collate must carry the reference's camera matrices,
waypoints_1d and run_id encoding. Their reference definitions are pure numpy / torch, but the modules that hold them
import cv2 / hydra / pytorch_lightning (absent), so the definitions are read from the reference files with `ast` and
executed on their own, unmodified (nothing is copied into this repository):
  simlingo_base_training/utils/projection.py      get_camera_intrinsics(w, h, fov), get_camera_extrinsics()
                                                  (the ones datamodule.py:39 imports, used at :252-253)
  simlingo_base_training/dataloader/datamodule.py encode_uint8(strings, common_length) (:42-62, used at :264)
  simlingo_base_training/dataloader/dataset_base.py BaseDataset.load_waypoints (:368-392), run on a stub `self`
                                                  whose get_waypoints returns the given ego-frame waypoint list, so
                                                  data['waypoints'] / data['waypoints_1d'] (:373, :381-385) come out
                                                  of the reference's own arithmetic
Inputs: seeded 13-point ego-frame waypoint lists (origin first, like get_waypoints' current-frame entry), frame sizes
(1024 x 359 cut, 1024 x 512 uncut, 256 x 80 tiny) and measurement-path strings.

    python oracle/gen_golden_base_labels.py
"""
import ast
import os
import sys
from typing import List

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REFB = "/root/reference/simlingo_base_training"
OUT = os.path.join(ROOT, "tests", "golden", "base_labels.npz")


def _defs(path, names, ns):
    tree = ast.parse(open(path).read())
    keep = [n for n in tree.body if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in names]
    exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
    return ns


def _method(path, cls, name, ns):
    tree = ast.parse(open(path).read())
    c = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == cls)
    m = next(n for n in c.body if isinstance(n, ast.FunctionDef) and n.name == name)
    exec(compile(ast.Module(body=[m], type_ignores=[]), path, "exec"), ns)
    return ns[name]


def reference_functions():
    ns = {"np": np, "torch": torch, "List": List}
    _defs(os.path.join(REFB, "utils", "projection.py"), ("get_camera_intrinsics", "get_camera_extrinsics"), ns)
    _defs(os.path.join(REFB, "dataloader", "datamodule.py"), ("encode_uint8",), ns)
    load_waypoints = _method(os.path.join(REFB, "dataloader", "dataset_base.py"), "BaseDataset", "load_waypoints", ns)
    return ns["get_camera_intrinsics"], ns["get_camera_extrinsics"], ns["encode_uint8"], load_waypoints


class _StubDataset:
    """Only what load_waypoints reads from `self`: hist_len and get_waypoints (returns the stored list)."""
    hist_len = 1

    def __init__(self, wps):
        self._wps = wps

    def get_waypoints(self, measurements, y_augmentation=0.0, yaw_augmentation=0.0):
        return [np.asarray(w) for w in self._wps]


def synthetic_full_waypoints(seed, n=13):
    """Ego-frame positions of the current (origin) and next n-1 measurements, as get_waypoints returns them."""
    rng = np.random.default_rng(seed)
    steps = np.array([0.8, 0.0]) + 0.3 * rng.normal(size=(n - 1, 2))
    return np.concatenate([np.zeros((1, 2)), np.cumsum(steps, 0)], 0)


def main():
    intr, extr, encode_uint8, load_waypoints = reference_functions()
    out = {}
    sizes = [(1024, 359), (1024, 512), (256, 80)]
    out["cam.sizes"] = np.asarray(sizes)
    for i, (w, h) in enumerate(sizes):
        out[f"cam.K.{i}"] = intr(w, h, 110).numpy()
    out["cam.E"] = extr().numpy()
    seeds = [11, 12, 13]
    out["wp.seeds"] = np.asarray(seeds)
    for s in seeds:
        full = synthetic_full_waypoints(s)
        data = load_waypoints(_StubDataset(full), {}, [None])
        out[f"wp.full.{s}"] = full
        out[f"wp.waypoints.{s}"] = np.asarray(data["waypoints"], dtype=np.float64)
        out[f"wp.waypoints_1d.{s}"] = np.asarray(data["waypoints_1d"], dtype=np.float64)
    paths = ["data/simlingo/training_1_scenario/routes_training/random_weather_seed_1/Town12_Rep0_1234_route0/"
             "measurements", "x", ""]
    out["run.paths"] = np.asarray(paths)
    out["run.enc"] = encode_uint8(paths, 1000).numpy()
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, sorted(out))


if __name__ == "__main__":
    main()
