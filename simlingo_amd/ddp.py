"""Data-parallel gradient exchange: bucketed all-reduce over RCCL (xGMI) overlapped with backward.

Replaces DeepSpeed ZeRO-2's bucketed reduce + param all-gather and Lightning DDP's hook-driven
all-reduce (simlingo_training/train.py:160-168). The flat f32 gradient
buffer is laid out in backward-completion order, so each bucket is one contiguous slice: when the
backward finishes the last parameter group of a bucket, one async all_reduce(SUM) of that slice is
issued on RCCL's stream (ordered after the producing kernels of the compute stream), while the
backward of earlier layers keeps running. The optimizer waits on the handles and applies 1/world
inside the fused AdamW kernel (no extra pass). Device-agnostic (the CPU tests drive it with gloo).

wire="bf16" (SURVEY.md §8e): each bucket is cast to a bf16 staging slice before its all-reduce (half the xGMI
bytes: 655 MB instead of 1.31 GB for the full model) and cast back into the f32 gradient when the optimizer waits, so
the optimizer still accumulates in f32. trace=True records (event, bucket, perf_counter) tuples - "issue" when a
bucket's all-reduce is launched, "backward_end" from the engine, "done" when a handle is found complete - the
evidence that the exchange overlaps the backward (tests/test_ddp_gloo.py).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import time

import torch


@dataclass
class Bucket:
    start: int
    end: int
    groups: list
    done: int = 0
    handle: object = None


class GradBucketer:
    def __init__(self, flat_grad: torch.Tensor, group_ranges: dict[str, tuple[int, int]], bucket_bytes: int = 32 << 20,
                 wire: str = "f32", trace: bool = False):
        if wire not in ("f32", "bf16"):
            raise ValueError(f"wire must be 'f32' or 'bf16', got {wire!r}")
        self.flat = flat_grad
        self.wire = wire
        self.wire_buf = None
        self.trace_on = trace
        self.trace: list[tuple[str, int, float]] = []
        order = sorted(group_ranges, key=lambda g: group_ranges[g][0])
        self.buckets: list[Bucket] = []
        cur = None
        for g in order:
            a, b = group_ranges[g]
            if cur is None or (cur.end - cur.start) * flat_grad.element_size() >= bucket_bytes or cur.end != a:
                cur = Bucket(a, b, [g])
                self.buckets.append(cur)
            else:
                cur.end = b
                cur.groups.append(g)
        self.group_bucket = {g: bk for bk in self.buckets for g in bk.groups}
        self.pg = None
        self.world = 1

    def set_distributed(self, pg=None, world: int = 1):
        self.pg = pg
        self.world = world

    def group_done(self, g: str):
        """Called by the backward when every gradient of parameter group `g` has been written."""
        if self.world <= 1:
            return
        bk = self.group_bucket[g]
        bk.done += 1
        if bk.done == len(bk.groups):
            import torch.distributed as dist
            src = self.flat[bk.start:bk.end]
            if self.wire == "bf16":
                if self.wire_buf is None:
                    self.wire_buf = torch.empty(self.flat.numel(), dtype=torch.bfloat16, device=self.flat.device)
                src = self.wire_buf[bk.start:bk.end]
                src.copy_(self.flat[bk.start:bk.end])
            bk.handle = dist.all_reduce(src, group=self.pg, async_op=True)
            if self.trace_on:
                self.trace.append(("issue", self.buckets.index(bk), time.perf_counter()))

    def mark(self, event: str):
        if self.trace_on:
            self.trace.append((event, -1, time.perf_counter()))

    def poll(self):
        """Trace which in-flight all-reduces have completed (test instrumentation)."""
        for i, bk in enumerate(self.buckets):
            if bk.handle is not None and bk.handle.is_completed() and not getattr(bk, "_seen", False):
                bk._seen = True
                if self.trace_on:
                    self.trace.append(("done", i, time.perf_counter()))

    def wait(self):
        for bk in self.buckets:
            if bk.handle is not None:
                bk.handle.wait()
                bk.handle = None
                if self.wire == "bf16":  # back into the f32 gradient the optimizer reads
                    self.flat[bk.start:bk.end].copy_(self.wire_buf[bk.start:bk.end])
            bk.done = 0
            bk._seen = False

    def summary(self) -> list[tuple[int, int, int]]:
        """[(start, end, n_groups)] in launch order."""
        return [(b.start, b.end, len(b.groups)) for b in self.buckets]
