"""Data-parallel gradient exchange on CPU with gloo, world_size 2 (the N>1 path of bench.py)."""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from simlingo_amd.config import full_config, tiny_config
from simlingo_amd.ddp import GradBucketer
from simlingo_amd.params import param_specs


def group_ranges(cfg, align=64):
    off, ranges = 0, {}
    for s in param_specs(cfg):
        if not s.trainable:
            continue
        n = (math.prod(s.shape) + align - 1) // align * align
        a, b = ranges.get(s.group, (off, off + n))
        ranges[s.group] = (min(a, off), max(b, off + n))
        off += n
    return ranges, off


def test_buckets_cover_flat_buffer_in_backward_order():
    cfg = full_config()
    ranges, n = group_ranges(cfg)
    bk = GradBucketer(torch.zeros(n), ranges, bucket_bytes=32 << 20)
    spans = bk.summary()
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, b0, _), (a1, b1, _) in zip(spans, spans[1:]):
        assert b0 == a1  # contiguous, no overlap
    # backward order: heads first, LoRA layers last->first, assembly, projector, ViT last->first, embeddings
    order = [g for b in bk.buckets for g in b.groups]
    assert order[0] == "heads" and order[-1] == "vit_embed"
    assert order.index("llm23") < order.index("llm0") < order.index("assembly") < order.index("proj")
    assert order.index("vit23") < order.index("vit0")
    # ViT layers (12.6 M params = 50 MB f32) are their own buckets; LoRA layers are merged
    assert any(b.groups == ["vit12"] for b in bk.buckets)
    assert sum(1 for b in bk.buckets if any(g.startswith("llm") for g in b.groups)) < cfg.llm_layers


def _worker(rank, world, port, n, ranges, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.arange(n, dtype=torch.float32) * (rank + 1)
    bk = GradBucketer(g, ranges, bucket_bytes=4096)
    bk.set_distributed(None, world)
    order = sorted(ranges, key=lambda k: ranges[k][0])
    for name in order:  # the backward signals groups in layout order
        bk.group_done(name)
    bk.wait()
    ret[rank] = g.clone()
    dist.destroy_process_group()


def test_bucketed_allreduce_gloo_world2():
    cfg = tiny_config()
    ranges, n = group_ranges(cfg)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mgr = mp.Manager()
    ret = mgr.dict()
    mp.spawn(_worker, args=(2, port, n, ranges, ret), nprocs=2, join=True)
    want = torch.arange(n, dtype=torch.float32) * 3  # sum over ranks (1x + 2x); AdamW applies 1/world
    for r in range(2):
        torch.testing.assert_close(ret[r], want)


def _overlap_worker(rank, world, port, n, ranges, wire, ret):
    """A backward that signals its parameter groups in layout order with ~10 ms of compute between them: the first
    buckets' all-reduces (gloo runs them on its own thread, as RCCL runs them on its own stream) must complete
    while the backward is still running."""
    import time
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    g = torch.arange(n, dtype=torch.float32) * (rank + 1) * 1e-3
    bk = GradBucketer(g, ranges, bucket_bytes=1 << 16, wire=wire, trace=True, timing=True)
    bk.set_distributed(None, world)
    work = torch.randn(192, 192)
    # one collective first (as every training step after the first has had): connection setup and the two ranks'
    # start-up skew stay out of the measured backward (without it the first bucket intermittently completed only
    # after backward_end on a loaded host)
    dist.all_reduce(torch.zeros(1))
    dist.barrier()
    for name in sorted(ranges, key=lambda k: ranges[k][0]):
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 10e-3:  # "backward compute" of this group (10 ms: host stalls of ~10 ms happen)
            work = torch.tanh(work @ work.t() * 1e-3)
            bk.poll()
        bk.group_done(name)
    bk.mark("backward_end")
    bk.wait()
    og, is_bf16 = bk.optimizer_grad()  # what the optimizer reads (the bf16 wire buffer itself on the bf16 wire)
    assert is_bf16 == (wire == "bf16") and (is_bf16 or og is g)
    ret[rank] = (og.float().clone(), list(bk.trace), len(bk.buckets), bk.comm_summary())
    dist.destroy_process_group()


def _overlap_attempt(wire):
    cfg = tiny_config()
    ranges, n = group_ranges(cfg)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ret = mp.Manager().dict()
    mp.spawn(_overlap_worker, args=(2, port, n, ranges, wire, ret), nprocs=2, join=True)
    want = torch.arange(n, dtype=torch.float32) * 3e-3
    overlapped = True
    for r in range(2):
        g, trace, nb, cs = ret[r]
        # bench.py's comm keys (device clock on GPUs, host clock here): the exposed tail after backward_end and each
        # bucket's issue / done time relative to it; the first bucket is issued ~nb * 10 ms before the end
        assert cs["n_buckets"] == nb and cs["wire"] == wire and cs["steps"] == 1
        assert 0.0 <= cs["comm_exposed_ms"] < 1e3
        rows = cs["bucket_issue_done_ms"]
        assert len(rows) == nb and rows[0][1] < -4.0 and all(d is not None and d >= t for _, t, d in rows)
        if wire == "f32":
            torch.testing.assert_close(g, want)
        else:  # bf16 on the wire, widened in the optimizer: within world * 2^-8 of the sum of magnitudes (ddp.py)
            assert bool(((g - want).abs() <= 2 * 2.0 ** -8 * want.abs() + 1e-30).all())
            assert not torch.equal(g, want)  # the wire really was bf16
        t_end = next(t for ev, _, t in trace if ev == "backward_end")
        issued = [(b, t) for ev, b, t in trace if ev == "issue"]
        done = {b: t for ev, b, t in trace if ev == "done"}
        assert len(issued) == nb > 2
        # every bucket but the last is launched before the backward ends (deterministic: the issue order)
        assert sum(t < t_end for _, t in issued) >= nb - 1
        # and the first one completes before it ends (timing: gloo's worker threads against the host's scheduling)
        overlapped = overlapped and 0 in done and done[0] < t_end
    return overlapped


@pytest.mark.parametrize("wire", ["f32", "bf16"])
def test_allreduce_overlaps_backward_and_bf16_wire(wire):
    # the numerics and the issue order are checked on every attempt; the completion-before-backward_end property is a
    # timing one, and on this shared CPU host gloo's threads were seen to make no progress for ~100 ms in about one
    # run in six, so it must hold in one of three attempts
    assert any(_overlap_attempt(wire) for _ in range(3))


def _world8_worker(rank, world, port, n, ranges, wire, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    gen = torch.Generator().manual_seed(100 + rank)
    g = torch.randn(n, generator=gen) * torch.logspace(-6, 0, n)  # mixed signs and magnitudes, as gradients are
    local = g.clone()
    bk = GradBucketer(g, ranges, bucket_bytes=1 << 16, wire=wire)
    bk.set_distributed(None, world)
    for name in sorted(ranges, key=lambda k: ranges[k][0]):
        bk.group_done(name)
    bk.mark("backward_end")
    bk.wait()
    og, _ = bk.optimizer_grad()
    ret[rank] = (local, og.float().clone())
    dist.destroy_process_group()


@pytest.mark.parametrize("wire", ["f32", "bf16"])
def test_bucketed_allreduce_world8(wire):
    """VERDICT r4 do-this #7: 8 ranks (the N = 8 node), every bucket summed; on the bf16 wire each element of the
    optimizer's gradient lies within 8 * 2^-8 * sum_r |g_r| of the exact sum (ddp.py's stated bound), on the f32 wire
    within f32 summation order."""
    cfg = tiny_config()
    ranges, n = group_ranges(cfg)
    world = 8
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ret = mp.Manager().dict()
    mp.spawn(_world8_worker, args=(world, port, n, ranges, wire, ret), nprocs=world, join=True)
    locals_ = torch.stack([ret[r][0] for r in range(world)]).double()
    exact = locals_.sum(0)
    mag = locals_.abs().sum(0)
    for r in range(world):
        got = ret[r][1].double()
        assert torch.equal(ret[r][1], ret[0][1])  # every rank holds the same summed gradient
        if wire == "f32":
            assert bool(((got - exact).abs() <= 8 * 2.0 ** -24 * mag + 1e-30).all())
        else:
            err = (got - exact).abs()
            assert bool((err <= world * 2.0 ** -8 * mag + 1e-30).all()), (err / mag.clamp_min(1e-30)).max().item()
            print(f"bf16 wire, world {world}: max error / sum|g| = {(err / mag.clamp_min(1e-30)).max().item():.3g}")
            assert not torch.equal(ret[r][1], exact.float())


def test_wait_refuses_unexchanged_buckets():
    """at world > 1 a bucket the backward never issued would hand AdamW a stale (bf16 wire) or un-summed
    (f32 wire) slice; wait() refuses it instead."""
    g = torch.zeros(4096)
    bk = GradBucketer(g, {"a": (0, 2048), "b": (2048, 4096)}, bucket_bytes=1024, wire="bf16")
    bk.set_distributed(None, 2)
    with pytest.raises(RuntimeError, match="not exchanged"):
        bk.wait()
    bk.set_distributed(None, 1)
    bk.wait()  # single process: nothing to exchange


def test_wait_is_idempotent_after_an_exchange():
    """wait() twice in one step (the optimizer's own wait after an explicit one) is a no-op the second time; a new
    step's partial exchange is refused again."""
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ret = mp.Manager().dict()
    mp.spawn(_idem_worker, args=(port, ret), nprocs=1, join=True)
    assert ret["ok"], dict(ret)


def _idem_worker(rank, port, ret):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=0, world_size=1)
    g = torch.ones(4096)
    bk = GradBucketer(g, {"a": (0, 2048), "b": (2048, 4096)}, bucket_bytes=1024)
    bk.set_distributed(None, 2)  # issue as at N = 2; the group has one rank
    bk.group_done("a")
    bk.group_done("b")
    bk.wait()
    bk.wait()
    bk.group_done("a")  # next step: only one bucket issued
    try:
        bk.wait()
        ret["ok"] = False
    except RuntimeError:
        ret["ok"] = True
    dist.destroy_process_group()
