"""Data-parallel step with the real HIP engine: 2 ranks sharing one GPU over gloo (RCCL needs one
GPU per rank; the driver's 8-GPU scaling run exercises it). The bucketed all-reduce overlapped with
backward must produce the SUM of the per-rank gradients in every bucket."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, ret):
    import torch.distributed as dist
    from simlingo_amd.config import tiny_config
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    from simlingo_amd.synthetic import make_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    cfg = tiny_config()

    def grads(seed, distributed):
        eng = VLAEngine(cfg, dev, seed=5, bucket_bytes=64 << 10)
        if distributed:
            eng.set_distributed(None, world)
            eng.bucketer.trace_on = True
        ex = make_batch(cfg, B=2, s_text=24, n_loss=4, seed=seed)
        plan = plan_from_example(cfg, ex)
        eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev),
                    ex.driving_label.path.to(dev), ex.driving_label.waypoints.to(dev))
        eng.backward(None)
        trace = list(eng.bucketer.trace)
        eng.wait_grads()
        torch.cuda.synchronize()
        return eng.grad.cpu().clone(), len(eng.bucketer.buckets), trace

    g_dp, nb, trace = grads(100 + rank, True)
    ret[rank] = (g_dp, nb, trace)
    if rank == 0:
        ret["ref"] = grads(100, False)[0] + grads(101, False)[0]
    dist.barrier()
    dist.destroy_process_group()


def test_dp_allreduce_matches_sum_of_rank_grads(dev):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ret = mp.Manager().dict()
    mp.spawn(_worker, args=(2, port, ret), nprocs=2, join=True)
    ref = ret["ref"]
    for r in range(2):
        g, nb, trace = ret[r]
        assert nb > 1
        err = ((g - ref).norm() / ref.norm()).item()
        assert err < 1e-2, err
        # the exchange is issued during the backward: every bucket but the last (the patch embedding's) is launched
        # before the engine's backward returns, while later layers' kernels are still being queued
        t_end = next(t for ev, _, t in trace if ev == "backward_end")
        issued = [t for ev, _, t in trace if ev == "issue"]
        assert len(issued) == nb and sum(t < t_end for t in issued) >= nb - 1
