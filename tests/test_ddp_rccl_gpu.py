"""The bucketed gradient exchange over RCCL itself (torch.distributed backend "nccl" = RCCL on ROCm) on the one GPU of
a test box (the RCCL path had never executed on hardware; test_ddp_gpu.py shares one GPU between two ranks
and so must use gloo). One rank, an "nccl" process group of size 1, and the bucketer told world = 2 so that it
issues every bucket's asynchronous all_reduce during the backward exactly as at N > 1 (bench.py / ddp.py), on the
f32 wire (the default) and the bf16 wire, with the device-clock timing on: a one-rank all-reduce returns the rank's
own gradient, so the buffer the optimizer reads (GradBucketer.optimizer_grad: the bf16 wire buffer itself, or the f32
buffer summed in place) must equal the non-distributed gradient to the wire rounding, every bucket must have been
issued before backward_end (except the last) and comm_summary() must report the exposed tail."""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _worker(rank, port, ret, geom="tiny", wire="bf16"):
    import torch.distributed as dist
    from simlingo_amd.config import full_config, tiny_config
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.plan import plan_from_example
    from simlingo_amd.synthetic import make_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
    # full: the real widths (1 ViT + 2 Qwen2 layers), where the LoRA gradients take the grouped slx_lora_grad path
    cfg = tiny_config() if geom == "tiny" else full_config(vit_layers=1, llm_layers=2)
    ex = make_batch(cfg, B=2, s_text=24 if geom == "tiny" else 64, n_loss=4, seed=7)
    plan = plan_from_example(cfg, ex)

    def run(distributed):
        eng = VLAEngine(cfg, dev, seed=5, bucket_bytes=64 << 10, wire=wire)
        if distributed:
            eng.set_distributed(None, 2)  # issue the exchange as at N = 2; the group has one rank
            eng.bucketer.trace_on = True
            eng.bucketer.timing = True
        eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev),
                    ex.driving_label.path.to(dev), ex.driving_label.waypoints.to(dev))
        eng.backward(None)
        eng.wait_grads()
        torch.cuda.synchronize()
        summ = eng.bucketer.comm_summary() if distributed else None
        # what AdamW reads after the exchange: the summed bf16 wire buffer itself on the bf16 wire (ddp.py no longer
        # copies it back into eng.grad), the flat f32 buffer summed in place on the f32 wire
        g, is_bf16 = eng.bucketer.optimizer_grad()
        return g.float().cpu().clone(), len(eng.bucketer.buckets), list(eng.bucketer.trace), summ, is_bf16

    g_ref, _, _, _, _ = run(False)
    g_dp, nb, trace, summ, is_bf16 = run(True)
    ret["is_bf16"] = is_bf16
    ret["bitwise_equal"] = torch.equal(g_dp, g_ref)
    ret["err"] = ((g_dp - g_ref).norm() / g_ref.norm()).item()
    ret["nb"] = nb
    t_end = next(t for ev, _, t in trace if ev == "backward_end")
    issued = [t for ev, _, t in trace if ev == "issue"]
    ret["issued"] = len(issued)
    ret["before_end"] = sum(t < t_end for t in issued)
    ret["summary"] = summ
    ret["backend"] = dist.get_backend()
    dist.destroy_process_group()


@pytest.mark.parametrize("geom,wire", [("tiny", "bf16"), ("full", "bf16"), ("full", "f32")])
def test_rccl_bucketed_exchange_on_hardware(dev, geom, wire):
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ret = mp.Manager().dict()
    mp.spawn(_worker, args=(port, ret, geom, wire), nprocs=1, join=True)
    print(dict(ret))
    assert ret["backend"] == "nccl"
    assert ret["nb"] > 1 and ret["issued"] == ret["nb"] and ret["before_end"] >= ret["nb"] - 1
    assert ret["is_bf16"] == (wire == "bf16")
    if wire == "bf16":
        assert ret["err"] < 1e-2, ret["err"]  # bf16 wire rounding of each gradient
        assert not ret["bitwise_equal"]       # the optimizer really reads the bf16 wire buffer
    else:
        assert ret["err"] < 1e-3, ret["err"]  # the exchanged f32 gradient: run-to-run atomic order only
    s = ret["summary"]
    assert s is not None and s["n_buckets"] == ret["nb"] and s["wire"] == wire and s["comm_exposed_ms"] >= 0.0
