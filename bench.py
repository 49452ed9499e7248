"""SimLingo VLA training throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config vla|tiny] [--no-cpu-baseline]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[2], the config the metric is quoted on at 1/2/4/8 GPUs): SimLingo full
VLA = InternViT-300M (2 tiles of 448^2 per frame) + mlp1 + Qwen2-0.5B with LoRA r32 (dropout 0.1)
+ driving heads, bf16 MFMA / f32 accumulation, B = 8 samples per GPU, 256 text tokens per prompt
(S_llm = 798), 16 LM-loss tokens per sample. One step = forward + backward + bucketed RCCL
gradient all-reduce + clip + AdamW on 327.5 M trainable parameters, synthetic seeded data of the
reference's shape (no dataset / checkpoint offline), random-init weights of that architecture.
Data parallel, one process per GPU, per-GPU batch fixed -> weak scaling.

Roofline: the dominant kernel is the bf16 MFMA GEMM; `roofline` reports the InternViT FC1 GEMM
(M = 16*1025 tokens, N = 4096, K = 1024, gelu epilogue, 24 launches per step) timed with HIP events
on its launch stream during the timed steps, against the 2.5 PFLOP/s dense bf16 peak.
`step_mfma_frac` = samples/s x 5670.1 GFLOP/sample (required FLOPs) / (n_gpu x peak).
cpu_baseline: the oracle (CPU fp32 PyTorch restatement, oracle/vla_oracle.py) forward+backward of
one full-size sample on the host cores, rank 0, N = 1 only.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0        # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
GFLOP_PER_SAMPLE = {"vla": 5670.1, "tiny": None}  # SURVEY.md §8d config 3 (required FLOPs)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="vla", choices=["vla", "tiny"])
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--s-text", type=int, default=256)
    ap.add_argument("--n-loss", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    return ap.parse_args()


def cpu_baseline(cfg, s_text, n_loss, threads):
    """Oracle fwd+bwd of ONE full-size sample on the host (bounded ~10-30 s)."""
    from oracle import vla_oracle as O
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    torch.set_num_threads(threads)
    P = init_params(cfg, seed=0)
    ex = make_batch(cfg, B=1, s_text=s_text, n_loss=n_loss, seed=1234)
    t0 = time.perf_counter()
    O.loss_and_grads(P, cfg, ex)
    dt = time.perf_counter() - t0
    return {"value": 1.0 / dt, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"1 sample fwd+bwd (S_llm={s_text + cfg.img_tokens + cfg.n_queries}), fp32, {dt:.1f} s"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    from simlingo_amd.config import full_config, tiny_config
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.params import init_params
    from simlingo_amd.plan import plan_from_example
    from simlingo_amd.synthetic import make_batch

    cfg = full_config() if args.config == "vla" else tiny_config(lora_dropout=0.1)
    B = args.batch
    s_text = args.s_text if args.config == "vla" else 24
    n_loss = args.n_loss if args.config == "vla" else 6
    params = init_params(cfg, seed=0, device=dev)
    eng = VLAEngine(cfg, dev, params)
    del params
    if world > 1:
        import torch.distributed as dist
        dist.broadcast(eng.master, src=0)
        eng.wbf.copy_(eng.master.to(torch.bfloat16))
        eng._refresh_derived()
        eng.set_distributed(None, world)
    # per-rank synthetic batch (rank-offset seed), resident in HBM before timing
    ex = make_batch(cfg, B=B, s_text=s_text, n_loss=n_loss, seed=1000 + rank)
    plan = plan_from_example(cfg, ex)
    dplan = plan.to_device(dev)
    pix = ex.driving_input.camera_images.to(dev)
    path = ex.driving_label.path.to(dev)
    wps = ex.driving_label.waypoints.to(dev)
    torch.cuda.synchronize()
    lr = cfg.lr

    def step(i):
        out4, _, _ = eng.forward(pix, plan, dplan, path, wps, training=True)
        eng.backward(None)
        eng.adamw_step(lr, i + 1, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay, max_norm=cfg.grad_clip)
        return out4

    out4 = None
    for i in range(args.warmup):
        out4 = step(i)
    if out4 is None:  # --warmup 0: the first timed step's loss is reported as loss_first
        out4 = torch.full((4,), float("nan"), device=dev)
    torch.cuda.synchronize()
    loss0 = out4[0].item()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    eng.probe_site = "vit.fc1" if args.config == "vla" else None
    eng.probe_events = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        out4 = step(args.warmup + i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    eng.probe_site = None
    t = torch.tensor([dt], device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = t.item()
    loss_last = out4[0].item()
    samples = B * world * args.steps
    value = samples / dt
    res = {
        "metric": "training samples/sec (frame+prompt->waypoints)",
        "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": "simlingo full VLA train step (InternViT-300M x2 tiles + mlp1 + Qwen2-0.5B LoRA r32 + heads)"
                   if args.config == "vla" else "tiny parity geometry",
                   "model": "InternVL2-1B geometry, random init" if args.config == "vla" else "tiny",
                   "global_batch": B * world, "per_gpu_batch": B, "seq_len": plan.S, "s_text": s_text,
                   "loss_tokens_per_sample": n_loss, "parallelism": f"dp{world}"},
        "loss_first": round(loss0, 5), "loss_last": round(loss_last, 5),
    }
    gf = GFLOP_PER_SAMPLE[args.config]
    if gf:
        res["step_mfma_frac"] = round(value * gf / 1e3 / (world * PEAK_BF16_TFLOPS), 4)
        res["step_tflops_per_gpu"] = round(value * gf / 1e3 / world, 1)
    if eng.probe_events:
        ms = [a.elapsed_time(b) for a, b in eng.probe_events]
        avg_ms = sum(ms) / len(ms)
        M = 2 * B * cfg.vit_tokens
        flop = 2.0 * M * cfg.vit_ffn * cfg.vit_dim
        ach = flop / (avg_ms * 1e-3) / 1e12
        res["roofline"] = {"bound": "mfma", "kernel": "slx gemm_bf16 NT+gelu (InternViT fc1)",
                           "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                           "frac": round(ach / PEAK_BF16_TFLOPS, 4), "traffic": None,
                           "flop_per_launch": flop, "avg_launch_ms": round(avg_ms, 4), "launches": len(ms)}
    if rank == 0 and world == 1 and args.config == "vla" and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = cpu_baseline(cfg, s_text, n_loss, args.cpu_threads)
        except Exception as e:  # the bench line must still be printed
            res["cpu_baseline"] = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
