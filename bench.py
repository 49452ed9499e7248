"""SimLingo training throughput on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config vla|base|tiny|base_tiny] [--no-cpu-baseline]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Default workload `vla` (BASELINE.json configs[2], the config the metric is quoted on at 1/2/4/8 GPUs): SimLingo
full VLA = InternViT-300M (2 tiles of 448^2 per frame) + mlp1 + Qwen2-0.5B with LoRA r32 (dropout 0.1)
+ driving heads, bf16 MFMA / f32 accumulation, B = 8 samples per GPU, 256 text tokens per prompt
(S_llm = 798), 16 LM-loss tokens per sample. One step = forward + backward + bucketed RCCL
gradient all-reduce + clip + AdamW on 327.5 M trainable parameters, synthetic seeded data of the
reference's shape (no dataset / checkpoint offline), random-init weights of that architecture.
Data parallel, one process per GPU, per-GPU batch fixed -> weak scaling.

`base` (BASELINE.json configs[1]): SimLingo-Base = CLIP ViT-L/14-336 (2 tiles of 336^2, first 23 layers) +
LLaVA-NeXT projector + unpad / avg-pool / image_newline (200 tokens for the 1024x359 frame) + Linear 4096->512
+ speed / target-point tokens + Llama 'tiny' + heads, every parameter trainable, B = 32, S = 233; one step =
forward + backward + clip 1.0 + four-group AdamW.

Roofline: the dominant kernel is the bf16 MFMA GEMM; `roofline` reports the ViT FC1 GEMM (vla: M = 16*1025,
N = 4096, K = 1024, GELU epilogue, 24 launches per step; base: M = 64*577, quick_gelu, 23 launches) timed with
HIP events on its launch stream during the timed steps, against the 2.5 PFLOP/s dense bf16 peak.
`step_mfma_frac` = samples/s x required GFLOP/sample / (n_gpu x peak). `traffic` = HBM bytes
per launch from the rocprofv3 FETCH_SIZE / WRITE_SIZE passes recorded in profiles/*_fc1_traffic.json
(tools/pmc_traffic.py), when one matches the workload.
cpu_baseline: the oracle (CPU fp32 PyTorch restatement, oracle/) forward+backward of one full-size sample on
the host cores (1 warmup + median of 3), rank 0, N = 1 only.
"""
from __future__ import annotations

import argparse
import glob
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_BF16_TFLOPS = 2500.0        # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
VLA_GFLOP_PER_SAMPLE = 5670.1    # SURVEY.md §8d config 3 (required FLOPs)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="vla", choices=["vla", "tiny", "base", "base_tiny"])
    ap.add_argument("--batch", type=int, default=None, help="per-GPU batch (vla 8, base 32)")
    ap.add_argument("--s-text", type=int, default=256)
    ap.add_argument("--n-loss", type=int, default=16)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--wire", default="auto", choices=["auto", "f32", "bf16"],
                    help="gradient all-reduce wire dtype (auto = f32: the exchange is exact to f32 summation order, "
                         "stricter than the reference's fp16 ZeRO-2 reduce; bf16: half the xGMI bytes, opt-in)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in loop key (DataLoader + Collate + "
                    "DrivingModel.training_step + FusedAdamW + OneCycleLR)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the config-4 (S_text 512, 128 loss tokens) step, the config-5 agent latency and the "
                         "config-2 SimLingo-Base step that the N = 1 vla line carries as extra keys")
    return ap.parse_args()


def base_gflop(cfg) -> float:
    """Required GFLOP per SimLingo-Base sample (2414.7 at S = 233): CLIP layers
    0..vit_used-1 and the patch embedding on every tile, the projector on every patch feature, Linear(4096 -> E)
    on the merged tokens, Llama with causal-half attention; backward = 2x forward minus the patch-embedding
    dgrad (its input is the pixels). Heads and elementwise work ignored."""
    T, D, F = cfg.vit_tokens, cfg.vit_dim, cfg.vit_ffn
    g2 = cfg.vit_grid ** 2
    n = cfg.npatch
    clip = n * cfg.vit_used * (2 * T * (4 * D * D + 2 * D * F) + 4 * T * T * D)
    patch = n * 2 * g2 * cfg.patch_k * D
    proj = n * g2 * 2 * (D * cfg.proj_dim + cfg.proj_dim * cfg.proj_dim)
    enc = 2 * cfg.img_tokens * cfg.proj_dim * cfg.embed_dim
    S, d, Fl = cfg.seq, cfg.llm_dim, cfg.llm_ffn
    llm = cfg.llm_layers * (2 * S * (4 * d * d + 3 * d * Fl) + 2 * S * S * d)
    fwd = clip + patch + proj + enc + llm
    return (fwd + 2 * fwd - patch) / 1e9


def _timed(fn, warmup=1, reps=3):
    """SURVEY.md §8d CPU protocol: 1 warmup + median of 3."""
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return sorted(ts)[len(ts) // 2]


def cpu_baseline_vla(cfg, s_text, n_loss, threads):
    """Oracle fwd+bwd of ONE full-size sample on the host, 1 warmup + median of 3 (~12 s each)."""
    from oracle import vla_oracle as O
    from simlingo_amd.params import init_params
    from simlingo_amd.synthetic import make_batch
    torch.set_num_threads(threads)
    P = init_params(cfg, seed=0, lora_b_std=0.02)
    ex = make_batch(cfg, B=1, s_text=s_text, n_loss=n_loss, seed=1234)
    dt = _timed(lambda: O.loss_and_grads(P, cfg, ex))
    return {"value": 1.0 / dt, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"1 sample fwd+bwd (S_llm={s_text + cfg.img_tokens + cfg.n_queries}), fp32, "
                      f"1 warmup + median of 3: {dt:.1f} s"}


def cpu_baseline_base(cfg, threads):
    from oracle import base_oracle as O
    from simlingo_amd.base_params import init_base_params
    from simlingo_amd.base_types import make_base_batch
    torch.set_num_threads(threads)
    P = init_base_params(cfg, seed=0)
    ex = make_base_batch(cfg, B=1, seed=1234)
    dt = _timed(lambda: O.loss_and_grads(P, cfg, ex))
    return {"value": 1.0 / dt, "unit": "samples/s", "cores": threads, "kind": "port",
            "sample": f"1 sample fwd+bwd (S={cfg.seq}, 2 CLIP tiles), fp32, 1 warmup + median of 3: {dt:.1f} s"}


def setup_vla(args, dev, world, rank):
    from simlingo_amd.config import full_config, tiny_config
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.params import init_params
    from simlingo_amd.plan import plan_from_example
    from simlingo_amd.synthetic import make_batch
    full = args.config == "vla"
    cfg = full_config() if full else tiny_config(lora_dropout=0.1)
    B = args.batch or (8 if full else 4)
    s_text = args.s_text if full else 24
    n_loss = args.n_loss if full else 6
    eng = VLAEngine(cfg, dev, init_params(cfg, seed=0, lora_b_std=0.02, device=dev), wire=args.wire_eff)
    ex = make_batch(cfg, B=B, s_text=s_text, n_loss=n_loss, seed=1000 + rank)
    plan = plan_from_example(cfg, ex)
    dplan = plan.to_device(dev)
    pix = ex.driving_input.camera_images.to(dev)
    path = ex.driving_label.path.to(dev)
    wps = ex.driving_label.waypoints.to(dev)

    def step(i):
        out4, _, _ = eng.forward(pix, plan, dplan, path, wps, training=True)
        eng.backward(None)
        eng.adamw_step(cfg.lr, i + 1, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay,
                       max_norm=cfg.grad_clip)
        return out4

    return dict(
        eng=eng, step=step, B=B, gflop=VLA_GFLOP_PER_SAMPLE if full else None,
        metric_cfg={"workload": "simlingo full VLA train step (InternViT-300M x2 tiles + mlp1 + Qwen2-0.5B LoRA r32 + heads)"
                    if full else "tiny parity geometry",
                    "model": "InternVL2-1B geometry, random init" if full else "tiny", "seq_len": plan.S,
                    "s_text": s_text, "loss_tokens_per_sample": n_loss},
        probe=dict(M=2 * B * cfg.vit_tokens, N=cfg.vit_ffn, K=cfg.vit_dim, kernel="slx gemm_bf16 NT+gelu (InternViT fc1)",
                   tag="vla_b8",
                   # the step's dominant kernel: the InternViT fc2.w + fc1.w weight-gradient pair (one launch, TN,
                   # K = tokens), 2 x 2 x M x N x K FLOP
                   pair=dict(site="vit.wgrad_fc", flop=2 * 2.0 * (2 * B * cfg.vit_tokens) * cfg.vit_ffn * cfg.vit_dim,
                             kernel="slx gemm_bf16_pair TN (InternViT fc2.w + fc1.w weight gradients)",
                             # dY (bf16) + GELU output + dH + LN2 output, f32 dW read + write: per launch
                             algorithmic_bytes=int((2 * B * cfg.vit_tokens) * 2 * (2 * cfg.vit_dim + 2 * cfg.vit_ffn)
                                                   + 2 * 2 * 4 * cfg.vit_ffn * cfg.vit_dim))) if full else None,
        cpu=(lambda: cpu_baseline_vla(cfg, s_text, n_loss, args.cpu_threads)) if full else None)


def setup_base(args, dev, world, rank):
    from simlingo_amd.base_config import base_config, base_tiny_config
    from simlingo_amd.base_engine import BaseEngine
    from simlingo_amd.base_params import init_base_params
    from simlingo_amd.base_types import make_base_batch
    full = args.config == "base"
    cfg = base_config() if full else base_tiny_config()
    B = args.batch or (32 if full else 4)
    eng = BaseEngine(cfg, dev, init_base_params(cfg, seed=0))
    ex = make_base_batch(cfg, B, seed=1000 + rank)
    di, dl = ex.driving_input, ex.driving_label
    pix, speed, tp = di.camera_images.to(dev), di.vehicle_speed.to(dev), di.map_route.to(dev)
    route, wps = dl.route_adjusted.to(dev), dl.waypoints.to(dev)
    size = (cfg.frame_h, cfg.frame_w)

    def step(i):
        out4, _, _ = eng.forward(pix, speed, tp, route, wps, image_size=size)
        eng.backward(None)
        eng.adamw_step(cfg.lr, cfg.vision_lr, i + 1, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay,
                       max_norm=cfg.grad_clip)
        return out4

    return dict(
        eng=eng, step=step, B=B, gflop=base_gflop(cfg) if full else None,
        metric_cfg={"workload": "SimLingo-Base train step (CLIP ViT-L/14-336 x2 tiles + LLaVA-NeXT projector/merge + "
                                "Llama 'tiny' + heads, all trainable)" if full else "base tiny parity geometry",
                    "model": "llava-v1.6 CLIP-L/14-336 + Llama CONFIGS['tiny'] geometry, random init" if full else "tiny",
                    "seq_len": cfg.seq, "image_tokens": cfg.img_tokens, "frame": f"{cfg.frame_w}x{cfg.frame_h}"},
        probe=dict(M=B * cfg.npatch * cfg.vit_tokens, N=cfg.vit_ffn, K=cfg.vit_dim,
                   kernel="slx gemm_bf16 NT+quick_gelu (CLIP fc1)", tag="base_b32") if full else None,
        cpu=(lambda: cpu_baseline_base(cfg, args.cpu_threads)) if full else None)


VLA_C4_GFLOP_PER_SAMPLE = 6185.6  # SURVEY.md §8d config 4 (S_text 512, 128 loss tokens, S_llm 1054)


def config4_step(args, dev, steps=5, warmup=2):
    """BASELINE.json configs[3] on one GPU: the VLA step with mixed action + text loss at S_text = 512 (S_llm = 1054)
    and 128 LM-loss tokens per sample, B = 8, same protocol as the headline line (fwd + bwd + clip + AdamW)."""
    from simlingo_amd.config import full_config
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.params import init_params
    from simlingo_amd.plan import plan_from_example
    from simlingo_amd.synthetic import make_batch
    cfg = full_config()
    B = 8
    eng = VLAEngine(cfg, dev, init_params(cfg, seed=0, lora_b_std=0.02, device=dev))
    ex = make_batch(cfg, B=B, s_text=512, n_loss=128, seed=1000)
    plan = plan_from_example(cfg, ex)
    dplan = plan.to_device(dev)
    pix, path, wps = ex.driving_input.camera_images.to(dev), ex.driving_label.path.to(dev), ex.driving_label.waypoints.to(dev)

    def step(i):
        out4, _, _ = eng.forward(pix, plan, dplan, path, wps, training=True)
        eng.backward(None)
        eng.adamw_step(cfg.lr, i + 1, betas=cfg.betas, eps=cfg.eps, weight_decay=cfg.weight_decay, max_norm=cfg.grad_clip)
        return out4
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        out4 = step(warmup + i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    v = B * steps / dt
    del eng
    return {"workload": "config 4: S_text 512 (S_llm 1054), 128 LM-loss tokens/sample, B=8, 1 GPU", "value": round(v, 3),
            "unit": "samples/s", "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "seq_len": plan.S, "gflop_per_sample": VLA_C4_GFLOP_PER_SAMPLE,
            "step_mfma_frac": round(v * VLA_C4_GFLOP_PER_SAMPLE / 1e3 / PEAK_BF16_TFLOPS, 4),
            "loss_last": round(out4[0].item(), 5)}


def base_line(args, dev, steps=5, warmup=2):
    """BASELINE.json configs[1] on one GPU, carried as the `base` key of the N = 1 vla line: SimLingo-Base B = 32,
    fwd + bwd + clip 1.0 + four-group AdamW, with its own roofline (the CLIP FC1 GEMM, HIP events on its stream over
    the timed steps; traffic from the base PMC record)."""
    import argparse as _ap
    a = _ap.Namespace(**vars(args))
    a.config, a.batch = "base", None
    w = setup_base(a, dev, 1, 0)
    eng, step, B = w["eng"], w["step"], w["B"]
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    pr = w["probe"]
    eng.probe_site, eng.probe_events = "vit.fc1", []
    t0 = time.perf_counter()
    for i in range(steps):
        out4 = step(warmup + i)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    eng.probe_site = None
    v = B * steps / dt
    res = {"workload": "config 2: SimLingo-Base (CLIP ViT-L/14-336 x2 tiles + projector + Llama 'tiny'), B=32, 1 GPU",
           "value": round(v, 3), "unit": "samples/s", "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps,
           "warmup": warmup, "seq_len": w["metric_cfg"]["seq_len"], "gflop_per_sample": round(w["gflop"], 1),
           "step_mfma_frac": round(v * w["gflop"] / 1e3 / PEAK_BF16_TFLOPS, 4), "loss_last": round(out4[0].item(), 5)}
    if eng.probe_events:
        ms = [e0.elapsed_time(e1) for e0, e1 in eng.probe_events]
        avg_ms = sum(ms) / len(ms)
        flop = 2.0 * pr["M"] * pr["N"] * pr["K"]
        ach = flop / (avg_ms * 1e-3) / 1e12
        rec, src = traffic_record(pr["tag"], pr["M"])
        res["roofline"] = {"bound": "mfma", "kernel": pr["kernel"], "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS,
                           "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
                           "traffic": rec["traffic_bytes"] if rec else None, "flop_per_launch": flop,
                           "avg_launch_ms": round(avg_ms, 4), "launches": len(ms),
                           "algorithmic_bytes": rec.get("algorithmic_bytes") if rec else None,
                           "traffic_source": src}
    del eng, w
    return res


def agent_latency(dev, frames=5, new_tokens=100, s_text=64):
    """BASELINE.json configs[4]: team_code/agent_simlingo.py:797's DrivingModel.forward at bs = 1 (bench_infer.py's
    protocol: InternViT + assembly, prefill, KV-cached greedy decode of max_new_tokens, driving forward; median
    frame of `frames`)."""
    import bench_infer
    return bench_infer.measure(dev, frames=frames, warmup=1, new_tokens=new_tokens, s_text=s_text)


def dropin_loader(B=8, steps=10, warmup=3, workers=4, s_text=256, n_loss=16):
    """The reference's data path for the drop-in step (datamodule.py:275-284: DataLoader(num_workers, collate_fn=
    dl_collate_fn, pin_memory)): a 'dataset' of (warmup + steps) * B distinct synthetic DatasetOutputs (1024 x 512
    frames cropped to 359 rows, chat conversations of the config-3 length), batched by a DataLoader whose workers run
    Collate.host (tokenisation, masks, labels, stacked uint8 frames). Built and its workers forked BEFORE the process
    touches the GPU, so no worker inherits device state; the training process runs Collate.device (pinned-ring H2D +
    HIP frame kernel) per batch."""
    os.environ.setdefault("TOKENIZERS_PARALLELISM", "false")
    from torch.utils.data import DataLoader
    from simlingo_amd.collate import Collate
    from simlingo_amd.config import full_config
    from simlingo_amd.synthetic import synthetic_samples, synthetic_tokenizer
    cfg = full_config()
    col = Collate(synthetic_tokenizer(cfg), num_image_tokens_per_patch=cfg.img_tokens_per_tile,
                  num_image_patches=cfg.tiles, device="cuda:0")
    data = synthetic_samples(cfg, (warmup + steps) * B, s_text=s_text, n_loss=n_loss, seed=4242)
    loader = DataLoader(data, batch_size=B, shuffle=False, num_workers=workers, collate_fn=col.host,
                        prefetch_factor=2, persistent_workers=False)
    return dict(col=col, it=iter(loader), B=B, steps=steps, warmup=warmup, workers=workers, cfg=cfg)


def dropin_line(dl, dev):
    """The drop-in training loop, timed: per step one fresh collated batch (Collate.device on the DataLoader's host
    batch: H2D + HIP frames), DrivingModel.training_step -> loss.backward() -> FusedAdamW.step() ->
    OneCycleLR.step() -> zero_grad(), exactly the calls Lightning makes (driving.py:263-271, 718-732)."""
    from simlingo_amd.driving import DrivingModel
    from simlingo_amd.params import init_params
    cfg, col, it, B = dl["cfg"], dl["col"], dl["it"], dl["B"]
    variant = {"variant": "OpenGVLab/InternVL2-1B"}
    m = DrivingModel(vision_model=dict(variant), language_model=dict(variant, lora=True, lora_r=32, lora_alpha=64,
                                                                     lora_dropout=0.1),
                     lr=cfg.lr, init_params=init_params(cfg, seed=0, lora_b_std=0.02, device=dev))
    m.max_steps = 10000
    m.build_engine(dev)
    conf = m.configure_optimizers()
    opt, sched = conf["optimizer"], conf["lr_scheduler"]["scheduler"]

    sync = os.environ.get("SLX_DROPIN_SYNC", "0") == "1"  # debugging aid: synchronise after every step

    def step():
        ex = col.device(next(it))
        out = m.training_step(ex, 0)
        out["loss"].backward()
        opt.step()
        sched.step()
        opt.zero_grad()
        if sync:
            torch.cuda.synchronize()
        return out["loss"]

    losses = []
    for _ in range(dl["warmup"]):
        losses.append(step())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(dl["steps"]):
        losses.append(step())
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    loss = losses[-1]
    v = B * dl["steps"] / dt
    res = {"workload": "drop-in loop: DataLoader(workers run Collate.host) -> Collate.device (pinned H2D + HIP frames) "
                       "-> DrivingModel.training_step -> loss.backward() -> FusedAdamW.step -> OneCycleLR.step, "
                       "fresh batch per step, B=8, S_llm 798",
           "value": round(v, 3), "unit": "samples/s", "ms_per_step": round(dt / dl["steps"] * 1e3, 3),
           "steps": dl["steps"], "warmup": dl["warmup"], "loader_workers": dl["workers"],
           "step_mfma_frac": round(v * VLA_GFLOP_PER_SAMPLE / 1e3 / PEAK_BF16_TFLOPS, 4),
           "loss_last": round(loss.item(), 5), "losses": [round(x.item(), 4) for x in losses]}
    res["losses_finite"] = all(math.isfinite(x) for x in res["losses"])
    del m, opt, sched
    return res


def calibration(dev) -> dict:
    """the bf16 ceiling measured on this box beside the 2.5 PFLOP/s spec. `mfma_loop` = a bare
    back-to-back v_mfma_f32_32x32x16_bf16 loop on random register operands, one wave per SIMD on every CU (slx_mfma_peak:
    what the matrix cores sustain at the clock the chip holds under a bf16 load); `gemm_8192` = this library's own bf16
    GEMM (v3, NT) at M = N = K = 8192 on N(0, 1) operands. HIP events, median of 5."""
    from simlingo_amd import kernels as K

    def med(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e-3)
        return sorted(ts)[len(ts) // 2]

    grid, iters = 256 * 4, 20000
    out = torch.empty(grid * 256, device=dev)
    t = med(lambda: K.call("slx_mfma_peak", grid, iters, K.P(out), K.stream_ptr()))
    mfma = grid * 4 * iters * 4 * 32 * 32 * 16 * 2 / t / 1e12
    n = 8192
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.randn(n, n, device=dev, generator=g).bfloat16()
    b = torch.randn(n, n, device=dev, generator=g).bfloat16()
    c = torch.empty(n, n, device=dev, dtype=torch.bfloat16)
    tg = med(lambda: K.mm(a, b, c))
    del a, b, c, out
    gemm = 2.0 * n ** 3 / tg / 1e12
    return {"spec_peak_tflops": PEAK_BF16_TFLOPS, "mfma_loop_tflops": round(mfma, 1),
            "mfma_loop_frac_of_spec": round(mfma / PEAK_BF16_TFLOPS, 4), "gemm_8192_tflops": round(gemm, 1),
            "gemm_8192_frac_of_spec": round(gemm / PEAK_BF16_TFLOPS, 4),
            "note": "mfma_loop: bare back-to-back 32x32x16 bf16 MFMAs on random operands, all 1024 SIMDs (the clock "
                    "the chip holds under bf16 load); gemm_8192: this library's v3 GEMM at 8192^3"}


def traffic_record(tag, flop_M):
    """PMC-measured HBM bytes per FC1 launch (profiles/*_{tag}_fc1_traffic.json, newest first)."""
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", f"*{tag}_fc1_traffic.json")), reverse=True):
        try:
            rec = json.load(open(path))
        except Exception:
            continue
        if rec.get("M") == flop_M:
            return rec, os.path.relpath(path, ROOT)
    return None, None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dl = None
    if world == 1 and args.config == "vla" and not args.no_extras and not args.no_dropin:
        try:  # forks the loader workers now, before anything touches the GPU
            dl = dropin_loader()
        except Exception as e:
            dl = {"error": repr(e)[:200]}
    # rehearsal of the N > 1 path on a one-GPU box (the driver's scaling runs use one GPU per rank over RCCL):
    # SLX_BENCH_ONE_DEVICE=1 puts every rank on cuda:0 and SLX_BENCH_BACKEND=gloo exchanges the buckets through gloo
    # (RCCL refuses two ranks on one GPU)
    if os.environ.get("SLX_BENCH_ONE_DEVICE", "0") == "1":
        local = 0
    backend = os.environ.get("SLX_BENCH_BACKEND", "nccl")
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    args.wire_eff = "f32" if args.wire == "auto" else args.wire
    w = (setup_base if args.config.startswith("base") else setup_vla)(args, dev, world, rank)
    eng, step, B = w["eng"], w["step"], w["B"]
    if world > 1:
        import torch.distributed as dist
        dist.broadcast(eng.master, src=0)
        eng.wbf.copy_(eng.master.to(torch.bfloat16))
        eng._refresh_derived()
        eng.set_distributed(None, world)
    torch.cuda.synchronize()

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
    pr = w["probe"]
    eng.probe_site = ({"vit.fc1"} | ({pr["pair"]["site"]} if pr.get("pair") else set())) if pr else None
    eng.probe_events = {}
    if world > 1:
        eng.bucketer.timing = True  # device-clock exposed-communication tail (ddp.GradBucketer.comm_summary)
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
    cfg_out = dict(w["metric_cfg"])
    cfg_out.update(global_batch=B * world, per_gpu_batch=B, parallelism=f"dp{world}")
    res = {
        "metric": "training samples/sec (frame+prompt->waypoints)",
        "value": round(value, 3), "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic", "config": cfg_out,
        "loss_first": round(loss0, 5), "loss_last": round(loss_last, 5),
    }
    gf = w["gflop"]
    if gf:
        res["gflop_per_sample"] = round(gf, 1)
        res["step_mfma_frac"] = round(value * gf / 1e3 / (world * PEAK_BF16_TFLOPS), 4)
        res["step_tflops_per_gpu"] = round(value * gf / 1e3 / world, 1)
    if pr and eng.probe_events.get("vit.fc1"):
        ms = [a.elapsed_time(b) for a, b in eng.probe_events["vit.fc1"]]
        avg_ms = sum(ms) / len(ms)
        flop = 2.0 * pr["M"] * pr["N"] * pr["K"]
        ach = flop / (avg_ms * 1e-3) / 1e12
        rec, src = traffic_record(pr["tag"], pr["M"])
        fc1 = {"bound": "mfma", "kernel": pr["kernel"], "achieved": round(ach, 1), "peak": PEAK_BF16_TFLOPS,
               "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
               "traffic": rec["traffic_bytes"] if rec else None,
               "flop_per_launch": flop, "avg_launch_ms": round(avg_ms, 4), "launches": len(ms)}
        if rec:
            fc1["traffic_source"] = src
            fc1["algorithmic_bytes"] = rec.get("algorithmic_bytes")
        res["roofline"] = fc1
        pp = pr.get("pair")
        if pp and eng.probe_events.get(pp["site"]):  # the dominant kernel becomes `roofline`, FC1 stays beside it
            ms = [a.elapsed_time(b) for a, b in eng.probe_events[pp["site"]]]
            avg_ms = sum(ms) / len(ms)
            ach = pp["flop"] / (avg_ms * 1e-3) / 1e12
            prec, psrc = traffic_record(pr["tag"] + "_pair", pr["M"])
            res["roofline"] = {"bound": "mfma", "kernel": pp["kernel"], "achieved": round(ach, 1),
                               "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_BF16_TFLOPS, 4),
                               "traffic": prec["traffic_bytes"] if prec else None, "flop_per_launch": pp["flop"],
                               "avg_launch_ms": round(avg_ms, 4), "launches": len(ms),
                               "algorithmic_bytes": pp["algorithmic_bytes"]}
            if prec:
                res["roofline"]["traffic_source"] = psrc
            res["roofline_fc1"] = fc1
    if world > 1:
        res["dist_backend"] = "rccl" if backend == "nccl" else backend
        res["grad_wire"] = args.wire_eff
        cs = eng.bucketer.comm_summary()
        if cs:
            res["comm_exposed_ms"] = cs.pop("comm_exposed_ms")
            res["comm"] = cs
    if rank == 0 and world == 1 and args.config == "vla" and not args.no_extras:
        try:
            res["calibration"] = calibration(dev)
            res["step_frac_of_mfma_loop"] = round(res["step_mfma_frac"] * PEAK_BF16_TFLOPS
                                                  / res["calibration"]["mfma_loop_tflops"], 4)
        except Exception as e:
            res["calibration"] = {"error": repr(e)[:200]}
        if dl is not None and "error" not in dl:
            try:
                res["dropin"] = dropin_line(dl, dev)
                res["dropin"]["vs_value"] = round(res["dropin"]["value"] / value, 4)
            except Exception as e:
                res["dropin"] = {"error": repr(e)[:300]}
        elif dl is not None:
            res["dropin"] = dl
        try:
            res["config4"] = config4_step(args, dev)
        except Exception as e:  # the bench line must still be printed
            res["config4"] = {"error": repr(e)[:200]}
        try:
            res["agent"] = agent_latency(dev)
        except Exception as e:
            res["agent"] = {"error": repr(e)[:200]}
        try:
            res["base"] = base_line(args, dev)
        except Exception as e:
            res["base"] = {"error": repr(e)[:200]}
    if rank == 0 and world == 1 and w["cpu"] and not args.no_cpu_baseline:
        try:
            res["cpu_baseline"] = w["cpu"]()
        except Exception as e:  # the bench line must still be printed
            res["cpu_baseline"] = {"value": None, "error": repr(e)[:200]}
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
