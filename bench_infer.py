"""Closed-loop agent latency on one MI355X (BASELINE.json configs[4]): team_code/agent_simlingo.py's call of
DrivingModel.forward (driving.py:104-187) at bs=1 — InternViT on the 2 tiles of one 1024x512 frame, the
prompt prefill, greedy decode of up to 100 tokens (llm.py:178-250, KV-cached here), then the driving forward
over prompt + generated + 30 queries and the route / speed heads.

    python bench_infer.py [--frames 5] [--warmup 1] [--new-tokens 100] [--s-text 64]

Synthetic seeded frame + prompt, random-init weights of the InternVL2-1B geometry (no checkpoint offline); a
random model never emits EOS, so every frame decodes the full max_new_tokens (the worst case). Prints one
JSON line: per-frame latency (median), its phases, decode ms/token and the decode step's HBM rate
(weight bytes streamed per token / decode step time, against the 8 TB/s peak); the decode time is taken
with HIP events around the graph-replayed steps inside GreedyDecoder.generate.
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


def measure(dev, frames=5, warmup=1, new_tokens=100, s_text=64) -> dict:
    from simlingo_amd.config import full_config
    from simlingo_amd.decode import GreedyDecoder
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.params import init_params
    from simlingo_amd.plan import plan_from_example
    from simlingo_amd.synthetic import make_batch

    cfg = full_config()
    eng = VLAEngine(cfg, dev, init_params(cfg, seed=0, lora_b_std=0.02, device=dev))
    dec = GreedyDecoder(eng, max_len=1024, max_new_tokens=new_tokens, eos_id=cfg.eos_id)
    ex = make_batch(cfg, B=1, s_text=s_text, n_loss=1, seed=7)
    pix = ex.driving_input.camera_images.to(dev)
    NQ = cfg.n_queries

    def frame():
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        ev[0].record()
        plan = plan_from_example(cfg, ex, inference=True)
        dplan = plan.to_device(dev)
        X = eng.encode_inputs(pix, plan, dplan, {})
        nv = int(plan.seqlens[0]) - NQ
        prefix, queries = X[:nv], X[nv:nv + NQ]
        ev[1].record()
        toks = dec.generate(prefix)
        ev[2].record()
        dec.drive(prefix, queries, toks)
        ev[3].record()
        torch.cuda.synchronize()
        return [ev[0].elapsed_time(ev[1]), ev[1].elapsed_time(ev[2]), ev[2].elapsed_time(ev[3])], len(toks), nv, \
            dict(dec.last_timing)

    for _ in range(warmup):
        frame()
    rows = []
    for _ in range(frames):
        t0 = time.perf_counter()
        ph, n, nv, tm = frame()
        rows.append(((time.perf_counter() - t0) * 1e3, ph, n, tm))
    rows.sort(key=lambda r: r[0])
    wall, ph, n, tm = rows[len(rows) // 2]
    step_ms = tm["decode_ms"] / max(tm["decode_steps"], 1)
    d, F = cfg.llm_dim, cfg.llm_ffn
    w_bytes = cfg.llm_layers * 2 * (dec.nqkv * d + d * dec.qn + 2 * F * d + d * F) + 2 * cfg.vocab * d
    return {
        "metric": "closed-loop agent latency per frame (DrivingModel.forward, greedy decode)", "value": round(wall, 2),
        "unit": "ms", "higher_is_better": False, "n_gpus": 1, "batch": 1, "dtype": "bf16", "data": "synthetic",
        "config": {"workload": "InternViT-300M x2 tiles + Qwen2-0.5B (LoRA merged) greedy decode + driving forward",
                   "prompt_tokens": nv, "new_tokens": n, "max_new_tokens": new_tokens},
        "phases_ms": {"encode_vit_assembly": round(ph[0], 2), "prefill": round(tm["prefill_ms"], 2),
                      "decode": round(tm["decode_ms"], 2), "driving_forward": round(ph[2], 2)},
        "decode_ms_per_token": round(step_ms, 4),
        "decode_roofline": {"bound": "hbm", "bytes_per_token": w_bytes,
                            "achieved": round(w_bytes / (step_ms * 1e-3) / 1e9, 1), "peak": 8000.0, "unit": "GB/s",
                            "frac": round(w_bytes / (step_ms * 1e-3) / 8e12, 4)},
        "frames": frames,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--new-tokens", type=int, default=100)
    ap.add_argument("--s-text", type=int, default=64)
    args = ap.parse_args()
    res = measure(torch.device("cuda", 0), frames=args.frames, warmup=args.warmup, new_tokens=args.new_tokens,
                  s_text=args.s_text)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
