"""Optimizer state of the fused AdamW kernels in a torch-style state dict, for resume.

The reference resumes with `trainer.fit(model, dm, ckpt_path=resume_path)` (simlingo_training/train.py:128-142,217):
Lightning restores the model's state dict, then `optimizer.load_state_dict(...)` and the scheduler's, so AdamW
continues with its moments and bias-correction step (configure_optimizers, models/driving.py:718-732). The engines keep
m / v as flat f32 buffers beside the master weights; this module cuts them into per-parameter tensors keyed by the
reference's state-dict names ({key: {"step", "exp_avg", "exp_avg_sq"}}, torch.optim.AdamW's per-parameter fields)
and writes them back. The engine's dropout-mask counter (step_seed) rides along, so a resumed run draws the same LoRA
dropout masks as an uninterrupted one.
"""
from __future__ import annotations

import math

import torch

FORMAT = "simlingo_amd.fused_adamw/1"


def export_state(opt: torch.optim.Optimizer, eng, names: dict) -> dict:
    """names: {internal trainable name: (reference key, reference shape)}."""
    groups = [{k: v for k, v in g.items() if k != "params"} for g in opt.param_groups]
    state = {}
    if eng is not None and hasattr(eng, "m_state"):
        torch.cuda.current_stream(eng.device).synchronize()
        step = torch.tensor(float(opt.step_count))
        for name, (key, shape) in names.items():
            o, n = eng.offsets[name], math.prod(shape)
            state[key] = {"step": step.clone(),
                          "exp_avg": eng.m_state[o:o + n].detach().view(shape).cpu(),
                          "exp_avg_sq": eng.v_state[o:o + n].detach().view(shape).cpu()}
    return {"format": FORMAT, "state": state, "param_groups": groups, "step_count": int(opt.step_count),
            "max_norm": opt.max_norm, "step_seed": int(getattr(eng, "step_seed", 0)) if eng is not None else 0}


def import_state(opt: torch.optim.Optimizer, eng, names: dict, sd: dict) -> None:
    if sd.get("format") != FORMAT:
        raise ValueError(f"not a {FORMAT} optimizer state (format {sd.get('format')!r})")
    if len(sd["param_groups"]) != len(opt.param_groups):
        raise ValueError(f"{len(sd['param_groups'])} saved param groups, the optimizer has {len(opt.param_groups)}")
    for g, saved in zip(opt.param_groups, sd["param_groups"]):
        g.update({k: v for k, v in saved.items() if k != "params"})
    opt.step_count = int(sd["step_count"])
    opt.max_norm = sd.get("max_norm", opt.max_norm)
    state = sd["state"]
    if eng is None:
        raise RuntimeError("build the engine (model.build_engine()) before loading optimizer state")
    eng.step_seed = int(sd.get("step_seed", eng.step_seed))
    if not state:  # saved before the first step: no moments yet
        for attr in ("m_state", "v_state"):
            if hasattr(eng, attr):
                delattr(eng, attr)
        return
    missing = [key for key, _ in names.values() if key not in state]
    unexpected = sorted(set(state) - {key for key, _ in names.values()})
    if missing or unexpected:
        raise KeyError(f"optimizer state does not match the model: missing {missing[:4]} ({len(missing)}), "
                       f"unexpected {unexpected[:4]} ({len(unexpected)})")
    if not hasattr(eng, "m_state"):
        eng.m_state = torch.zeros_like(eng.master)
        eng.v_state = torch.zeros_like(eng.master)
        eng.sumsq = torch.zeros(1, dtype=torch.float32, device=eng.device)
    with torch.no_grad():
        for name, (key, shape) in names.items():
            o, n = eng.offsets[name], math.prod(shape)
            ent = state[key]
            for fld, dst in (("exp_avg", eng.m_state), ("exp_avg_sq", eng.v_state)):
                t = ent[fld]
                if tuple(t.shape) != tuple(shape):
                    raise ValueError(f"{key}.{fld}: shape {tuple(t.shape)} != {tuple(shape)}")
                dst[o:o + n].copy_(t.reshape(-1).to(eng.device, torch.float32), non_blocking=False)
