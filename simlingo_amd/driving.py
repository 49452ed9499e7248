"""Drop-in DrivingModel for the SimLingo VLA hot path on MI355X.

Mirrors simlingo_training.models.driving.DrivingModel (simlingo_training/models/driving.py:40-732):
same constructor (cfg_data_module, processor, cache_dir, **cfg with the Hydra keys of
DrivingModelConfig, config.py:75-104), same methods forward_loss / training_step / forward /
configure_optimizers, same TrainingOutput. The arithmetic of forward_loss + backward is one
VLAEngine step (HIP kernels); autograd sees a single node so `loss.backward()` from Lightning (or a
plain loop) runs the hand-written backward, which also launches the bucketed RCCL all-reduce.
Subclasses pytorch_lightning.LightningModule when Lightning is installed, nn.Module otherwise.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from .config import VLAConfig, full_config, tiny_config
from .plan import plan_from_example
from .types import TrainingOutput

try:  # Lightning is optional (absent in this image); the surface is the same either way
    import pytorch_lightning as _pl
    _Base = _pl.LightningModule
except Exception:  # pragma: no cover - depends on the environment
    _Base = nn.Module


def _get(obj, key, default=None):
    if obj is None:
        return default
    if isinstance(obj, dict):
        return obj.get(key, default)
    return getattr(obj, key, default)


def geometry_for(variant: str, **overrides) -> VLAConfig:
    """InternVL2 variant string (config.py:42,65) -> kernel geometry."""
    v = (variant or "").lower()
    if "internvl2-1b" in v:
        return full_config(**overrides)
    if v in ("tiny", "simlingo-tiny"):
        return tiny_config(**overrides)
    raise ValueError(f"Unknown variant {variant}")  # same error type as vlm.py:24-25 / llm.py:94-95


class _VLAStep(torch.autograd.Function):
    """One autograd node for the whole hot path: forward = VLAEngine.forward, backward = VLAEngine.backward."""

    @staticmethod
    def forward(ctx, anchor, model, example, plan, dplan):
        eng = model.engine
        dev = eng.device
        di, lab = example.driving_input, example.driving_label
        path = dplan["path"] if "path" in dplan else lab.path.to(dev, non_blocking=True)
        wps = dplan["waypoints"] if "waypoints" in dplan else lab.waypoints.to(dev, non_blocking=True)
        out4, rp, sp = eng.forward(di.camera_images.to(dev, non_blocking=True), plan, dplan, path, wps,
                                   training=model.training)
        ctx.model = model
        model._last_predictions = {"route": rp, "speed_wps": sp}
        return out4

    @staticmethod
    def backward(ctx, dout4):
        ctx.model.engine.backward(dout4)
        return None, None, None, None, None


class DrivingModel(_Base):
    def __init__(self, cfg_data_module=None, processor=None, cache_dir=None, **cfg):
        super().__init__()
        for key, value in cfg.items():   # driving.py:51-52
            if key not in ("vision_model", "language_model"):
                setattr(self, key, value)
        self.cfg_data_module = cfg_data_module
        self.processor = processor
        self.cache_dir = cache_dir
        vm = cfg.get("vision_model", {"variant": "OpenGVLab/InternVL2-1B"})
        lm = cfg.get("language_model", {"variant": "OpenGVLab/InternVL2-1B"})
        # speed_wps_mode '1d' reads label.waypoints_1d, which simlingo_training's DrivingLabel does not carry, and
        # predict_route_as_wps=False leaves DrivingAdaptor.queries unset (adaptors.py:110-133): both fail in the
        # reference, so only the configuration it can run is accepted
        if _get(cfg, "speed_wps_mode", "2d") != "2d" or not _get(cfg, "predict_route_as_wps", True):
            raise NotImplementedError("speed_wps_mode='2d' with predict_route_as_wps=True is the configuration "
                                      "simlingo_training runs (adaptors.py:110-133, 189-199)")
        over = dict(vit_freeze=bool(_get(vm, "freeze", False)),
                    lora=bool(_get(lm, "lora", True)), lora_r=int(_get(lm, "lora_r", 32)),
                    lora_alpha=int(_get(lm, "lora_alpha", 64)), lora_dropout=float(_get(lm, "lora_dropout", 0.1)),
                    lr=float(cfg.get("lr", 3e-5)), weight_decay=float(cfg.get("weight_decay", 0.1)),
                    betas=tuple(cfg.get("betas", (0.9, 0.999))), pct_start=float(cfg.get("pct_start", 0.05)))
        if "grad_clip" in cfg:
            over["grad_clip"] = float(cfg["grad_clip"])
        self.vla_cfg = geometry_for(_get(lm, "variant", "OpenGVLab/InternVL2-1B"), **over)
        self.seed = int(cfg.get("seed", 0))
        self._init_params = cfg.get("init_params")  # optional {name: tensor} (tests, checkpoints)
        self.anchor = nn.Parameter(torch.zeros(()))  # autograd anchor of the fused step
        self.engine = None
        self.hidden_size = self.vla_cfg.llm_dim
        self._last_predictions = None
        self.predict_language = bool(cfg.get("predict_language", True))   # driving.py:58
        # inner seams (driving.py:62-96): the reference's submodules, served by the engine (simlingo_amd.vlm/adaptors)
        from .adaptors import AdaptorList
        from .vlm import LLM, VLMEncoderModel
        vkw = dict(vm) if isinstance(vm, dict) else {k: getattr(vm, k) for k in ("variant", "embed_dim", "freeze")
                                                        if hasattr(vm, k)}
        lkw = dict(lm) if isinstance(lm, dict) else {k: getattr(lm, k) for k in ("variant", "lora", "lora_alpha",
                                                                                  "lora_r", "lora_dropout") if hasattr(lm, k)}
        vkw.pop("_target_", None)
        lkw.pop("_target_", None)
        self.vision_model = VLMEncoderModel(cfg_data_module, processor, cache_dir, **vkw)._bind(self)
        self.language_model = LLM(**lkw)._bind(self)
        object.__setattr__(self, "adaptors", AdaptorList()._bind(self))
        self.max_new_tokens = int(cfg.get("max_new_tokens", 100))   # driving.py:147
        self._decoder = None
        self.sampled_tokens = None

    # ---- device placement ----------------------------------------------------------------------
    def build_engine(self, device=None):
        from .engine import VLAEngine
        if self.engine is None:
            dev = torch.device(device) if device is not None else (
                torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
            self.engine = VLAEngine(self.vla_cfg, dev, params=self._init_params, seed=self.seed)
            self._maybe_distributed()
        return self.engine

    def _maybe_distributed(self):
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            dist.broadcast(self.engine.master, src=0)
            self.engine.wbf.copy_(self.engine.master.to(torch.bfloat16))
            self.engine._refresh_derived()
            self.engine.set_distributed(None, dist.get_world_size())

    # ---- reference surface ----------------------------------------------------------------------
    def forward_loss(self, example, per_sample: bool = False):
        """driving.py:236-261 -> (TrainingOutput, loss_logs) or (loss_dict, pred_labels)."""
        eng = self.build_engine()
        plan = plan_from_example(self.vla_cfg, example)
        lab = example.driving_label
        # host-side labels ride in the plan's single pinned H2D copy (no pageable copy, no host sync per step)
        extra = {k: getattr(lab, k) for k in ("path", "waypoints") if not getattr(lab, k).is_cuda}
        dplan = plan.to_device(eng.device, extra=extra)
        out4 = _VLAStep.apply(self.anchor, self, example, plan, dplan)
        values, counts = self._per_sample_losses(eng, plan, dplan)
        averages = {"language_loss": out4[1], "route_loss": out4[2], "speed_wps_loss": out4[3]}
        preds = self._last_predictions
        if per_sample:  # driving.py:256-259: ({key: (values, counts)}, prediction labels)
            return ({k: (values[k], counts[k]) for k in values},
                    {"route_prediction": preds["route"], "speed_wps_prediction": preds["speed_wps"]})
        out = TrainingOutput(loss=out4[0], loss_averages=averages, loss_values=values, loss_counts=counts)
        return out, {}

    def _per_sample_losses(self, eng, plan, dplan):
        """summarise_losses inputs (models/utils.py:7-41, AdaptorList.compute_loss adaptors.py:333-355): language_loss
        CE per shifted label position [B, L-1] with its mask, route_loss [B, 20] and speed_wps_loss [B, 10] with ones
        counts - read from the engine's per-row loss buffers of this step (no host sync)."""
        sv = eng.saved
        cfg = self.vla_cfg
        B, L = plan.B, plan.L
        dev = eng.device
        lang = torch.zeros(B, max(L - 1, 0), dtype=torch.float32, device=dev)
        cnt = torch.zeros(B, max(L - 1, 0), dtype=torch.bool, device=dev)
        R = plan.loss_pos.shape[0]
        if R:
            bt = dplan["loss_bt"].long()
            lang[bt[:, 0], bt[:, 1]] = sv["ce_loss"][:R]
            cnt[bt[:, 0], bt[:, 1]] = True
        route = sv["route_loss"].view(B, cfg.n_route)
        speed = sv["speed_loss"].view(B, cfg.n_speed)
        values = {"language_loss": lang, "route_loss": route, "speed_wps_loss": speed}
        counts = {"language_loss": cnt, "route_loss": torch.ones_like(route), "speed_wps_loss": torch.ones_like(speed)}
        return values, counts

    def training_step(self, batch, _batch_idx: int = 0):
        """driving.py:263-271 (logging through Lightning when present; sync_dist scalars dropped)."""
        output, _ = self.forward_loss(batch)
        if _Base is not nn.Module:
            self.log("train/loss", output.loss.detach(), on_step=True, prog_bar=True, logger=True)
        return {"loss": output.loss, "outputs": output}

    def decoder(self):
        """The KV-cached greedy decoder (simlingo_amd.decode), built on first use."""
        from .decode import GreedyDecoder
        if self._decoder is None:
            self._decoder = GreedyDecoder(self.build_engine(), max_new_tokens=self.max_new_tokens)
        return self._decoder

    @torch.no_grad()
    def forward(self, example, return_language: Optional[bool] = None, prompt_ids=None):
        """driving.py:104-187 -> (speed_wps [B,10,2], route [B,20,2], language: List[str]).
        predict_language=True (the reference's setting, :58): greedy decode of up to max_new_tokens tokens
        per sample, then the driving forward over prompt + generated + queries (:131-176). The generated
        ids are kept in self.sampled_tokens; language strings are decoded with the processor's tokenizer
        when one was given (the InternVL2 tokenizer is not available offline), else the ids are joined.
        predict_language=False: the single training-style forward (:177-185)."""
        if self.predict_language:
            from .decode import infer_example
            eng = self.build_engine()
            sp, rp, toks = infer_example(eng, self.decoder(), example)
            self.sampled_tokens = toks
            tok = getattr(self.processor, "tokenizer", self.processor)
            if tok is not None and hasattr(tok, "batch_decode"):
                language = [tok.batch_decode([t], skip_special_tokens=True)[0] for t in toks]
            else:
                language = [" ".join(str(t) for t in ts) for ts in toks]
            return sp, rp, language
        eng = self.build_engine()
        plan = plan_from_example(self.vla_cfg, example, inference=True)
        dplan = plan.to_device(eng.device)
        di = example.driving_input if hasattr(example, "driving_input") else example
        B = di.camera_images.shape[0]
        lab = getattr(example, "driving_label", None)
        zeros_p = torch.zeros(B, self.vla_cfg.n_route, 2, device=eng.device)
        zeros_s = torch.zeros(B, self.vla_cfg.n_speed, self.vla_cfg.speed_dims, device=eng.device)
        path = lab.path.to(eng.device) if lab is not None else zeros_p
        wps = lab.waypoints.to(eng.device) if lab is not None else zeros_s
        _, rp, sp = eng.forward(di.camera_images.to(eng.device), plan, dplan, path, wps, training=False)
        eng.saved = None
        return sp, rp, []

    def configure_optimizers(self):
        """driving.py:718-732: AdamW(lr, weight_decay, betas) + OneCycleLR(interval='step')."""
        eng = self.build_engine()
        opt = FusedAdamW(self, lr=self.vla_cfg.lr, betas=self.vla_cfg.betas, weight_decay=self.vla_cfg.weight_decay,
                         eps=self.vla_cfg.eps, max_norm=self.vla_cfg.grad_clip)
        trainer = getattr(self, "_trainer", None)
        max_steps = getattr(self, "max_steps", None) or (
            getattr(trainer, "max_steps", -1) if trainer is not None else -1)
        if max_steps is None or max_steps <= 0:
            max_steps = int(getattr(trainer, "estimated_stepping_batches", 10000) or 10000) if trainer is not None else 10000
        sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=self.vla_cfg.lr, total_steps=int(max_steps),
                                                    pct_start=self.vla_cfg.pct_start)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": sched, "frequency": 1, "interval": "step"}}

    # ---- parameters in the reference's state-dict layout ------------------
    def vla_params(self) -> dict:
        """{internal name: f32 CPU tensor}: the engine's parameters, or the ones it will be built with."""
        if self.engine is not None:
            return self.engine.params_cpu()
        if self._init_params is None:
            from .params import init_params
            self._init_params = init_params(self.vla_cfg, self.seed)
        return {k: v.detach().float().cpu() for k, v in self._init_params.items()}

    def state_dict(self, *args, **kwargs):
        """The reference DrivingModel.state_dict() layout (vision_model.image_encoder.model..., language_model.model.
        base_model.model... with peft base_layer / lora_A.default / lora_B.default names, adaptors..., wp_encoder...,
        shared-module aliases included), so checkpoints round-trip with the reference trainer and agent
        (train.py:104-111, agent_simlingo.py:223). Frozen LLM weights come from the engine's bf16 copies."""
        from .checkpoint import to_reference
        prefix = kwargs.get("prefix", args[1] if len(args) > 1 else "") or ""
        return type(torch.nn.Module.state_dict(self))(
            (prefix + k, v) for k, v in to_reference(self.vla_params(), self.vla_cfg).items())

    def load_state_dict(self, state_dict, strict: bool = True, assign: bool = False):
        """Load a reference-layout state dict (flat, Lightning {'state_dict'}, DeepSpeed {'module'}, 'module.' /
        '_forward_module.' prefixes, or a ZeRO directory path / checkpoint file path). q/k/v and gate/up are fused,
        the engine (if built) is overwritten in place and its optimizer moments reset."""
        from torch.nn.modules.module import _IncompatibleKeys
        from .checkpoint import from_reference, load_checkpoint, to_reference
        from .checkpoint import _unwrap
        if isinstance(state_dict, str):
            state_dict = load_checkpoint(state_dict)
        missing, unexpected = [], []
        if strict:
            P = from_reference(state_dict, self.vla_cfg, strict=True)
        else:  # keys the dict does not carry keep their current values (torch's strict=False semantics)
            sd = _unwrap(state_dict)
            full = to_reference(self.vla_params(), self.vla_cfg, aliases=False)
            missing = [k for k in full if k not in sd]
            unexpected = [k for k in sd if k not in full and k not in to_reference(self.vla_params(), self.vla_cfg)]
            full.update({k: v for k, v in sd.items() if k in full})
            P = from_reference(full, self.vla_cfg, strict=True)
        if self.engine is not None:
            self.engine.load_params(P)
        else:
            self._init_params = P
        return _IncompatibleKeys(missing, unexpected)


class FusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics (decoupled weight decay on every parameter, as driving.py:719 uses
    self.parameters()) + global-norm clipping (train.py:206 gradient_clip_val=0.3), executed as one
    HIP kernel over the engine's flat fp32 master buffer. param_groups carry lr/betas so
    OneCycleLR (with its beta1 cycling) drives it exactly like the reference's optimizer."""

    def __init__(self, model: DrivingModel, lr=3e-5, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.1, max_norm=0.3):
        super().__init__([model.anchor], dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.model = model
        self.max_norm = max_norm
        self.step_count = 0

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        self.step_count += 1
        self.model.engine.adamw_step(g["lr"], self.step_count, betas=g["betas"], eps=g["eps"],
                                     weight_decay=g["weight_decay"], max_norm=self.max_norm)
        return loss

    def zero_grad(self, set_to_none: bool = True):
        # gradients are overwritten by every backward (no accumulation across steps)
        self.model.anchor.grad = None

    def state_dict(self):
        """AdamW's moments and step keyed by the reference's parameter names (simlingo_amd.optstate), so Lightning's
        `ckpt_path` resume (train.py:128-142,217) restores them: {format, state: {key: {step, exp_avg, exp_avg_sq}},
        param_groups (lr / betas / OneCycleLR's fields), step_count, max_norm, step_seed}."""
        from .checkpoint import trainable_ref_keys
        from .optstate import export_state
        return export_state(self, self.model.engine, trainable_ref_keys(self.model.vla_cfg))

    def load_state_dict(self, state_dict):
        from .checkpoint import trainable_ref_keys
        from .optstate import import_state
        import_state(self, self.model.build_engine(), trainable_ref_keys(self.model.vla_cfg), state_dict)
