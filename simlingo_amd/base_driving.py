"""Drop-in SimLingo-Base modules on MI355X (BASELINE.json configs[1]).

Mirrors the Hydra targets of simlingo_base_training (config.py:33-131, experiment/simlingo_base_1.yaml):
  * LLaVAnextEncoderModel(variant, embed_dim, freeze, downsample_feature_grid_factor, use_global_img)
    (models/encoder/llavanext.py:44-80) -> geometry of the CLIP ViT-L/14-336 tower + projector;
  * Llama(variant, lora) (models/language_model/llama.py:77-108) -> Llama CONFIGS geometry;
  * DrivingModel(vision_model, language_model, lr, vision_lr, weight_decay, betas, pct_start, ...)
    (models/driving.py:131-400) with forward / forward_loss / training_step / configure_optimizers.
The hub checkpoints are not loaded (no network); weights are seeded (base_params.init_base_params) or
passed as `init_params={name: tensor}`. forward_loss + backward is one BaseEngine step (HIP kernels):
autograd sees a single node, so `loss.backward()` runs the hand-written backward (and the bucketed RCCL
all-reduce under torch.distributed). The optimizer exposes the four param groups configure_params_groups
builds (driving.py:384-391: rest-decay, rest-no-decay, vision-decay, vision-no-decay) so OneCycleLR with
max_lr = [lr, lr, vision_lr, vision_lr] drives it as it drives the reference's AdamW.
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from .base_config import BaseConfig, base_config, base_tiny_config
from .types import TrainingOutput

try:  # Lightning is optional (absent in this image); the surface is the same either way
    import pytorch_lightning as _pl
    _Base = _pl.LightningModule
except Exception:  # pragma: no cover - depends on the environment
    _Base = nn.Module

# llama.py:43-60 CONFIGS whose head_dim is 64 (the attention kernels' head size)
_LLAMA = {"tiny": dict(llm_layers=12, llm_heads=8, llm_dim=512, llm_ffn=2048)}
_VISION = ("llava-hf/llava-v1.6-mistral-7b-hf", "llava-hf/llava-v1.6-vicuna-7b-hf")


class LLaVAnextEncoderModel(nn.Module):
    """Geometry holder for the vision encoder (llavanext.py:44-80). `variant='tiny'` selects the reduced test
    geometry of base_config.base_tiny_config."""

    def __init__(self, variant: str, embed_dim: int, freeze: bool, downsample_feature_grid_factor: int = 2,
                 use_global_img=False):
        super().__init__()
        if freeze:
            raise NotImplementedError("vision_model.freeze=True is not on the MI355X hot path (simlingo_base_1 trains it)")
        if use_global_img:
            raise NotImplementedError("use_global_img=True is not on the MI355X hot path (simlingo_base_1 uses False)")
        if variant not in _VISION and variant != "tiny":
            raise ValueError(f"Unknown vision variant {variant}")
        self.variant = variant
        self.num_cameras = 1
        self.num_frames = 1
        self.token_size = int(embed_dim)
        self.downsample_feature_grid_factor = int(downsample_feature_grid_factor)


class Llama(nn.Module):
    """Geometry holder for the language model (llama.py:77-108); `variant='debug-tiny'` is the reduced test
    geometry. LoRA is not part of the base recipe."""

    def __init__(self, variant: str, lora: bool = False):
        super().__init__()
        if lora:
            raise NotImplementedError("Llama(lora=True) is not on the MI355X hot path (simlingo_base_1 uses False)")
        if variant not in _LLAMA and variant != "debug-tiny":
            raise ValueError(f"Llama variant {variant} is not supported on MI355X (head_dim must be 64)")
        self.variant = variant
        self.geometry = dict(_LLAMA.get(variant, {}))
        self.hidden_size = self.geometry.get("llm_dim", 128)
        self.tokenizer = None   # the Llama-2 tokenizer is hub-only; the base path never tokenizes


class _BaseStep(torch.autograd.Function):
    """One autograd node for the whole base step: forward = BaseEngine.forward, backward = BaseEngine.backward."""

    @staticmethod
    def forward(ctx, anchor, model, example):
        eng = model.engine
        dev = eng.device
        di, lab = example.driving_input, example.driving_label
        size = tuple(int(v) for v in di.image_sizes[0]) if di.image_sizes is not None else None
        out4, rp, sp = eng.forward(di.camera_images.to(dev, non_blocking=True), di.vehicle_speed.to(dev),
                                   di.map_route.to(dev), lab.route_adjusted.to(dev), lab.waypoints.to(dev),
                                   image_size=size)
        ctx.model = model
        model._last_predictions = {"route": rp, "speed_wps": sp}
        return out4

    @staticmethod
    def backward(ctx, dout4):
        ctx.model.engine.backward(dout4)
        return None, None, None


class DrivingModel(_Base):
    def __init__(self, vision_model: nn.Module, language_model: nn.Module, lr: float = 1e-4,
                 vision_lr: Optional[float] = None, weight_decay: float = 0.1, betas=(0.9, 0.999),
                 pct_start: float = 0.05, enable_language=False, route_as="target_point", speed_as_input=True,
                 new_layer_norm_minmax=False, predict_route_as_wps=True, speed_wps_mode="2d", variant=None,
                 init_params=None, seed: int = 0):
        super().__init__()
        if route_as not in ("target_point", "coords"):
            raise NotImplementedError("route_as must be 'target_point' on the MI355X hot path (RouteEncode is a ResNet)")
        if not speed_as_input or not predict_route_as_wps or speed_wps_mode != "2d":
            raise NotImplementedError("MI355X base path implements speed_as_input, predict_route_as_wps, speed_wps_mode='2d'")
        self.vision_model = vision_model
        self.language_model = language_model
        self.lr = lr
        self.vision_lr = vision_lr if vision_lr is not None else lr
        self.weight_decay = weight_decay
        self.betas = tuple(betas)
        self.pct_start = pct_start
        self.enable_language = enable_language
        self.route_as = route_as
        self.speed_as_input = speed_as_input
        self.new_layer_norm_minmax = new_layer_norm_minmax
        self.predict_route_as_wps = predict_route_as_wps
        self.speed_wps_mode = speed_wps_mode
        over = dict(lr=float(lr), vision_lr=float(self.vision_lr), weight_decay=float(weight_decay), betas=self.betas,
                    pct_start=float(pct_start), embed_dim=vision_model.token_size,
                    pool=vision_model.downsample_feature_grid_factor, **language_model.geometry)
        if new_layer_norm_minmax:   # driving.py:197-212
            over.update(speed_max=110.0 / 3.6, tp_min=-200.0, tp_max=200.0)
        tiny = vision_model.variant == "tiny" or language_model.variant == "debug-tiny"
        self.base_cfg: BaseConfig = base_tiny_config(**over) if tiny else base_config(**over)
        if self.base_cfg.embed_dim != self.base_cfg.llm_dim:
            raise NotImplementedError("language_projection (embed_dim != hidden_size) is not on the MI355X hot path")
        self.hidden_size = self.base_cfg.llm_dim
        self.seed = int(seed)
        self._init_params = init_params
        self.anchor = nn.Parameter(torch.zeros(()))   # autograd anchor of the fused step
        self.engine = None
        self._last_predictions = None
        self.speed_wps, self.route, self.target_speed = None, None, None

    # ---- device placement ----------------------------------------------------------------------
    def build_engine(self, device=None):
        from .base_engine import BaseEngine
        if self.engine is None:
            dev = torch.device(device) if device is not None else (
                torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
            self.engine = BaseEngine(self.base_cfg, dev, params=self._init_params, seed=self.seed)
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
                dist.broadcast(self.engine.master, src=0)
                self.engine.wbf.copy_(self.engine.master.to(torch.bfloat16))
                self.engine._refresh_derived()
                self.engine.set_distributed(None, dist.get_world_size())
        return self.engine

    # ---- reference surface ----------------------------------------------------------------------
    def forward_loss(self, example, per_sample: bool = False):
        """driving.py:302-324 -> TrainingOutput (summarise_losses), or (loss_dict, pred_labels) per sample."""
        self.build_engine()
        out4 = _BaseStep.apply(self.anchor, self, example)
        preds = self._last_predictions
        if per_sample:
            lab = example.driving_label
            dev = preds["route"].device
            lr_ = lab.route_adjusted.to(dev)
            ls_ = lab.waypoints[:, :self.base_cfg.n_speed].to(dev)
            r = ((preds["route"] - lr_) ** 2).sum(-1).mean(-1)
            s = ((preds["speed_wps"] - ls_) ** 2).sum(-1).mean(-1)
            ones = torch.ones_like(r, dtype=torch.long)
            return ({"route_loss": (r, ones), "speed_wps_loss": (s, ones)},
                    {"route_prediction": preds["route"], "route_label": lr_,
                     "speed_wps_prediction": preds["speed_wps"], "speed_wps_label": ls_})
        B = preds["route"].shape[0]
        averages = {"route_loss": out4[2], "speed_wps_loss": out4[3]}
        counts = {k: torch.ones(B, dtype=torch.long) for k in averages}
        return TrainingOutput(loss=out4[0], loss_averages=averages, loss_values=averages, loss_counts=counts)

    def training_step(self, batch, _batch_idx: int = 0):
        """driving.py:326-333."""
        output = self.forward_loss(batch)
        if _Base is not nn.Module:
            self.log("train/loss", output.loss.detach(), on_step=True, prog_bar=True, logger=True)
        return {"loss": output.loss, "outputs": output}

    @torch.no_grad()
    def forward(self, driving_input, prompt_ids=None):
        """driving.py:231-251 -> (speed_wps [B,10,2], route [B,20,2]); the labels fed to the fused forward are
        zeros (the loss it also computes is discarded)."""
        eng = self.build_engine()
        di = driving_input.driving_input if hasattr(driving_input, "driving_input") else driving_input
        B = di.camera_images.shape[0]
        cfg = self.base_cfg
        size = tuple(int(v) for v in di.image_sizes[0]) if di.image_sizes is not None else None
        zr = torch.zeros(B, cfg.n_route, 2, device=eng.device)
        zs = torch.zeros(B, cfg.n_speed, cfg.speed_dims, device=eng.device)
        _, rp, sp = eng.forward(di.camera_images.to(eng.device), di.vehicle_speed.to(eng.device),
                                di.map_route.to(eng.device), zr, zs, image_size=size)
        eng.saved = None
        self.speed_wps, self.route = sp, rp
        return self.speed_wps, self.route

    def configure_optimizers(self):
        """driving.py:382-400: AdamW over configure_params_groups + OneCycleLR(max_lr=[per group], 'step')."""
        self.build_engine()
        opt = BaseFusedAdamW(self, lr=self.lr, vision_lr=self.vision_lr, betas=self.betas,
                             weight_decay=self.weight_decay, eps=self.base_cfg.eps, max_norm=self.base_cfg.grad_clip)
        trainer = getattr(self, "_trainer", None)
        max_steps = getattr(self, "max_steps", None) or (
            getattr(trainer, "max_steps", -1) if trainer is not None else -1)
        if max_steps is None or max_steps <= 0:
            max_steps = int(getattr(trainer, "estimated_stepping_batches", 10000) or 10000) if trainer is not None else 10000
        lrs = [pg["lr"] for pg in opt.param_groups]
        sched = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=lrs, total_steps=int(max_steps),
                                                    pct_start=self.pct_start)
        return {"optimizer": opt, "lr_scheduler": {"scheduler": sched, "frequency": 1, "interval": "step"}}

    def base_state_dict(self):
        """{reference state-dict key: fp32 tensor} of the engine's parameters (fused q/k/v and gate/up kept
        fused under a brace key, e.g. '...self_attn.{q,k,v}_proj.weight')."""
        eng = self.build_engine()
        return {s.ref: eng.P[s.name] for s in eng.specs}


class BaseFusedAdamW(torch.optim.Optimizer):
    """torch.optim.AdamW over the four configure_params_groups groups (in the reference's order: rest decay,
    rest no-decay, vision decay, vision no-decay) + global-norm clipping (train.py:189 gradient_clip_val 1.0),
    executed as the fused HIP AdamW over BaseEngine's four flat segments. Each group carries lr/betas so
    OneCycleLR drives it exactly like the reference's optimizer; group 0's betas are used (OneCycleLR cycles
    every group's momentum identically)."""

    def __init__(self, model: DrivingModel, lr=3e-5, vision_lr=3e-5, betas=(0.9, 0.999), eps=1e-8,
                 weight_decay=0.1, max_norm=1.0):
        anchors = [nn.Parameter(torch.zeros(())) for _ in range(3)]
        groups = [dict(params=[model.anchor], lr=lr, weight_decay=weight_decay),
                  dict(params=[anchors[0]], lr=lr, weight_decay=0.0),
                  dict(params=[anchors[1]], lr=vision_lr, weight_decay=weight_decay),
                  dict(params=[anchors[2]], lr=vision_lr, weight_decay=0.0)]
        super().__init__(groups, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.model = model
        self.max_norm = max_norm
        self.step_count = 0

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g0, g2 = self.param_groups[0], self.param_groups[2]
        self.step_count += 1
        self.model.engine.adamw_step(g0["lr"], g2["lr"], self.step_count, betas=g0["betas"], eps=g0["eps"],
                                     weight_decay=g0["weight_decay"], max_norm=self.max_norm)
        return loss

    def zero_grad(self, set_to_none: bool = True):
        # gradients are overwritten by every backward (no accumulation across steps)
        self.model.anchor.grad = None

    def _names(self):
        return {sp.name: (sp.ref, tuple(sp.shape)) for sp in self.model.build_engine().specs}

    def state_dict(self):
        """The four groups' AdamW moments and step keyed by the reference's state-dict names (simlingo_amd.optstate),
        for Lightning's ckpt_path resume."""
        from .optstate import export_state
        return export_state(self, self.model.engine, self._names())

    def load_state_dict(self, state_dict):
        from .optstate import import_state
        import_state(self, self.model.build_engine(), self._names(), state_dict)
