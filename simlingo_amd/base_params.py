"""Parameters of the SimLingo-Base path: specification, optimizer grouping and seeded initialisation.

Every parameter that receives a gradient in the reference is trainable (vision_model.freeze False,
Llama without LoRA, simlingo_base_1.yaml). The CLIP tower's last layer and post_layernorm get no gradient
(hidden_states[-2] is read, llavanext_model.py:98) — torch's AdamW skips parameters whose .grad is None,
so they are not part of the optimised set here either (they are not even computed).

Optimizer groups follow configure_params_groups (simlingo_base_training/models/utils.py:47-150) with the
two ParamGroups of DrivingModel.configure_optimizers (driving.py:372-376): weight decay only on the
weights of Linear / Conv2d modules, none on biases, norms, embeddings, image_newline, class_embedding,
temporal/camera encodings, query embeddings and anything under route_head; lr = vision_lr under
`vision_model.`, lr elsewhere. The flat f32 master buffer is laid out as four contiguous segments
(non-vision decay | vision decay | vision no-decay | non-vision no-decay), each in backward-completion
order, so the optimizer is four launches of the fused AdamW kernel and DDP buckets stay contiguous.
"""
from __future__ import annotations

import math
import zlib
from dataclasses import dataclass

import torch

from .base_config import BaseConfig


@dataclass(frozen=True)
class BSpec:
    name: str
    shape: tuple
    init: str         # normal | zeros | ones | small
    decay: bool
    vision: bool
    group: str        # DDP bucket group (backward-completion order)
    ref: str          # reference state-dict key (simlingo_base_training DrivingModel)


def base_specs(cfg: BaseConfig) -> list[BSpec]:
    """All trainable parameters, in backward-completion order (before segmenting)."""
    D, F, d, Fl = cfg.vit_dim, cfg.vit_ffn, cfg.llm_dim, cfg.llm_ffn
    P, E, m, h = cfg.proj_dim, cfg.embed_dim, cfg.head_mlp, cfg.in_hidden
    out: list[BSpec] = []

    def a(name, shape, init, decay, vision, group, ref):
        out.append(BSpec(name, tuple(shape), init, decay, vision, group, ref))

    drv = "adaptors.driving."
    a("route.0.w", (m, d), "normal", False, False, "heads", drv + "route_head.0.weight")
    a("route.0.b", (m,), "zeros", False, False, "heads", drv + "route_head.0.bias")
    a("route.1.w", (2, m), "normal", False, False, "heads", drv + "route_head.2.weight")
    a("speed.0.w", (m, d), "normal", True, False, "heads", drv + "speed_wps_head.0.weight")
    a("speed.0.b", (m,), "zeros", False, False, "heads", drv + "speed_wps_head.0.bias")
    a("speed.1.w", (cfg.speed_dims, m), "normal", True, False, "heads", drv + "speed_wps_head.2.weight")
    lm = "language_model.model."
    a("llm.norm", (d,), "ones", False, False, "llm", lm + "norm.weight")
    for i in reversed(range(cfg.llm_layers)):
        p, r, g = f"llm.{i}.", f"{lm}layers.{i}.", f"llm{i}"
        a(p + "down_w", (d, Fl), "normal", True, False, g, r + "mlp.down_proj.weight")
        a(p + "gate_up_w", (2 * Fl, d), "normal", True, False, g, r + "mlp.{gate,up}_proj.weight")
        a(p + "ln2", (d,), "ones", False, False, g, r + "post_attention_layernorm.weight")
        a(p + "o_w", (d, d), "normal", True, False, g, r + "self_attn.o_proj.weight")
        a(p + "qkv_w", (3 * d, d), "normal", True, False, g, r + "self_attn.{q,k,v}_proj.weight")
        a(p + "ln1", (d,), "ones", False, False, g, r + "input_layernorm.weight")
    a("drv.query_route", (cfg.n_route, d), "small", False, False, "inputs", drv + "query_embeds_wps")
    a("drv.query_speed", (cfg.n_speed, d), "small", False, False, "inputs", drv + "query_embeds_speed")
    for tag, ref, k in (("spd", "speed_encoder", 1), ("rte", "route_encoder", 2)):
        a(f"{tag}.0.w", (h, k), "normal", True, False, "inputs", f"{ref}.mlp.0.weight")
        a(f"{tag}.0.b", (h,), "zeros", False, False, "inputs", f"{ref}.mlp.0.bias")
        a(f"{tag}.1.w", (d, h), "normal", True, False, "inputs", f"{ref}.mlp.2.weight")
        a(f"{tag}.1.b", (d,), "zeros", False, False, "inputs", f"{ref}.mlp.2.bias")
    vm = "vision_model."
    a("enc.proj.w", (E, P), "normal", True, True, "venc", vm + "projection.weight")
    a("enc.proj.b", (E,), "zeros", False, True, "venc", vm + "projection.bias")
    a("enc.temporal", (E,), "small", False, True, "venc", vm + "temporal_encoding")
    a("enc.camera", (E,), "small", False, True, "venc", vm + "camera_encoding")
    ie = vm + "image_encoder."
    a("mm.newline", (P,), "small", False, True, "venc", ie + "image_newline")
    a("mm.fc2.w", (P, P), "normal", True, True, "venc", ie + "multi_modal_projector.linear_2.weight")
    a("mm.fc2.b", (P,), "zeros", False, True, "venc", ie + "multi_modal_projector.linear_2.bias")
    a("mm.fc1.w", (P, D), "normal", True, True, "venc", ie + "multi_modal_projector.linear_1.weight")
    a("mm.fc1.b", (P,), "zeros", False, True, "venc", ie + "multi_modal_projector.linear_1.bias")
    vt = ie + "vision_tower.vision_model."
    for i in reversed(range(cfg.vit_used)):
        p, r, g = f"vit.{i}.", f"{vt}encoder.layers.{i}.", f"vit{i}"
        a(p + "fc2.w", (D, F), "normal", True, True, g, r + "mlp.fc2.weight")
        a(p + "fc2.b", (D,), "zeros", False, True, g, r + "mlp.fc2.bias")
        a(p + "fc1.w", (F, D), "normal", True, True, g, r + "mlp.fc1.weight")
        a(p + "fc1.b", (F,), "zeros", False, True, g, r + "mlp.fc1.bias")
        a(p + "ln2.w", (D,), "ones", False, True, g, r + "layer_norm2.weight")
        a(p + "ln2.b", (D,), "zeros", False, True, g, r + "layer_norm2.bias")
        a(p + "proj.w", (D, D), "normal", True, True, g, r + "self_attn.out_proj.weight")
        a(p + "proj.b", (D,), "zeros", False, True, g, r + "self_attn.out_proj.bias")
        a(p + "qkv.w", (3 * D, D), "normal", True, True, g, r + "self_attn.{q,k,v}_proj.weight")
        a(p + "qkv.b", (3 * D,), "zeros", False, True, g, r + "self_attn.{q,k,v}_proj.bias")
        a(p + "ln1.w", (D,), "ones", False, True, g, r + "layer_norm1.weight")
        a(p + "ln1.b", (D,), "zeros", False, True, g, r + "layer_norm1.bias")
    ve = vt + "embeddings."
    a("vit.pre_ln.w", (D,), "ones", False, True, "vit_embed", vt + "pre_layrnorm.weight")
    a("vit.pre_ln.b", (D,), "zeros", False, True, "vit_embed", vt + "pre_layrnorm.bias")
    a("vit.cls", (D,), "small", False, True, "vit_embed", ve + "class_embedding")
    a("vit.pos", (cfg.vit_tokens, D), "small", False, True, "vit_embed", ve + "position_embedding.weight")
    a("vit.patch.w", (D, cfg.patch_k), "normal", True, True, "vit_embed", ve + "patch_embedding.weight")
    return out


SEGMENTS = (("decay", False), ("decay", True), ("nodecay", True), ("nodecay", False))


def segment_of(s: BSpec) -> int:
    return SEGMENTS.index(("decay" if s.decay else "nodecay", s.vision))


def flat_layout(cfg: BaseConfig, align: int = 64):
    """-> (ordered specs, offsets {name: start}, segment bounds [(start, end)] x 4, total, group of each spec).
    No-decay parameters all join one DDP group ('nodecay', completed after the whole backward)."""
    specs = base_specs(cfg)
    ordered = sorted(specs, key=lambda s: segment_of(s))  # stable: keeps backward order inside a segment
    offs, bounds, off = {}, [], 0
    for k in range(len(SEGMENTS)):
        a = off
        for s in ordered:
            if segment_of(s) == k:
                offs[s.name] = off
                off += (math.prod(s.shape) + align - 1) // align * align
        bounds.append((a, off))
    groups = {s.name: (s.group if s.decay else "nodecay") for s in specs}
    return ordered, offs, bounds, off, groups


def init_base_params(cfg: BaseConfig, seed: int = 0, std: float = 0.02, device="cpu") -> dict[str, torch.Tensor]:
    """Seeded fp32 initialisation (HF-style: Linear/Conv N(0, std), biases 0, norms 1, embeddings and
    encodings 0.02 randn, llavanext.py:60-61, adaptors.py:117,128)."""
    out = {}
    for s in base_specs(cfg):
        g = torch.Generator(device=device).manual_seed(seed * 1000003 + zlib.crc32(s.name.encode()))
        if s.init == "normal":
            t = torch.randn(s.shape, generator=g, device=device) * std
        elif s.init == "small":
            t = torch.randn(s.shape, generator=g, device=device) * 0.02
        elif s.init == "zeros":
            t = torch.zeros(s.shape, device=device)
        elif s.init == "ones":
            t = torch.ones(s.shape, device=device)
        else:
            raise ValueError(s.init)
        out[s.name] = t.float().contiguous()
    return out
