"""Parameter specification of the VLA hot path and its seeded initialisation.

Names are internal; `reference_key()` gives the reference's DrivingModel state-dict key for each
(InternVL2 remote layout + peft LoRA wrapping), so checkpoints can be mapped.
Frozen LLM weights are stored fused: qkv = [q; k; v] rows, gate_up = [gate; up] rows.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch

from .config import VLAConfig

LORA_SITES = ("q", "k", "v", "o", "gate", "up", "down")


@dataclass(frozen=True)
class PSpec:
    name: str
    shape: tuple
    trainable: bool
    init: str          # 'normal' | 'zeros' | 'ones' | 'ls' | 'query' | 'lora_a' | 'lora_b'
    group: str         # bucket / backward-order group


def lora_io(cfg: VLAConfig, site: str) -> tuple[int, int]:
    d, kv, f = cfg.llm_dim, cfg.llm_kv_heads * 64, cfg.llm_ffn
    return {"q": (d, d), "k": (d, kv), "v": (d, kv), "o": (d, d), "gate": (d, f), "up": (d, f), "down": (f, d)}[site]


def param_specs(cfg: VLAConfig) -> list[PSpec]:
    """Listed in backward-completion order (heads first, patch embedding last) so that gradient
    buckets are contiguous ranges of one flat buffer."""
    D, F, T = cfg.vit_dim, cfg.vit_ffn, cfg.vit_tokens
    d = cfg.llm_dim
    out: list[PSpec] = []
    a = out.append
    # driving heads (adaptors.py:110-136)
    m = cfg.head_mlp
    for nm, shp, init in (("route.0.w", (2 * m, d), "normal"), ("route.0.b", (2 * m,), "zeros"),
                          ("route.1.w", (m, 2 * m), "normal"), ("route.1.b", (m,), "zeros"),
                          ("route.2.w", (2, m), "normal"),
                          ("speed.0.w", (m, d), "normal"), ("speed.0.b", (m,), "zeros"),
                          ("speed.1.w", (cfg.speed_dims, m), "normal")):
        a(PSpec(nm, shp, True, init, "heads"))
    # frozen LLM (bf16 only)
    V = cfg.vocab
    a(PSpec("llm.lm_head", (V, d), False, "normal", "llm_frozen"))
    a(PSpec("llm.norm", (d,), False, "ones", "llm_frozen"))
    qkv_n = d + 2 * cfg.llm_kv_heads * 64
    for i in reversed(range(cfg.llm_layers)):
        p = f"llm.{i}."
        a(PSpec(p + "ln1", (d,), False, "ones", "llm_frozen"))
        a(PSpec(p + "qkv_w", (qkv_n, d), False, "normal", "llm_frozen"))
        a(PSpec(p + "qkv_b", (qkv_n,), False, "normal_small", "llm_frozen"))
        a(PSpec(p + "o_w", (d, d), False, "normal", "llm_frozen"))
        a(PSpec(p + "ln2", (d,), False, "ones", "llm_frozen"))
        a(PSpec(p + "gate_up_w", (2 * cfg.llm_ffn, d), False, "normal", "llm_frozen"))
        a(PSpec(p + "down_w", (d, cfg.llm_ffn), False, "normal", "llm_frozen"))
        if cfg.lora:
            for s in LORA_SITES:
                fin, fout = lora_io(cfg, s)
                a(PSpec(p + f"lora.{s}.a", (cfg.lora_r, fin), True, "lora_a", f"llm{i}"))
                a(PSpec(p + f"lora.{s}.b", (fout, cfg.lora_r), True, "lora_b", f"llm{i}"))
    a(PSpec("llm.embed", (V, d), False, "normal", "llm_frozen"))
    # token assembly inputs: driving queries (adjacent, [30, d]) and wp_encoder (driving.py:91-96)
    a(PSpec("drv.query_route", (cfg.n_route, d), True, "query", "assembly"))
    a(PSpec("drv.query_speed", (cfg.n_speed, d), True, "query", "assembly"))
    a(PSpec("wp.0.w", (cfg.wp_hidden, 2), True, "normal", "assembly"))
    a(PSpec("wp.0.b", (cfg.wp_hidden,), True, "zeros", "assembly"))
    a(PSpec("wp.1.w", (cfg.wp_hidden2, cfg.wp_hidden), True, "normal", "assembly"))
    a(PSpec("wp.1.b", (cfg.wp_hidden2,), True, "zeros", "assembly"))
    a(PSpec("wp.2.w", (d, cfg.wp_hidden2), True, "normal", "assembly"))
    a(PSpec("wp.2.b", (d,), True, "zeros", "assembly"))
    # mlp1 projector
    a(PSpec("proj.ln.w", (4 * D,), True, "ones", "proj"))
    a(PSpec("proj.ln.b", (4 * D,), True, "zeros", "proj"))
    a(PSpec("proj.fc1.w", (d, 4 * D), True, "normal", "proj"))
    a(PSpec("proj.fc1.b", (d,), True, "zeros", "proj"))
    a(PSpec("proj.fc2.w", (d, d), True, "normal", "proj"))
    a(PSpec("proj.fc2.b", (d,), True, "zeros", "proj"))
    # InternViT layers, last first (vision_model.freeze: requires_grad False for all but mlp1, encoder/vlm.py:36-44)
    vt = not cfg.vit_freeze
    for i in reversed(range(cfg.vit_layers)):
        p = f"vit.{i}."
        g = f"vit{i}"
        a(PSpec(p + "ln1.w", (D,), vt, "ones", g)); a(PSpec(p + "ln1.b", (D,), vt, "zeros", g))
        a(PSpec(p + "qkv.w", (3 * D, D), vt, "normal", g)); a(PSpec(p + "qkv.b", (3 * D,), vt, "zeros", g))
        a(PSpec(p + "proj.w", (D, D), vt, "normal", g)); a(PSpec(p + "proj.b", (D,), vt, "zeros", g))
        a(PSpec(p + "ls1", (D,), vt, "ls", g))
        a(PSpec(p + "ln2.w", (D,), vt, "ones", g)); a(PSpec(p + "ln2.b", (D,), vt, "zeros", g))
        a(PSpec(p + "fc1.w", (F, D), vt, "normal", g)); a(PSpec(p + "fc1.b", (F,), vt, "zeros", g))
        a(PSpec(p + "fc2.w", (D, F), vt, "normal", g)); a(PSpec(p + "fc2.b", (D,), vt, "zeros", g))
        a(PSpec(p + "ls2", (D,), vt, "ls", g))
    a(PSpec("vit.cls", (D,), vt, "normal", "vit_embed"))
    a(PSpec("vit.pos", (T, D), vt, "normal", "vit_embed"))
    a(PSpec("vit.patch.w", (D, cfg.patch_k), vt, "normal", "vit_embed"))
    a(PSpec("vit.patch.b", (D,), vt, "zeros", "vit_embed"))
    return out


def init_params(cfg: VLAConfig, seed: int = 0, lora_b_std: float = 0.0, std: float = 0.02,
                device="cpu") -> dict[str, torch.Tensor]:
    """Seeded fp32 CPU initialisation. Weights N(0, std) (HF default initializer_range 0.02), biases 0,
    norms 1, layer scale ls_init (InternViT), queries 0.02*randn (adaptors.py:112,129),
    LoRA A kaiming-uniform(a=sqrt(5)) as peft; LoRA B N(0, lora_b_std) (peft inits B = 0; a non-zero
    B exercises the LoRA path in parity runs)."""
    import zlib
    out = {}
    for s in param_specs(cfg):
        # one generator per parameter: values do not depend on the order of the spec list
        g = torch.Generator(device=device).manual_seed(seed * 1000003 + zlib.crc32(s.name.encode()))
        kw = dict(generator=g, device=device)
        if s.init == "normal":
            t = torch.randn(s.shape, **kw) * std
        elif s.init == "normal_small":
            t = torch.randn(s.shape, **kw) * std
        elif s.init == "zeros":
            t = torch.zeros(s.shape, device=device)
        elif s.init == "ones":
            t = torch.ones(s.shape, device=device)
        elif s.init == "ls":
            t = torch.full(s.shape, cfg.ls_init, device=device)
        elif s.init == "query":
            t = 0.02 * torch.randn(s.shape, **kw)
        elif s.init == "lora_a":
            bound = 1.0 / math.sqrt(s.shape[1])  # kaiming_uniform(a=sqrt(5)) on fan_in
            t = (torch.rand(s.shape, **kw) * 2 - 1) * bound
        elif s.init == "lora_b":
            t = torch.randn(s.shape, **kw) * lora_b_std
        else:
            raise ValueError(s.init)
        out[s.name] = t.float().contiguous()
    return out


def reference_key(name: str) -> str:
    """Internal name -> reference DrivingModel state-dict key (fused tensors map to several keys)."""
    vit = "vision_model.image_encoder.model.vision_model."
    llm = "language_model.model.base_model.model."
    parts = name.split(".")
    if name == "vit.cls":
        return vit + "embeddings.class_embedding"
    if name == "vit.pos":
        return vit + "embeddings.position_embedding"
    if name.startswith("vit.patch."):
        return vit + "embeddings.patch_embedding." + ("weight" if parts[-1] == "w" else "bias")
    if name.startswith("vit."):
        i, rest = parts[1], ".".join(parts[2:])
        m = {"ln1.w": "norm1.weight", "ln1.b": "norm1.bias", "qkv.w": "attn.qkv.weight", "qkv.b": "attn.qkv.bias",
             "proj.w": "attn.proj.weight", "proj.b": "attn.proj.bias", "ls1": "ls1", "ln2.w": "norm2.weight",
             "ln2.b": "norm2.bias", "fc1.w": "mlp.fc1.weight", "fc1.b": "mlp.fc1.bias", "fc2.w": "mlp.fc2.weight",
             "fc2.b": "mlp.fc2.bias", "ls2": "ls2"}[rest]
        return f"{vit}encoder.layers.{i}.{m}"
    if name.startswith("proj."):
        m = {"ln.w": "0.weight", "ln.b": "0.bias", "fc1.w": "1.weight", "fc1.b": "1.bias", "fc2.w": "3.weight",
             "fc2.b": "3.bias"}[".".join(parts[1:])]
        return "vision_model.image_encoder.model.mlp1." + m
    if name == "llm.embed":
        return llm + "model.embed_tokens.weight"
    if name == "llm.lm_head":
        return llm + "lm_head.weight"
    if name == "llm.norm":
        return llm + "model.norm.weight"
    if name.startswith("llm."):
        i, rest = parts[1], ".".join(parts[2:])
        base = f"{llm}model.layers.{i}."
        if rest.startswith("lora."):
            site, ab = parts[3], parts[4]
            mod = {"q": "self_attn.q_proj", "k": "self_attn.k_proj", "v": "self_attn.v_proj", "o": "self_attn.o_proj",
                   "gate": "mlp.gate_proj", "up": "mlp.up_proj", "down": "mlp.down_proj"}[site]
            return f"{base}{mod}.lora_{ab.upper()}.default.weight"
        m = {"ln1": "input_layernorm.weight", "ln2": "post_attention_layernorm.weight",
             "qkv_w": "self_attn.{q,k,v}_proj.base_layer.weight", "qkv_b": "self_attn.{q,k,v}_proj.base_layer.bias",
             "o_w": "self_attn.o_proj.base_layer.weight", "gate_up_w": "mlp.{gate,up}_proj.base_layer.weight",
             "down_w": "mlp.down_proj.base_layer.weight"}[rest]
        return base + m
    if name.startswith("drv."):
        return "adaptors.driving." + {"query_route": "query_embeds_wps", "query_speed": "query_embeds_speed"}[parts[1]]
    if name.startswith("route.") or name.startswith("speed."):
        head = "route_head" if parts[0] == "route" else "speed_wps_head"
        return f"adaptors.driving.{head}.{2 * int(parts[1])}.{'weight' if parts[2] == 'w' else 'bias'}"
    if name.startswith("wp."):
        return f"wp_encoder.mlp.{2 * int(parts[1])}.{'weight' if parts[2] == 'w' else 'bias'}"
    raise KeyError(name)
