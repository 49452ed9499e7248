"""Checkpoint compatibility with the reference DrivingModel.

The reference warm-starts from a flat state dict or a DeepSpeed ZeRO directory
(simlingo_training/train.py:104-111: `get_fp32_state_dict_from_zero_checkpoint(dir)` or `torch.load(file)`,
then `model.load_state_dict(state_dict)`), and the closed-loop agent loads a flat state dict
(team_code/agent_simlingo.py:223). Its keys follow the module tree of
  DrivingModel (models/driving.py:40-103)
    vision_model = VLMEncoderModel -> image_encoder = LingoInternVLModel -> model = InternVLChatModel (remote code,
                   language_model set to None, encoder/vlm.py:27-31): vision_model.{embeddings, encoder.layers.i}, mlp1
    language_model = LLM -> model = peft(Qwen2ForCausalLM) (language_model/llm.py:88-119): peft 0.13.2 wraps every
                   Linear except lm_head as {base_layer, lora_A.default, lora_B.default}; llm.py:91-93 aliases
                   `embed_tokens` onto the causal-LM module, so its weight appears twice
    adaptors = AdaptorList(language=LanguageAdaptor (holds embed_tokens / lm_head again, adaptors.py:225-233),
                           driving=DrivingAdaptor (adaptors.py:96-136))
    wp_encoder = WaypointInputAdaptor (adaptors.py:73-80)
This module maps that layout to the engine's parameters and back: the InternViT qkv stays fused (the remote code
stores it fused), Qwen2 q/k/v and gate/up are fused on load and split on save, the class / position embeddings and
the driving queries lose / regain their leading singleton dims, the patch-embedding Conv2d weight is flattened to
the im2col GEMM operand [1024, 3*14*14]. Key names are pinned by tests/golden/ckpt_keys.json, generated from the
reference's own adaptor modules + transformers' Qwen2ForCausalLM (oracle/gen_golden_ckpt.py).
"""
from __future__ import annotations

import glob
import os
import re
from collections import OrderedDict

import torch

from .config import VLAConfig
from .params import LORA_SITES, lora_io, param_specs

VIT = "vision_model.image_encoder.model.vision_model."
MLP1 = "vision_model.image_encoder.model.mlp1."
LLM = "language_model.model.base_model.model."
_VIT_LAYER = {"ln1.w": "norm1.weight", "ln1.b": "norm1.bias", "qkv.w": "attn.qkv.weight", "qkv.b": "attn.qkv.bias",
              "proj.w": "attn.proj.weight", "proj.b": "attn.proj.bias", "ls1": "ls1", "ln2.w": "norm2.weight",
              "ln2.b": "norm2.bias", "fc1.w": "mlp.fc1.weight", "fc1.b": "mlp.fc1.bias", "fc2.w": "mlp.fc2.weight",
              "fc2.b": "mlp.fc2.bias", "ls2": "ls2"}
_MLP1 = {"proj.ln.w": "0.weight", "proj.ln.b": "0.bias", "proj.fc1.w": "1.weight", "proj.fc1.b": "1.bias",
         "proj.fc2.w": "3.weight", "proj.fc2.b": "3.bias"}
_SITE_MOD = {"q": "self_attn.q_proj", "k": "self_attn.k_proj", "v": "self_attn.v_proj", "o": "self_attn.o_proj",
             "gate": "mlp.gate_proj", "up": "mlp.up_proj", "down": "mlp.down_proj"}
_HEADS = {"route.0.w": "route_head.0.weight", "route.0.b": "route_head.0.bias", "route.1.w": "route_head.2.weight",
          "route.1.b": "route_head.2.bias", "route.2.w": "route_head.4.weight", "speed.0.w": "speed_wps_head.0.weight",
          "speed.0.b": "speed_wps_head.0.bias", "speed.1.w": "speed_wps_head.2.weight"}
_WP = {f"wp.{i}.{t}": f"wp_encoder.mlp.{2 * i}.{'weight' if t == 'w' else 'bias'}" for i in range(3) for t in "wb"}
# keys that alias another key's tensor in the reference module tree (shared modules)
ALIASES = {LLM + "embed_tokens.weight": LLM + "model.embed_tokens.weight",
           "adaptors.language.embed_tokens.weight": LLM + "model.embed_tokens.weight",
           "adaptors.language.lm_head.weight": LLM + "lm_head.weight"}


def to_reference(P: dict, cfg: VLAConfig, aliases: bool = True) -> "OrderedDict[str, torch.Tensor]":
    """Engine parameters {internal name: tensor} -> the reference DrivingModel.state_dict() layout."""
    D, d = cfg.vit_dim, cfg.llm_dim
    qn, kn, F = cfg.llm_heads * 64, cfg.llm_kv_heads * 64, cfg.llm_ffn
    sd: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    sd[VIT + "embeddings.class_embedding"] = P["vit.cls"].reshape(1, 1, D)
    sd[VIT + "embeddings.patch_embedding.weight"] = P["vit.patch.w"].reshape(D, 3, cfg.patch, cfg.patch)
    sd[VIT + "embeddings.patch_embedding.bias"] = P["vit.patch.b"]
    sd[VIT + "embeddings.position_embedding"] = P["vit.pos"].reshape(1, cfg.vit_tokens, D)
    for i in range(cfg.vit_layers):
        for k, v in _VIT_LAYER.items():
            sd[f"{VIT}encoder.layers.{i}.{v}"] = P[f"vit.{i}.{k}"]
    for k, v in _MLP1.items():
        sd[MLP1 + v] = P[k]
    sd[LLM + "model.embed_tokens.weight"] = P["llm.embed"]
    for i in range(cfg.llm_layers):
        p, base = f"llm.{i}.", f"{LLM}model.layers.{i}."
        lin = "base_layer." if cfg.lora else ""
        q, k, v = P[p + "qkv_w"].split([qn, kn, kn], 0)
        qb, kb, vb = P[p + "qkv_b"].split([qn, kn, kn], 0)
        g, u = P[p + "gate_up_w"].split([F, F], 0)
        weights = {"q": (q, qb), "k": (k, kb), "v": (v, vb), "o": (P[p + "o_w"], None), "gate": (g, None),
                   "up": (u, None), "down": (P[p + "down_w"], None)}
        sd[base + "input_layernorm.weight"] = P[p + "ln1"]
        for site in LORA_SITES:
            w, b = weights[site]
            mod = base + _SITE_MOD[site] + "."
            sd[mod + lin + "weight"] = w
            if b is not None:
                sd[mod + lin + "bias"] = b
            if cfg.lora:
                sd[mod + "lora_A.default.weight"] = P[p + f"lora.{site}.a"]
                sd[mod + "lora_B.default.weight"] = P[p + f"lora.{site}.b"]
        sd[base + "post_attention_layernorm.weight"] = P[p + "ln2"]
    sd[LLM + "model.norm.weight"] = P["llm.norm"]
    sd[LLM + "lm_head.weight"] = P["llm.lm_head"]
    sd["adaptors.driving.query_embeds_wps"] = P["drv.query_route"].reshape(1, cfg.n_route, d)
    for k, v in _HEADS.items():
        if k.startswith("route"):
            sd["adaptors.driving." + v] = P[k]
    sd["adaptors.driving.query_embeds_speed"] = P["drv.query_speed"].reshape(1, cfg.n_speed, d)
    for k, v in _HEADS.items():
        if k.startswith("speed"):
            sd["adaptors.driving." + v] = P[k]
    for k, v in _WP.items():
        sd[v] = P[k]
    if aliases:
        for a, src in ALIASES.items():
            sd[a] = sd[src]
    return sd


def trainable_ref_keys(cfg: VLAConfig) -> "OrderedDict[str, tuple[str, tuple]]":
    """{internal trainable name: (reference state-dict key, reference shape)} — the keys to_reference gives each
    trainable tensor (its class / position / patch / query reshapes included). Optimizer state is keyed by these, so
    a checkpoint's moments line up with the reference's parameter names (FusedAdamW.state_dict)."""
    D, d = cfg.vit_dim, cfg.llm_dim
    special = {"vit.cls": (VIT + "embeddings.class_embedding", (1, 1, D)),
               "vit.patch.w": (VIT + "embeddings.patch_embedding.weight", (D, 3, cfg.patch, cfg.patch)),
               "vit.patch.b": (VIT + "embeddings.patch_embedding.bias", (D,)),
               "vit.pos": (VIT + "embeddings.position_embedding", (1, cfg.vit_tokens, D)),
               "drv.query_route": ("adaptors.driving.query_embeds_wps", (1, cfg.n_route, d)),
               "drv.query_speed": ("adaptors.driving.query_embeds_speed", (1, cfg.n_speed, d))}
    out: "OrderedDict[str, tuple[str, tuple]]" = OrderedDict()
    for s in param_specs(cfg):
        if not s.trainable:
            continue
        n = s.name
        if n in special:
            out[n] = special[n]
            continue
        m = re.fullmatch(r"vit\.(\d+)\.(.+)", n)
        l = re.fullmatch(r"llm\.(\d+)\.lora\.(\w+)\.([ab])", n)
        if m:
            key = f"{VIT}encoder.layers.{m.group(1)}.{_VIT_LAYER[m.group(2)]}"
        elif l:
            key = (f"{LLM}model.layers.{l.group(1)}.{_SITE_MOD[l.group(2)]}."
                   f"lora_{'A' if l.group(3) == 'a' else 'B'}.default.weight")
        elif n in _MLP1:
            key = MLP1 + _MLP1[n]
        elif n in _HEADS:
            key = "adaptors.driving." + _HEADS[n]
        elif n in _WP:
            key = _WP[n]
        else:
            raise KeyError(f"no reference key for trainable parameter {n}")
        out[n] = (key, tuple(s.shape))
    return out


def _unwrap(sd) -> dict:
    """Lightning checkpoint {'state_dict': ...} / DeepSpeed {'module': ...} / DDP 'module.' / Lightning-DeepSpeed
    '_forward_module.' prefixes -> plain DrivingModel keys."""
    for key in ("state_dict", "module"):
        if isinstance(sd, dict) and key in sd and isinstance(sd[key], dict):
            sd = sd[key]
    out = {}
    for k, v in sd.items():
        k = re.sub(r"^(_forward_module\.|module\.)+", "", k)
        out[k] = v
    return out


def from_reference(sd, cfg: VLAConfig, strict: bool = True) -> dict:
    """Reference DrivingModel state dict -> engine parameters {internal name: f32 CPU tensor}. strict: every engine
    parameter must be found and every key must be known (aliases must equal their source tensor)."""
    sd = _unwrap(sd)
    want = to_reference({s.name: torch.empty(s.shape) for s in param_specs(cfg)}, cfg)
    missing = [k for k in want if k not in sd and k not in ALIASES]
    unexpected = [k for k in sd if k not in want]
    if strict and (missing or unexpected):
        raise KeyError(f"state dict does not match the SimLingo VLA layout: missing {missing[:8]}"
                       f"{'...' if len(missing) > 8 else ''} ({len(missing)}), unexpected {unexpected[:8]}"
                       f"{'...' if len(unexpected) > 8 else ''} ({len(unexpected)})")
    for k, want_t in want.items():
        if k in sd and tuple(sd[k].shape) != tuple(want_t.shape):
            raise ValueError(f"{k}: shape {tuple(sd[k].shape)} != expected {tuple(want_t.shape)}")
    for a, src in ALIASES.items():
        if a in sd and src in sd and not torch.equal(sd[a].float(), sd[src].float()):
            raise ValueError(f"{a} must alias {src} (shared module in the reference) but differs")
    f = lambda k: sd[k].detach().to("cpu", torch.float32)  # noqa: E731
    D, d = cfg.vit_dim, cfg.llm_dim
    P = {"vit.cls": f(VIT + "embeddings.class_embedding").reshape(D),
         "vit.patch.w": f(VIT + "embeddings.patch_embedding.weight").reshape(D, cfg.patch_k),
         "vit.patch.b": f(VIT + "embeddings.patch_embedding.bias"),
         "vit.pos": f(VIT + "embeddings.position_embedding").reshape(cfg.vit_tokens, D)}
    for i in range(cfg.vit_layers):
        for k, v in _VIT_LAYER.items():
            P[f"vit.{i}.{k}"] = f(f"{VIT}encoder.layers.{i}.{v}")
    for k, v in _MLP1.items():
        P[k] = f(MLP1 + v)
    P["llm.embed"] = f(LLM + "model.embed_tokens.weight")
    lin = "base_layer." if cfg.lora else ""
    for i in range(cfg.llm_layers):
        p, base = f"llm.{i}.", f"{LLM}model.layers.{i}."
        m = {site: base + _SITE_MOD[site] + "." for site in LORA_SITES}
        P[p + "ln1"] = f(base + "input_layernorm.weight")
        P[p + "ln2"] = f(base + "post_attention_layernorm.weight")
        P[p + "qkv_w"] = torch.cat([f(m[s] + lin + "weight") for s in ("q", "k", "v")], 0)
        P[p + "qkv_b"] = torch.cat([f(m[s] + lin + "bias") for s in ("q", "k", "v")], 0)
        P[p + "o_w"] = f(m["o"] + lin + "weight")
        P[p + "gate_up_w"] = torch.cat([f(m["gate"] + lin + "weight"), f(m["up"] + lin + "weight")], 0)
        P[p + "down_w"] = f(m["down"] + lin + "weight")
        if cfg.lora:
            for site in LORA_SITES:
                P[p + f"lora.{site}.a"] = f(m[site] + "lora_A.default.weight")
                P[p + f"lora.{site}.b"] = f(m[site] + "lora_B.default.weight")
    P["llm.norm"] = f(LLM + "model.norm.weight")
    P["llm.lm_head"] = f(LLM + "lm_head.weight")
    P["drv.query_route"] = f("adaptors.driving.query_embeds_wps").reshape(cfg.n_route, d)
    P["drv.query_speed"] = f("adaptors.driving.query_embeds_speed").reshape(cfg.n_speed, d)
    for k, v in _HEADS.items():
        P[k] = f("adaptors.driving." + v)
    for k, v in _WP.items():
        P[k] = f(v)
    return P


# ---- weights-only loading of DeepSpeed / Lightning checkpoint files ---------------------------------------------------
# A real ZeRO-2 checkpoint of the reference (train.py:160-168, DeepSpeed 0.16.2 under Lightning 2.4) pickles more than
# tensors: the optimizer state holds a LossScaler / DynamicLossScaler instance, a ZeroStageEnum and, per group, an
# OrderedDict of tensor_fragment.fragment_address records; the model-states file holds ds_config and Lightning's
# client state (hyper_parameters, possibly omegaconf containers). torch's weights-only unpickler rejects every such
# global. They are mapped here to INERT stand-ins: a stand-in records its constructor arguments and pickled state and
# runs nothing (the real class is never imported, no code from the file executes). Only globals under the known
# DeepSpeed / Lightning / OmegaConf packages get one; any other global keeps the weights-only error, named.
_STANDIN_PREFIXES = ("deepspeed.", "pytorch_lightning.", "lightning.", "lightning_fabric.", "omegaconf.")


class _Inert:
    """Inert stand-in for a checkpoint object: keeps args / state as data, executes nothing."""
    _qualname = "?"

    def __init__(self, *args, **kwargs):
        self._args, self._kwargs = args, kwargs

    def __setstate__(self, state):
        self._state = state

    def __repr__(self):
        return f"<inert {self._qualname}>"


def _standin(qualname: str):
    return type(qualname.rsplit(".", 1)[-1], (_Inert,), {"_qualname": qualname, "__module__": __name__})


def safe_load(path: str, max_standins: int = 64):
    """torch.load(path, weights_only=True), with inert stand-ins for the DeepSpeed / Lightning / OmegaConf globals a
    reference checkpoint contains. Raises pickle.UnpicklingError naming any other unsupported global."""
    import pickle
    extra = []
    for _ in range(max_standins):
        try:
            with torch.serialization.safe_globals(extra):
                return torch.load(path, map_location="cpu", weights_only=True)
        except pickle.UnpicklingError as e:
            # a dict / list subclass (e.g. Lightning's AttributeDict) fills itself with SETITEM(S) / APPEND(S), which the
            # weights-only unpickler allows only on plain containers: stand in with the plain container instead
            # (torch 2.10 wording: 'Can only SETITEMS for dicts...' / 'Can only append to lists' / 'Can only extend lists')
            m = re.search(r"Can only (SETITEMS?|APPENDS?|append to lists|extend lists)[^<]*but got <class '[\w.]*\.(\w+)'>",
                          str(e))
            if m:
                i = next((j for j, (c, q) in enumerate(extra) if c.__name__ == m.group(2) and issubclass(c, _Inert)), None)
                if i is None:
                    raise
                extra[i] = (dict if m.group(1).startswith("SETITEM") else list, extra[i][1])
                continue
            m = re.search(r"GLOBAL ([\w.]+) was not an allowed global", str(e))
            if not m:
                raise
            name = m.group(1)
            if not name.startswith(_STANDIN_PREFIXES) or any(q == name for _, q in extra):
                raise pickle.UnpicklingError(f"{path}: unsupported object {name} in a weights-only load (only "
                                             f"{', '.join(_STANDIN_PREFIXES)} objects get inert stand-ins)") from None
            extra.append((_standin(name), name))
    raise pickle.UnpicklingError(f"{path}: more than {max_standins} non-tensor globals")


# ---- DeepSpeed ZeRO stage 1/2 directory -> consolidated fp32 state dict -------------------------------------------
def consolidate_zero(ckpt_dir: str) -> "OrderedDict[str, torch.Tensor]":
    """Restatement of deepspeed 0.16.2 `utils/zero_to_fp32.get_fp32_state_dict_from_zero_checkpoint` for ZeRO stage
    1/2 (the reference's strategy, config.py:298-299; deepspeed is not installed here, so this follows its published
    file format and is unpinned by a real DeepSpeed checkpoint). Layout: <dir>/latest names a tag subdirectory (or
    <dir> is the tag directory) holding mp_rank_00_model_states.pt (module: buffers and frozen params; param_shapes:
    [OrderedDict(name -> shape)] per optimizer group) and one *_optim_states.pt per data-parallel rank
    (optimizer_state_dict.single_partition_of_fp32_groups: that rank's fp32 slice of each flat group). Each group's
    slices are concatenated in rank order and cut into the named parameters in param_shapes order. Every file is
    read by safe_load (weights-only, inert stand-ins for the DeepSpeed / Lightning objects the files hold)."""
    tag_dir = ckpt_dir
    latest = os.path.join(ckpt_dir, "latest")
    if os.path.isfile(latest):
        tag_dir = os.path.join(ckpt_dir, open(latest).read().strip())
    model_files = sorted(glob.glob(os.path.join(tag_dir, "*mp_rank_00_model_states.pt")))
    def _rank(path):  # zero_pp_rank_{dp_rank}_mp_rank_00_optim_states.pt (numeric order, not alphabetical)
        m = re.search(r"(?:pp|dp)_rank_(\d+)_mp_rank", os.path.basename(path))
        return int(m.group(1)) if m else 0
    optim_files = sorted(glob.glob(os.path.join(tag_dir, "*_optim_states.pt")), key=_rank)
    if not model_files or not optim_files:
        raise FileNotFoundError(f"{tag_dir}: no mp_rank_00_model_states.pt / *_optim_states.pt (not a ZeRO dir)")
    ms = safe_load(model_files[0])
    out: "OrderedDict[str, torch.Tensor]" = OrderedDict()
    for k, v in (ms.get("module") or {}).items():  # buffers / frozen params saved in the module state
        out[k] = v.float() if torch.is_tensor(v) and v.is_floating_point() else v
    for k, v in (ms.get("frozen_param_fragments") or {}).items():
        out[k] = v.float()
    shapes = ms["param_shapes"]
    if isinstance(shapes, dict):
        shapes = [shapes]
    parts = [safe_load(p)["optimizer_state_dict"]["single_partition_of_fp32_groups"] for p in optim_files]
    for g, group_shapes in enumerate(shapes):
        flat = torch.cat([rank_parts[g].float().reshape(-1) for rank_parts in parts])
        off = 0
        for name, shape in group_shapes.items():
            n = int(torch.Size(shape).numel())
            out[name] = flat[off:off + n].view(tuple(shape)).clone()
            off += n
        if off > flat.numel():
            raise ValueError(f"group {g}: {off} elements in param_shapes but only {flat.numel()} saved")
    return out


def load_checkpoint(path: str) -> dict:
    """train.py:104-111: a ZeRO directory (consolidated) or a single torch file (loaded with weights_only=True)."""
    if os.path.isdir(path):
        return consolidate_zero(path)
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        return load_file(path)
    return safe_load(path)
