"""Generate the golden fixtures tests/golden/vla_tiny_*.npz from the REFERENCE code.

ORACLE TOOLING — test infrastructure only; runs in the build container where /root/reference exists:
    python oracle/gen_golden.py

What runs here is the reference's own Python for everything that is importable offline
(SURVEY.md §8c): AdaptorList / DrivingAdaptor / LanguageAdaptor / WaypointInputAdaptor
(simlingo_training/models/adaptors/adaptors.py), LingoInternVLModel.replace_placeholder_tokens
(simlingo_training/models/encoder/internvl2_model.py:17-144) and summarise_losses
(simlingo_training/models/utils.py). The InternVL2-1B remote code cannot be downloaded, so its
arithmetic is supplied by the transformers implementations that mirror it: InternVLVisionModel
(InternViT, use_mean_pooling=True -> no final norm), InternVLModel.pixel_shuffle (ps v2),
InternVLMultiModalProjector (mlp1) and Qwen2ForCausalLM (eager attention, rope_theta 1e6); peft is
absent, so LoRA is the 10-line restatement `LoraLinear` below (y = Wx + b + (alpha/r) B A x).
DrivingModel.forward_model/forward_loss (driving.py:190-261) need hydra/lightning to import, so
their 20 lines of glue are restated in `reference_forward_loss` with line references.
Geometry: tiny_config (head_dim 64), plus one full-width case `full1`: the InternVL2-1B widths
(InternViT 1024 x 16 heads at T = 1025, mlp1 4096 -> 896, Qwen2 896 with GQA 14/2, FFN 4864, V = 151655, LoRA r32)
with ONE InternViT and ONE Qwen2 layer, B = 2 with left padding, S_text = 256 (S_llm = 798). Its inputs are not
stored (make_batch is seeded; a checksum of every input is); its gradients as digests. Everything fp32 on the CPU.
"""
from __future__ import annotations

import json
import os
import sys
import types as pytypes

import numpy as np
import torch
from torch import nn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REF = os.environ.get("SIMLINGO_REFERENCE", "/root/reference")
sys.path.insert(0, REF)

from simlingo_training.models.adaptors.adaptors import (AdaptorList, DrivingAdaptor,  # noqa: E402
                                                       LanguageAdaptor, WaypointInputAdaptor)
from simlingo_training.models.encoder.internvl2_model import LingoInternVLModel  # noqa: E402
from simlingo_training.models.utils import summarise_losses  # noqa: E402
from simlingo_training.utils import custom_types as RT  # noqa: E402
from transformers import (InternVLConfig, InternVLVisionConfig, InternVLVisionModel, Qwen2Config,  # noqa: E402
                          Qwen2ForCausalLM)
from transformers.models.internvl.modeling_internvl import InternVLModel, InternVLMultiModalProjector  # noqa: E402

from simlingo_amd.config import full_config, tiny_config  # noqa: E402
from simlingo_amd.params import init_params, param_specs  # noqa: E402
from simlingo_amd.synthetic import make_batch  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")


class LoraLinear(nn.Module):
    """peft LoraLayer forward (dropout off): base(x) + lora_B(lora_A(x)) * lora_alpha / r."""

    def __init__(self, base: nn.Linear, a: torch.Tensor, b: torch.Tensor, scale: float):
        super().__init__()
        self.base_layer = base
        self.lora_A = nn.Linear(a.shape[1], a.shape[0], bias=False)
        self.lora_B = nn.Linear(b.shape[1], b.shape[0], bias=False)
        self.lora_A.weight.data.copy_(a)
        self.lora_B.weight.data.copy_(b)
        self.scale = scale

    def forward(self, x):
        return self.base_layer(x) + self.lora_B(self.lora_A(x)) * self.scale


def build_reference(cfg, P):
    D, d = cfg.vit_dim, cfg.llm_dim
    vcfg = InternVLVisionConfig(hidden_size=D, num_hidden_layers=cfg.vit_layers, num_attention_heads=cfg.vit_heads,
                                attention_bias=True, intermediate_size=cfg.vit_ffn, hidden_act="gelu",
                                layer_norm_eps=cfg.vit_eps, image_size=cfg.img_size, patch_size=cfg.patch,
                                layer_scale_init_value=cfg.ls_init, use_mean_pooling=True)
    vit = InternVLVisionModel(vcfg).float().eval()
    sd = {"embeddings.cls_token": P["vit.cls"].view(1, 1, D), "embeddings.position_embeddings": P["vit.pos"][None],
          "embeddings.patch_embeddings.projection.weight": P["vit.patch.w"].view(D, 3, cfg.patch, cfg.patch),
          "embeddings.patch_embeddings.projection.bias": P["vit.patch.b"]}
    for i in range(cfg.vit_layers):
        p, q = f"vit.{i}.", f"encoder.layer.{i}."
        for j, n in enumerate(("q_proj", "k_proj", "v_proj")):
            sd[q + f"attention.{n}.weight"] = P[p + "qkv.w"][j * D:(j + 1) * D]
            sd[q + f"attention.{n}.bias"] = P[p + "qkv.b"][j * D:(j + 1) * D]
        sd[q + "attention.projection_layer.weight"] = P[p + "proj.w"]
        sd[q + "attention.projection_layer.bias"] = P[p + "proj.b"]
        sd[q + "lambda_1"], sd[q + "lambda_2"] = P[p + "ls1"], P[p + "ls2"]
        sd[q + "layernorm_before.weight"], sd[q + "layernorm_before.bias"] = P[p + "ln1.w"], P[p + "ln1.b"]
        sd[q + "layernorm_after.weight"], sd[q + "layernorm_after.bias"] = P[p + "ln2.w"], P[p + "ln2.b"]
        for n in ("fc1", "fc2"):
            sd[q + f"mlp.{n}.weight"], sd[q + f"mlp.{n}.bias"] = P[p + f"{n}.w"], P[p + f"{n}.b"]
    vit.load_state_dict(sd, strict=True)
    tcfg = Qwen2Config(hidden_size=d, num_hidden_layers=cfg.llm_layers, num_attention_heads=cfg.llm_heads,
                       num_key_value_heads=cfg.llm_kv_heads, intermediate_size=cfg.llm_ffn, vocab_size=cfg.vocab,
                       rope_theta=cfg.rope_theta, rms_norm_eps=cfg.rms_eps, tie_word_embeddings=False,
                       max_position_embeddings=4096, attn_implementation="eager")
    try:
        tcfg.rope_parameters = {"rope_type": "default", "rope_theta": cfg.rope_theta}
    except Exception:
        pass
    icfg = InternVLConfig(vision_config=vcfg, text_config=tcfg, downsample_ratio=0.5, projector_hidden_act="gelu")
    proj = InternVLMultiModalProjector(icfg).float().eval()
    proj.load_state_dict({"layer_norm.weight": P["proj.ln.w"], "layer_norm.bias": P["proj.ln.b"],
                          "linear_1.weight": P["proj.fc1.w"], "linear_1.bias": P["proj.fc1.b"],
                          "linear_2.weight": P["proj.fc2.w"], "linear_2.bias": P["proj.fc2.b"]})
    proj.layer_norm.eps = cfg.proj_eps
    qwen = Qwen2ForCausalLM(tcfg).float().eval()
    H, Hk = cfg.llm_heads * 64, cfg.llm_kv_heads * 64
    sd = {"model.embed_tokens.weight": P["llm.embed"], "lm_head.weight": P["llm.lm_head"], "model.norm.weight": P["llm.norm"]}
    for i in range(cfg.llm_layers):
        p, q = f"llm.{i}.", f"model.layers.{i}."
        w, b = P[p + "qkv_w"], P[p + "qkv_b"]
        for n, sl in (("q_proj", slice(0, H)), ("k_proj", slice(H, H + Hk)), ("v_proj", slice(H + Hk, H + 2 * Hk))):
            sd[q + f"self_attn.{n}.weight"], sd[q + f"self_attn.{n}.bias"] = w[sl], b[sl]
        sd[q + "self_attn.o_proj.weight"] = P[p + "o_w"]
        F_ = cfg.llm_ffn
        sd[q + "mlp.gate_proj.weight"], sd[q + "mlp.up_proj.weight"] = P[p + "gate_up_w"][:F_], P[p + "gate_up_w"][F_:]
        sd[q + "mlp.down_proj.weight"] = P[p + "down_w"]
        sd[q + "input_layernorm.weight"], sd[q + "post_attention_layernorm.weight"] = P[p + "ln1"], P[p + "ln2"]
    qwen.load_state_dict(sd, strict=True)
    if cfg.lora:  # get_peft_model(target_modules="all-linear") minus lm_head
        for i in range(cfg.llm_layers):
            layer = qwen.model.layers[i]
            for site, parent, attr in (("q", layer.self_attn, "q_proj"), ("k", layer.self_attn, "k_proj"),
                                       ("v", layer.self_attn, "v_proj"), ("o", layer.self_attn, "o_proj"),
                                       ("gate", layer.mlp, "gate_proj"), ("up", layer.mlp, "up_proj"),
                                       ("down", layer.mlp, "down_proj")):
                setattr(parent, attr, LoraLinear(getattr(parent, attr), P[f"llm.{i}.lora.{site}.a"],
                                                 P[f"llm.{i}.lora.{site}.b"], cfg.lora_scale))
    qwen.embed_tokens = qwen.model.embed_tokens  # llm.py:277-278 (LanguageAdaptor reads .embed_tokens)

    def extract_feature(pixel_values):  # remote InternVLChatModel.extract_feature, select_layer -1
        x = vit(pixel_values).last_hidden_state[:, 1:, :]
        h = w_ = int(x.shape[1] ** 0.5)
        x = x.reshape(x.shape[0], h, w_, -1)
        x = InternVLModel.pixel_shuffle(None, x, scale_factor=0.5)
        x = x.reshape(x.shape[0], -1, x.shape[-1])
        return proj(x)

    enc = LingoInternVLModel.__new__(LingoInternVLModel)
    nn.Module.__init__(enc)
    enc.model = pytypes.SimpleNamespace(
        config=pytypes.SimpleNamespace(output_attentions=False, output_hidden_states=False, use_return_dict=True),
        extract_feature=extract_feature)
    tok = pytypes.SimpleNamespace(
        additional_special_tokens_ids=list(range(cfg.first_added_id, cfg.first_added_id + 8)),
        convert_tokens_to_ids=lambda t: {"<IMG_CONTEXT>": cfg.img_context_id}[t])
    enc.processor = tok
    lang_model = pytypes.SimpleNamespace(model=qwen, hidden_size=d)
    driving = DrivingAdaptor(d, speed_wps_mode="2d", predict_route_as_wps=True)
    driving.query_embeds_wps.data.copy_(P["drv.query_route"][None])
    driving.query_embeds_speed.data.copy_(P["drv.query_speed"][None])
    for j, k in ((0, 0), (2, 1), (4, 2)):
        driving.route_head[j].weight.data.copy_(P[f"route.{k}.w"])
        if driving.route_head[j].bias is not None:
            driving.route_head[j].bias.data.copy_(P[f"route.{k}.b"])
    for j, k in ((0, 0), (2, 1)):
        driving.speed_wps_head[j].weight.data.copy_(P[f"speed.{k}.w"])
        if driving.speed_wps_head[j].bias is not None:
            driving.speed_wps_head[j].bias.data.copy_(P[f"speed.{k}.b"])
    adaptors = AdaptorList(language=LanguageAdaptor(lang_model), driving=driving)
    wp_enc = WaypointInputAdaptor(token_size=d, hidden_size=cfg.wp_hidden, hidden_size2=cfg.wp_hidden2)
    for j, k in ((0, 0), (2, 1), (4, 2)):
        wp_enc.mlp[j].weight.data.copy_(P[f"wp.{k}.w"])
        wp_enc.mlp[j].bias.data.copy_(P[f"wp.{k}.b"])
    modules = dict(vit=vit, proj=proj, qwen=qwen, driving=driving, wp=wp_enc)
    return enc, adaptors, wp_enc, qwen, modules


def reference_forward_loss(enc, adaptors, wp_enc, qwen, example):
    """driving.py:247-261 forward_loss -> :190-233 forward_model, verbatim in structure."""
    adaptor_dict = adaptors(example)                                                   # :247
    adaptor_dict = enc.replace_placeholder_tokens(                                     # :200-205
        adaptor_dict=adaptor_dict, pixel_values=example.driving_input.camera_images,
        placeholder_values=example.driving_input.prompt.placeholder_values, wp_encoder=wp_enc)
    outputs = qwen(attention_mask=adaptor_dict["inputs_mask"], position_ids=None,     # :217-223
                   inputs_embeds=adaptor_dict["inputs"], output_hidden_states=True, return_dict=True)
    features, logits = outputs.hidden_states[-1], outputs[0]                          # :224-225
    loss_dict = adaptors.compute_loss(features, logits, adaptor_dict, example)        # :252
    only = {k: v for k, v in loss_dict.items() if k.endswith("loss")}                  # :254
    out = summarise_losses(only)                                                       # :261
    return out, loss_dict, features, adaptor_dict


def to_ref_types(ex):
    di, dl = ex.driving_input, ex.driving_label
    p = di.prompt
    lab = RT.LanguageLabel(phrase_ids=p.phrase_ids, phrase_valid=p.phrase_valid, phrase_mask=p.phrase_mask,
                           placeholder_values=p.placeholder_values, language_string=p.language_string,
                           loss_masking=p.loss_masking)
    din = RT.DrivingInput(camera_images=di.camera_images, image_sizes=di.image_sizes,
                          camera_intrinsics=di.camera_intrinsics, camera_extrinsics=di.camera_extrinsics,
                          vehicle_speed=di.vehicle_speed, target_point=di.target_point, prompt=lab, prompt_inference=lab)
    dlab = RT.DrivingLabel(waypoints=dl.waypoints, path=dl.path, answer=None, image_ff_org=dl.image_ff_org)
    return RT.DrivingExample(driving_input=din, driving_label=dlab, run_id=ex.run_id)


def param_checksum(t):
    t = t.double()
    return np.asarray([t.sum().item(), t.abs().sum().item(), t.pow(2).sum().item()])


def grad_digest(g):
    """Full gradient for small tensors; otherwise sum/|sum|/sumsq + 256 entries at fixed positions."""
    g = g.reshape(-1)
    out = {"gs": param_checksum(g)}
    if g.numel() <= 4096:
        out["g"] = g.numpy()
    else:
        idx = np.random.default_rng(0).choice(g.numel(), 256, replace=False)
        out["gi"] = idx.astype(np.int64)
        out["gv"] = g[torch.from_numpy(idx)].numpy()
    return out


FULL1 = dict(vit_layers=1, llm_layers=1, lora_dropout=0.0)  # the full1 case's geometry (full_config overrides)


def generate(name, B, s_text, n_loss, pad, seed, full=False):
    cfg = full_config(**FULL1) if full else tiny_config()
    torch.manual_seed(seed)
    P = init_params(cfg, seed=seed, lora_b_std=0.02) if full else init_params(cfg, seed=seed, lora_b_std=0.05, std=0.05)
    ex = make_batch(cfg, B=B, s_text=s_text, n_loss=n_loss, seed=seed + 1, pad=pad)
    enc, adaptors, wp_enc, qwen, mods = build_reference(cfg, P)
    out, loss_dict, feats, adict = reference_forward_loss(enc, adaptors, wp_enc, qwen, to_ref_types(ex))
    out.loss.backward()
    # collect reference grads back onto internal names
    vit, proj, drv = mods["vit"], mods["proj"], mods["driving"]
    D = cfg.vit_dim
    G = {"vit.cls": vit.embeddings.cls_token.grad.view(-1), "vit.pos": vit.embeddings.position_embeddings.grad[0],
         "vit.patch.w": vit.embeddings.patch_embeddings.projection.weight.grad.reshape(D, -1),
         "vit.patch.b": vit.embeddings.patch_embeddings.projection.bias.grad,
         "proj.ln.w": proj.layer_norm.weight.grad, "proj.ln.b": proj.layer_norm.bias.grad,
         "proj.fc1.w": proj.linear_1.weight.grad, "proj.fc1.b": proj.linear_1.bias.grad,
         "proj.fc2.w": proj.linear_2.weight.grad, "proj.fc2.b": proj.linear_2.bias.grad,
         "drv.query_route": drv.query_embeds_wps.grad[0], "drv.query_speed": drv.query_embeds_speed.grad[0]}
    for i in range(cfg.vit_layers):
        L = vit.encoder.layer[i]
        a = L.attention
        G[f"vit.{i}.qkv.w"] = torch.cat([a.q_proj.weight.grad, a.k_proj.weight.grad, a.v_proj.weight.grad])
        G[f"vit.{i}.qkv.b"] = torch.cat([a.q_proj.bias.grad, a.k_proj.bias.grad, a.v_proj.bias.grad])
        G[f"vit.{i}.proj.w"], G[f"vit.{i}.proj.b"] = a.projection_layer.weight.grad, a.projection_layer.bias.grad
        G[f"vit.{i}.ls1"], G[f"vit.{i}.ls2"] = L.lambda_1.grad, L.lambda_2.grad
        G[f"vit.{i}.ln1.w"], G[f"vit.{i}.ln1.b"] = L.layernorm_before.weight.grad, L.layernorm_before.bias.grad
        G[f"vit.{i}.ln2.w"], G[f"vit.{i}.ln2.b"] = L.layernorm_after.weight.grad, L.layernorm_after.bias.grad
        for n in ("fc1", "fc2"):
            m = getattr(L.mlp, n)
            G[f"vit.{i}.{n}.w"], G[f"vit.{i}.{n}.b"] = m.weight.grad, m.bias.grad
    for i in range(cfg.llm_layers):
        layer = qwen.model.layers[i]
        for site, mod in (("q", layer.self_attn.q_proj), ("k", layer.self_attn.k_proj), ("v", layer.self_attn.v_proj),
                          ("o", layer.self_attn.o_proj), ("gate", layer.mlp.gate_proj), ("up", layer.mlp.up_proj),
                          ("down", layer.mlp.down_proj)):
            G[f"llm.{i}.lora.{site}.a"] = mod.lora_A.weight.grad
            G[f"llm.{i}.lora.{site}.b"] = mod.lora_B.weight.grad
    for j, k in ((0, 0), (2, 1), (4, 2)):
        G[f"route.{k}.w"] = drv.route_head[j].weight.grad
        if drv.route_head[j].bias is not None:
            G[f"route.{k}.b"] = drv.route_head[j].bias.grad
        G[f"wp.{k}.w"], G[f"wp.{k}.b"] = mods["wp"].mlp[j].weight.grad, mods["wp"].mlp[j].bias.grad
    for j, k in ((0, 0), (2, 1)):
        G[f"speed.{k}.w"] = drv.speed_wps_head[j].weight.grad
        if drv.speed_wps_head[j].bias is not None:
            G[f"speed.{k}.b"] = drv.speed_wps_head[j].bias.grad
    trainable = [s.name for s in param_specs(cfg) if s.trainable]
    missing = [n for n in trainable if n not in G]
    assert not missing, missing
    di = ex.driving_input
    if full:  # inputs regenerated by make_batch(seed + 1); checksums pin them
        inputs = {"in.make_batch": np.asarray([B, s_text, n_loss, seed + 1] + list(pad or [0] * B)),
                  "in.pixel_cs": param_checksum(di.camera_images),
                  "in.ids_cs": param_checksum(di.prompt.phrase_ids.double()),
                  "in.tp_coords": np.stack([pv[cfg.target_point_id] for pv in di.prompt.placeholder_values]),
                  "in.path": ex.driving_label.path.numpy(), "in.waypoints": ex.driving_label.waypoints.numpy()}
    else:
        inputs = {"in.pixel": di.camera_images.numpy(), "in.ids": di.prompt.phrase_ids.numpy(),
                  "in.valid": di.prompt.phrase_valid.numpy(), "in.loss_mask": di.prompt.loss_masking.numpy(),
                  "in.tp_coords": np.stack([pv[cfg.target_point_id] for pv in di.prompt.placeholder_values]),
                  "in.path": ex.driving_label.path.numpy(), "in.waypoints": ex.driving_label.waypoints.numpy()}
    arrays = {
        "cfg": np.frombuffer(json.dumps({"name": "full1" if full else "tiny", **(FULL1 if full else {})}).encode(),
                             dtype=np.uint8),
        **inputs,
        "out.loss": out.loss.detach().numpy(),
        "out.language_loss": out.loss_averages["language_loss"].detach().numpy(),
        "out.route_loss": out.loss_averages["route_loss"].detach().numpy(),
        "out.speed_wps_loss": out.loss_averages["speed_wps_loss"].detach().numpy(),
        "out.route_pred": loss_dict["route_prediction"].detach().numpy(),
        "out.speed_pred": loss_dict["speed_wps_prediction"].detach().numpy(),
        "out.inputs_sum": np.asarray([adict["inputs"].detach().double().sum().item(),
                                      adict["inputs"].detach().double().abs().sum().item()]),
        "out.inputs_mask": adict["inputs_mask"].numpy(),
        "out.perm": adict["perm"].numpy(),
    }
    arrays["seed"] = np.asarray(seed)
    for k, v in P.items():  # parameters are regenerated by init_params(seed); keep a checksum
        arrays["pc." + k] = param_checksum(v)
    for k, v in G.items():
        for kk, vv in grad_digest(v.detach()).items():
            arrays[kk + "." + k] = vv
    os.makedirs(OUT, exist_ok=True)
    path = os.path.join(OUT, f"vla_{name}.npz" if full else f"vla_tiny_{name}.npz")
    np.savez_compressed(path, **arrays)
    print(f"wrote {path}: loss={out.loss.item():.6f} lang={arrays['out.language_loss']:.6f} "
          f"route={arrays['out.route_loss']:.6f} speed={arrays['out.speed_wps_loss']:.6f}")


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["nopad", "leftpad", "full1"]
    if "nopad" in which:
        generate("nopad", B=2, s_text=24, n_loss=6, pad=None, seed=11)
    if "leftpad" in which:
        generate("leftpad", B=3, s_text=24, n_loss=5, pad=[0, 5, 9], seed=23)
    if "full1" in which:  # InternVL2-1B widths, 1 + 1 layers, GQA 14/2, V = 151655, left-padded B = 2, S_llm = 798
        generate("full1", B=2, s_text=256, n_loss=16, pad=[0, 37], seed=31, full=True)
