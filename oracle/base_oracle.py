"""ORACLE — test infrastructure only. CPU fp32 restatement of the SimLingo-Base training step.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and only as
the checker / CPU baseline. The product path (simlingo_amd) never calls it.

DrivingModel.forward_loss (simlingo_base_training/models/driving.py:296-324) in plain PyTorch:
  * get_fixed_input_embeds (driving.py:280-294): LLaVAnextEncoderModel.forward (encoder/llavanext.py:87-113)
      - LingoLlavaNextModel.forward_image (encoder/llavanext_model.py:45-178): CLIP vision tower
        (patch conv without bias, class + position embedding, pre_layrnorm, pre-LN encoder layers with
        quick_gelu MLP), hidden_states[-2] (vision_feature_layer -2), CLS dropped ('default'),
        multi_modal_projector (linear_1, GELU, linear_2), per frame: the npatch_h x npatch_w grid ->
        unpad_image -> avg_pool2d(downsample_feature_grid_factor) -> image_newline column;
      - projection Linear(4096 -> embed_dim) + temporal_encoding + camera_encoding;
    + speed_encoder (VectorInputAdaptor with NormZeroOne, adaptors.py:56-88) and route_encoder
      (WaypointInputAdaptor with NormZeroOne on [target_point, next_target_point], adaptors.py:24-54);
  * AdaptorList.forward (adaptors.py:259-287): DrivingAdaptor queries (route 20 + speed 10), all valid;
  * forward_model (driving.py:260-278): Llama (llama.py:82-108) = LlamaModel over
    [vision | speed | route | queries], causal, no mask, RoPE theta 1e4, post-norm hidden_states[-1];
  * DrivingAdaptor.compute_loss (adaptors.py:187-232): heads Linear-SiLU-Linear(no bias), cumsum,
    mse.sum(-1).mean(-1); summarise_losses (models/utils.py:153-198).
Parity pin: tests/golden/base_tiny.npz is produced by oracle/gen_golden_base.py from the reference's own
LingoLlavaNextModel.forward_image, adaptors and summarise_losses plus the transformers CLIP/Llama models;
tests/test_base_oracle_golden.py checks this restatement against it.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from oracle.vla_oracle import apply_rope, rms, rope_cos_sin


def quick_gelu(x):
    return x * torch.sigmoid(1.702 * x)


def clip_forward(P, cfg, pix):
    """pix [N, 3, H, W] -> hidden_states[-2] of the CLIP tower: the output of layer vit_layers-1."""
    D, p = cfg.vit_dim, cfg.patch
    N = pix.shape[0]
    x = F.conv2d(pix, P["vit.patch.w"].view(D, 3, p, p), None, stride=p).flatten(2).transpose(1, 2)
    x = torch.cat([P["vit.cls"].view(1, 1, D).expand(N, 1, D), x], 1) + P["vit.pos"][None]
    x = F.layer_norm(x, (D,), P["vit.pre_ln.w"], P["vit.pre_ln.b"], cfg.vit_eps)
    H, T = cfg.vit_heads, x.shape[1]
    for i in range(cfg.vit_used):
        g = lambda n: P[f"vit.{i}.{n}"]
        h = F.layer_norm(x, (D,), g("ln1.w"), g("ln1.b"), cfg.vit_eps)
        qkv = (h @ g("qkv.w").t() + g("qkv.b")).view(N, T, 3, H, 64).permute(2, 0, 3, 1, 4)
        a = torch.softmax(qkv[0] @ qkv[1].transpose(-1, -2) * (64 ** -0.5), -1) @ qkv[2]
        x = x + a.transpose(1, 2).reshape(N, T, D) @ g("proj.w").t() + g("proj.b")
        h = F.layer_norm(x, (D,), g("ln2.w"), g("ln2.b"), cfg.vit_eps)
        x = x + quick_gelu(h @ g("fc1.w").t() + g("fc1.b")) @ g("fc2.w").t() + g("fc2.b")
    return x


def merge_image(P, cfg, feat):
    """One frame's projector rows [npatch, g*g, C] -> [tokens, C] (llavanext_model.py:128-157)."""
    g, C = cfg.vit_grid, feat.shape[-1]
    x = feat.view(cfg.npatch_h, cfg.npatch_w, g, g, C).permute(4, 0, 2, 1, 3).contiguous()
    x = x.flatten(1, 2).flatten(2, 3)
    r0, hu, c0, wu = cfg.unpad()
    x = x[:, r0:r0 + hu, c0:c0 + wu]
    x = F.avg_pool2d(x[None], cfg.pool)[0]
    x = torch.cat([x, P["mm.newline"][:, None, None].expand(C, x.shape[1], 1)], -1)
    return x.flatten(1, 2).transpose(0, 1)


def vision_embeds(P, cfg, pix):
    """LLaVAnextEncoderModel.forward: pix [B, 1, 1, npatch, 3, H, W] -> [B, tokens, embed_dim]."""
    B = pix.shape[0]
    x = clip_forward(P, cfg, pix.reshape(-1, 3, cfg.img_size, cfg.img_size))[:, 1:]
    x = F.gelu(x @ P["mm.fc1.w"].t() + P["mm.fc1.b"]) @ P["mm.fc2.w"].t() + P["mm.fc2.b"]
    x = x.view(B, cfg.npatch, -1, x.shape[-1])
    merged = torch.stack([merge_image(P, cfg, x[b]) for b in range(B)])
    return merged @ P["enc.proj.w"].t() + P["enc.proj.b"] + P["enc.temporal"] + P["enc.camera"]


def input_mlp(P, tag, x, lo, hi):
    x = (x - lo) / (hi - lo)
    return torch.relu(x @ P[f"{tag}.0.w"].t() + P[f"{tag}.0.b"]) @ P[f"{tag}.1.w"].t() + P[f"{tag}.1.b"]


def llama_forward(P, cfg, x):
    """LlamaModel(inputs_embeds) causal, no mask -> post-norm last hidden state."""
    B, S, d = x.shape
    H, Fl = cfg.llm_heads, cfg.llm_ffn
    cos, sin = rope_cos_sin(S, cfg.rope_theta)
    causal = torch.ones(S, S, dtype=torch.bool).tril()
    for i in range(cfg.llm_layers):
        g = lambda n: P[f"llm.{i}.{n}"]
        h = rms(x, g("ln1"), cfg.rms_eps)
        q, k, v = (h @ g("qkv_w").t()).split([d, d, d], -1)
        q = apply_rope(q.view(B, S, H, 64).transpose(1, 2), cos, sin)
        k = apply_rope(k.view(B, S, H, 64).transpose(1, 2), cos, sin)
        v = v.view(B, S, H, 64).transpose(1, 2)
        s = (q @ k.transpose(-1, -2)) / 8.0
        a = torch.softmax(s.masked_fill(~causal, float("-inf")), -1) @ v
        x = x + a.transpose(1, 2).reshape(B, S, d) @ g("o_w").t()
        h = rms(x, g("ln2"), cfg.rms_eps)
        gate, up = (h @ g("gate_up_w").t()).split([Fl, Fl], -1)
        x = x + (F.silu(gate) * up) @ g("down_w").t()
    return rms(x, P["llm.norm"], cfg.rms_eps)


def heads(P, cfg, feat):
    fr, fs = feat[:, :cfg.n_route], feat[:, cfg.n_route:]
    route = (F.silu(fr @ P["route.0.w"].t() + P["route.0.b"]) @ P["route.1.w"].t()).cumsum(1)
    speed = (F.silu(fs @ P["speed.0.w"].t() + P["speed.0.b"]) @ P["speed.1.w"].t()).cumsum(1)
    return route, speed


def forward_loss(P, cfg, example):
    di, lab = example.driving_input, example.driving_label
    vis = vision_embeds(P, cfg, di.camera_images)
    B = vis.shape[0]
    speed = input_mlp(P, "spd", di.vehicle_speed.view(B, 1), cfg.speed_min, cfg.speed_max)[:, None]
    route = input_mlp(P, "rte", di.map_route.view(B, cfg.n_tp, 2), cfg.tp_min, cfg.tp_max)
    queries = torch.cat([P["drv.query_route"], P["drv.query_speed"]], 0)[None].expand(B, -1, -1)
    x = torch.cat([vis, speed, route, queries], 1)
    feat = llama_forward(P, cfg, x)[:, -cfg.n_queries:]
    route_pred, speed_pred = heads(P, cfg, feat)
    route_loss = F.mse_loss(route_pred, lab.route_adjusted, reduction="none").sum(-1).mean(-1)
    speed_loss = F.mse_loss(speed_pred, lab.waypoints[:, :cfg.n_speed], reduction="none").sum(-1).mean(-1)
    avg = {"route_loss": route_loss.mean(), "speed_wps_loss": speed_loss.mean()}
    return {"loss": avg["route_loss"] + avg["speed_wps_loss"], **avg, "route_pred": route_pred,
            "speed_pred": speed_pred, "inputs": x}


def loss_and_grads(P, cfg, example):
    Pg = {k: v.detach().clone().requires_grad_(True) for k, v in P.items()}
    out = forward_loss(Pg, cfg, example)
    out["loss"].backward()
    grads = {k: (v.grad.detach().clone() if v.grad is not None else torch.zeros_like(v)) for k, v in Pg.items()}
    return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in out.items()}, grads
