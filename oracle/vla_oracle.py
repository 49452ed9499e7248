"""ORACLE — test infrastructure only. CPU fp32 restatement of the SimLingo VLA training step.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module, and
only as the checker / CPU baseline. The product path (simlingo_amd) never calls it.

It restates, in plain PyTorch on the CPU, exactly the arithmetic the reference runs for one
training step (DrivingModel.forward_loss, simlingo_training/models/driving.py:236-261):
  * AdaptorList.forward               adaptors.py:301-331  (+ LanguageAdaptor.forward :238-257,
                                                            DrivingAdaptor.forward :139-161)
  * replace_placeholder_tokens         encoder/internvl2_model.py:17-144
  * extract_feature (remote InternVL2) = InternViT (patch conv, CLS, pos-emb, 24 x
    [x += ls1*Attn(LN(x)); x += ls2*MLP(LN(x))]) -> drop CLS -> pixel_shuffle(0.5, v2) -> mlp1
  * language_model.model (driving.py:217-225) = Qwen2 + peft LoRA (llm.py:106-119), post-norm
    hidden_states[-1] and full logits
  * AdaptorList.compute_loss           adaptors.py:333-370 (+ :183-221, :259-274)
  * summarise_losses                   models/utils.py:7-41
Parity pin: tests/golden/*.npz were produced by oracle/gen_golden.py, which runs the reference's own
adaptors / replace_placeholder_tokens / summarise_losses code together with the transformers
implementations of InternViT / pixel_shuffle / projector / Qwen2 (the remote code is not available
offline); tests/test_oracle_golden.py checks this restatement against them.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# ---------------------------------------------------------------------------------------------
# InternViT + mlp1  (remote InternVisionModel / extract_feature; called internvl2_model.py:114)


def vit_forward(P, cfg, pix):
    """pix [N, 3, H, W] -> last hidden state [N, 1 + g*g, D] (select_layer -1, no final norm)."""
    D, p = cfg.vit_dim, cfg.patch
    N = pix.shape[0]
    x = F.conv2d(pix, P["vit.patch.w"].view(D, 3, p, p), P["vit.patch.b"], stride=p)
    x = x.flatten(2).transpose(1, 2)
    x = torch.cat([P["vit.cls"].view(1, 1, D).expand(N, 1, D), x], 1) + P["vit.pos"][None]
    H = cfg.vit_heads
    T = x.shape[1]
    for i in range(cfg.vit_layers):
        g = lambda n: P[f"vit.{i}.{n}"]
        h = F.layer_norm(x, (D,), g("ln1.w"), g("ln1.b"), cfg.vit_eps)
        qkv = (h @ g("qkv.w").t() + g("qkv.b")).view(N, T, 3, H, 64).permute(2, 0, 3, 1, 4)
        a = torch.softmax(qkv[0] @ qkv[1].transpose(-1, -2) * (64 ** -0.5), -1) @ qkv[2]
        a = a.transpose(1, 2).reshape(N, T, D)
        x = x + g("ls1") * (a @ g("proj.w").t() + g("proj.b"))
        h = F.layer_norm(x, (D,), g("ln2.w"), g("ln2.b"), cfg.vit_eps)
        h = F.gelu(h @ g("fc1.w").t() + g("fc1.b")) @ g("fc2.w").t() + g("fc2.b")
        x = x + g("ls2") * h
    return x


def pixel_shuffle_v2(x, scale_factor=0.5):
    n, w, h, c = x.size()
    x = x.view(n, w, int(h * scale_factor), int(c / scale_factor))
    x = x.permute(0, 2, 1, 3).contiguous()
    x = x.view(n, int(h * scale_factor), int(w * scale_factor), int(c / (scale_factor * scale_factor)))
    return x.permute(0, 2, 1, 3).contiguous()


def extract_feature(P, cfg, pix):
    x = vit_forward(P, cfg, pix)[:, 1:]
    g = cfg.vit_grid
    x = pixel_shuffle_v2(x.reshape(x.shape[0], g, g, -1))
    x = x.reshape(x.shape[0], -1, x.shape[-1])
    x = F.layer_norm(x, (x.shape[-1],), P["proj.ln.w"], P["proj.ln.b"], cfg.proj_eps)
    x = F.gelu(x @ P["proj.fc1.w"].t() + P["proj.fc1.b"])
    return x @ P["proj.fc2.w"].t() + P["proj.fc2.b"]


# ---------------------------------------------------------------------------------------------
# Qwen2 + LoRA (language_model.model(...), driving.py:217-223)


def rms(x, w, eps):
    return w * (x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps))


def rope_cos_sin(S, theta, dtype=torch.float32):
    inv = 1.0 / (theta ** (torch.arange(0, 64, 2, dtype=torch.int64).float() / 64))
    fr = torch.outer(torch.arange(S, dtype=torch.int64).float(), inv)
    emb = torch.cat([fr, fr], -1)
    return emb.cos().to(dtype), emb.sin().to(dtype)


def apply_rope(x, cos, sin):  # x [B, H, S, 64]
    rot = torch.cat([-x[..., 32:], x[..., :32]], -1)
    return x * cos + rot * sin


def lora(P, cfg, i, site, x, masks=None):
    """peft LoRA: scale * B(A(dropout(x))). masks: optional {(layer, site): keep-scale [B*S, in]} — the
    dropout masks the engine applied (simlingo_amd.dropmask.lora_masks), so a dropout-on step can be checked."""
    if not cfg.lora:
        return 0.0
    if masks is not None:
        x = x * torch.as_tensor(masks[(i, site)]).view(x.shape)
    return (x @ P[f"llm.{i}.lora.{site}.a"].t()) @ P[f"llm.{i}.lora.{site}.b"].t() * cfg.lora_scale


def llm_forward(P, cfg, x, mask, masks=None):
    """x [B, S, d] inputs_embeds, mask [B, S] bool (valid) -> (post-norm features, logits)."""
    B, S, d = x.shape
    H, Hk, Fd = cfg.llm_heads, cfg.llm_kv_heads, cfg.llm_ffn
    cos, sin = rope_cos_sin(S, cfg.rope_theta)
    kk = torch.arange(S)
    allowed = (kk[None, :] <= kk[:, None])[None] & mask[:, None, :]  # causal & key padding
    for i in range(cfg.llm_layers):
        g = lambda n: P[f"llm.{i}.{n}"]
        h = rms(x, g("ln1"), cfg.rms_eps)
        qkv = h @ g("qkv_w").t() + g("qkv_b")
        q, k, v = qkv.split([H * 64, Hk * 64, Hk * 64], -1)
        q = q + lora(P, cfg, i, "q", h, masks)
        k = k + lora(P, cfg, i, "k", h, masks)
        v = v + lora(P, cfg, i, "v", h, masks)
        q = apply_rope(q.view(B, S, H, 64).transpose(1, 2), cos, sin)
        k = apply_rope(k.view(B, S, Hk, 64).transpose(1, 2), cos, sin).repeat_interleave(H // Hk, 1)
        v = v.view(B, S, Hk, 64).transpose(1, 2).repeat_interleave(H // Hk, 1)
        s = (q @ k.transpose(-1, -2)) / 8.0
        s = s.masked_fill(~allowed[:, None], float("-inf"))
        a = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(B, S, H * 64)
        x = x + a @ g("o_w").t() + lora(P, cfg, i, "o", a, masks)
        h = rms(x, g("ln2"), cfg.rms_eps)
        gu = h @ g("gate_up_w").t()
        gate, up = gu.split([Fd, Fd], -1)
        gate = gate + lora(P, cfg, i, "gate", h, masks)
        up = up + lora(P, cfg, i, "up", h, masks)
        act = F.silu(gate) * up
        x = x + act @ g("down_w").t() + lora(P, cfg, i, "down", act, masks)
    feat = rms(x, P["llm.norm"], cfg.rms_eps)
    return feat, feat @ P["llm.lm_head"].t()


# ---------------------------------------------------------------------------------------------
# token assembly (AdaptorList.forward + replace_placeholder_tokens), literal restatement


def assemble(P, cfg, example, vit_embeds, inference=False):
    di = example.driving_input
    lab = di.prompt_inference if inference else di.prompt
    ids = lab.phrase_ids.long()
    valid = lab.phrase_valid.bool()
    B, L = ids.shape
    V = cfg.vocab
    lang = P["llm.embed"][ids.clamp(min=0, max=V - 1)]                       # adaptors.py:256
    queries = torch.cat([P["drv.query_route"], P["drv.query_speed"]], 0)[None].expand(B, -1, -1)
    inputs = torch.cat([lang, queries], 1)                                   # adaptors.py:316
    inputs_mask = torch.cat([valid, torch.ones(B, cfg.n_queries, dtype=torch.bool)], 1)
    arange = torch.arange(B)[:, None]
    rand_perm = torch.arange(inputs.size(1)).expand(B, -1)
    valid_perm = inputs_mask[arange, rand_perm].byte().argsort(dim=-1, descending=True, stable=True)
    perm = rand_perm.gather(1, valid_perm)                                   # adaptors.py:322-325
    inputs_p = inputs[arange, perm]
    mask_p = inputs_mask[arange, perm]
    # replace_placeholder_tokens (internvl2_model.py:50-91)
    lang = lang.clone()
    special = sorted(set(ids[ids >= cfg.first_added_id].tolist()))
    pv = lab.placeholder_values
    if special and len(pv) > 0:
        for b in range(B):
            for key in special:
                hit = (ids[b] == key).nonzero()
                first = int(hit[0, 0]) if hit.numel() else 0
                if first == 0:
                    continue
                coords = torch.as_tensor(pv[b][key], dtype=P["wp.0.w"].dtype).view(-1, 2)
                lang[b, first:first + coords.shape[0]] = wp_encoder(P, coords)
    # image merge (internvl2_model.py:119-131)
    flat = lang.reshape(B * L, -1)
    sel = ids.reshape(-1) == cfg.img_context_id
    flat = flat.clone()
    flat[sel] = flat[sel] * 0.0 + vit_embeds.reshape(-1, flat.shape[-1])[: int(sel.sum())]
    lang = flat.reshape(B, L, -1)
    # copy into the permuted inputs (internvl2_model.py:139-142)
    rows = []
    for b in range(B):
        i0 = int(perm[b, 0])
        rows.append(torch.cat([lang[b, i0:], inputs_p[b, L - i0:]], 0))
    return torch.stack(rows), mask_p, perm


def wp_encoder(P, coords):  # WaypointInputAdaptor.mlp (adaptors.py:80)
    h = torch.relu(coords @ P["wp.0.w"].t() + P["wp.0.b"])
    h = torch.relu(h @ P["wp.1.w"].t() + P["wp.1.b"])
    return h @ P["wp.2.w"].t() + P["wp.2.b"]


def smooth_l1_sum(pred, label):
    return F.smooth_l1_loss(pred, label, reduction="none").sum(-1)


def forward_loss(P, cfg, example, dropout_masks=None):
    """DrivingModel.forward_loss (driving.py:236-261) -> dict of scalar losses and predictions."""
    di = example.driving_input
    pix = di.camera_images
    Bn, T_, NP, C, H, W = pix.shape
    vit = extract_feature(P, cfg, pix.reshape(Bn * NP, C, H, W))
    inputs, mask, perm = assemble(P, cfg, example, vit)
    feat, logits = llm_forward(P, cfg, inputs, mask, dropout_masks)
    # split_outputs_by_adaptor (adaptors.py:357-370)
    inv = perm.argsort(-1)
    ar = torch.arange(feat.shape[0])[:, None]
    feat_o, logit_o = feat[ar, inv], logits[ar, inv]
    L = di.prompt.phrase_ids.shape[1]
    # language loss (adaptors.py:259-274)
    labels = torch.where(di.prompt.loss_masking, di.prompt.phrase_ids, -1)[:, 1:]
    lg = logit_o[:, :L][:, :-1]
    lang = F.cross_entropy(lg.flatten(0, -2), labels.flatten(), ignore_index=-1, reduction="none").view_as(labels)
    lang_cnt = labels.ne(-1)
    # driving losses (adaptors.py:183-221)
    dfeat = feat_o[:, L:]
    f_route, f_speed = dfeat[:, :cfg.n_route], dfeat[:, cfg.n_route:]
    h = F.silu(f_route @ P["route.0.w"].t() + P["route.0.b"])
    h = F.silu(h @ P["route.1.w"].t() + P["route.1.b"])
    route_pred = (h @ P["route.2.w"].t()).cumsum(1)
    h = F.silu(f_speed @ P["speed.0.w"].t() + P["speed.0.b"])
    speed_pred = (h @ P["speed.1.w"].t()).cumsum(1)
    lab = example.driving_label
    route_loss = smooth_l1_sum(route_pred, lab.path)
    speed_loss = smooth_l1_sum(speed_pred, lab.waypoints[:, : cfg.n_route + 1])
    # summarise_losses (models/utils.py:7-41)
    losses = {"language_loss": (lang, lang_cnt), "route_loss": (route_loss, torch.ones_like(route_loss)),
              "speed_wps_loss": (speed_loss, torch.ones_like(speed_loss))}
    avg = {k: torch.where(n.sum() > 0, v.sum() / n.sum(), torch.zeros(())) for k, (v, n) in losses.items()}
    total = torch.stack(list(avg.values())).sum()
    return {"loss": total, **avg, "route_pred": route_pred, "speed_pred": speed_pred, "features": feat,
            "inputs": inputs}


# ---------------------------------------------------------------------------------------------
# inference: DrivingModel.forward with predict_language=True (driving.py:104-187)


def language_inputs(P, cfg, example, vit_embeds, inference=True):
    """adaptor_dict['language_inputs'] / ['language_inputs_mask'] after replace_placeholder_tokens
    (adaptors.py:256 embedding, internvl2_model.py:50-131 waypoint + image replacement) -> [B, L, d], [B, L]."""
    di = example.driving_input
    lab = di.prompt_inference if inference else di.prompt
    ids = lab.phrase_ids.long()
    valid = lab.phrase_valid.bool()
    B, L = ids.shape
    lang = P["llm.embed"][ids.clamp(min=0, max=cfg.vocab - 1)].clone()
    special = sorted(set(ids[ids >= cfg.first_added_id].tolist()))
    pv = lab.placeholder_values
    if special and len(pv) > 0:
        for b in range(B):
            for key in special:
                hit = (ids[b] == key).nonzero()
                first = int(hit[0, 0]) if hit.numel() else 0
                if first == 0:
                    continue
                coords = torch.as_tensor(pv[b][key], dtype=P["wp.0.w"].dtype).view(-1, 2)
                lang[b, first:first + coords.shape[0]] = wp_encoder(P, coords)
    flat = lang.reshape(B * L, -1)
    sel = ids.reshape(-1) == cfg.img_context_id
    flat[sel] = flat[sel] * 0.0 + vit_embeds.reshape(-1, flat.shape[-1])[: int(sel.sum())]
    return flat.reshape(B, L, -1), valid


def driving_heads(P, cfg, dfeat):
    """DrivingAdaptor.get_predictions (adaptors.py:163-181): dfeat [B, 30, d] -> route [B,20,2], speed [B,10,2]."""
    f_route, f_speed = dfeat[:, :cfg.n_route], dfeat[:, cfg.n_route:]
    h = F.silu(f_route @ P["route.0.w"].t() + P["route.0.b"])
    h = F.silu(h @ P["route.1.w"].t() + P["route.1.b"])
    route = (h @ P["route.2.w"].t()).cumsum(1)
    h = F.silu(f_speed @ P["speed.0.w"].t() + P["speed.0.b"])
    return route, (h @ P["speed.1.w"].t()).cumsum(1)


def greedy_sample(P, cfg, emb, max_new_tokens, eos):
    """LLM.greedy_sample (llm.py:178-250) literally: the whole sequence is re-run for every token, argmax
    of F.linear(features[:, -1], lm_head) (sample_categorical with temperature 0, llm.py:157-158), stop after
    recording EOS. emb [S0, d] (one sample, valid rows) -> (tokens list, input_embeds [S0 + n, d])."""
    x = emb[None]
    toks = []
    for _ in range(max_new_tokens):
        feat, _ = llm_forward(P, cfg, x, torch.ones(1, x.shape[1], dtype=torch.bool))
        tok = int((feat[0, -1] @ P["llm.lm_head"].t()).argmax())
        toks.append(tok)
        x = torch.cat([x, P["llm.embed"][tok][None, None]], 1)
        if tok == eos:
            break
    return toks, x[0]


def drive_after(P, cfg, input_embeds, queries):
    """driving.py:156-165: forward(cat(input_embeds, driving inputs)) (no mask) -> heads on the last 30 rows."""
    x = torch.cat([input_embeds, queries], 0)[None]
    feat, _ = llm_forward(P, cfg, x, torch.ones(1, x.shape[1], dtype=torch.bool))
    return driving_heads(P, cfg, feat[:, -queries.shape[0]:])


def infer(P, cfg, example, max_new_tokens, eos):
    """DrivingModel.forward (predict_language=True) per sample on its valid prompt rows
    -> (speed [B,10,2], route [B,20,2], token lists)."""
    pix = example.driving_input.camera_images
    Bn, _, NP, C, H, W = pix.shape
    vit = extract_feature(P, cfg, pix.reshape(Bn * NP, C, H, W))
    lang, valid = language_inputs(P, cfg, example, vit, inference=True)
    queries = torch.cat([P["drv.query_route"], P["drv.query_speed"]], 0)
    speeds, routes, toks = [], [], []
    for b in range(Bn):
        t, xe = greedy_sample(P, cfg, lang[b][valid[b]], max_new_tokens, eos)
        r, s = drive_after(P, cfg, xe, queries)
        speeds.append(s[0])
        routes.append(r[0])
        toks.append(t)
    return torch.stack(speeds), torch.stack(routes), toks


def trainable_names(cfg, P):
    from simlingo_amd.params import param_specs
    return [s.name for s in param_specs(cfg) if s.trainable and s.name in P]


def loss_and_grads(P, cfg, example, dropout_masks=None):
    """fp32 forward + autograd backward; returns (outputs, {name: grad})."""
    Pg = {k: (v.detach().clone().requires_grad_(True)) for k, v in P.items()}
    names = trainable_names(cfg, Pg)
    for k in Pg:
        if k not in names:
            Pg[k].requires_grad_(False)
    out = forward_loss(Pg, cfg, example, dropout_masks)
    out["loss"].backward()
    grads = {k: Pg[k].grad.detach().clone() if Pg[k].grad is not None else torch.zeros_like(Pg[k]) for k in names}
    return {k: (v.detach() if torch.is_tensor(v) else v) for k, v in out.items()}, grads
