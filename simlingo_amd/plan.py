"""Host-side token plan: the reference's token assembly restated as index arrays.

The reference builds the LLM input with host-synchronising Python loops
(AdaptorList.forward adaptors.py:301-331; replace_placeholder_tokens internvl2_model.py:44-142;
split_outputs_by_adaptor adaptors.py:357-370). Here the same decisions are taken once per batch on
the host from the CPU copies of ids/masks (the collate owns them), producing int32 index arrays that
one device gather (slx_assemble_tokens) and a few row gathers consume without any device->host sync.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from .config import VLAConfig

KIND_TOKEN, KIND_IMG, KIND_WP, KIND_QUERY = 0, 1, 2, 3


def _code(kind, idx):
    return (np.int64(kind) << 28) | np.asarray(idx, dtype=np.int64)


@dataclass
class Plan:
    B: int
    L: int                 # language positions per sample
    S: int                 # LLM sequence = L + n_queries
    code: np.ndarray       # [B*S] int32  (kind << 28 | index)
    seqlens: np.ndarray    # [B] int32 valid (leading) positions of each LLM sequence
    n_img: int             # vit rows expected (B * tiles * tokens_per_tile)
    img_pos: np.ndarray    # [n_img] int32 final flat position of each vit row (B*S = not referenced)
    wp_coords: np.ndarray  # [n_wp, 2] f32 coordinates fed to wp_encoder (row order as the reference)
    wp_pos: np.ndarray     # [n_wp] int32 final flat position of each wp row (B*S = not referenced)
    query_pos: np.ndarray  # [B, n_queries] int32 final flat positions of the driving queries
    loss_pos: np.ndarray   # [R] int32 final flat positions whose logits enter the LM loss
    loss_labels: np.ndarray  # [R] int32 next-token labels
    loss_bt: np.ndarray | None = None  # [R, 2] (sample, position in the shifted [B, L-1] label grid) of each loss row
    perm: np.ndarray | None = None     # [B, S] AdaptorList.forward's valid-first permutation (adaptors.py:322-325)

    def to_device(self, device) -> dict:
        t = lambda a, dt=torch.int32: torch.from_numpy(np.ascontiguousarray(a)).to(dt).pin_memory().to(device, non_blocking=True) \
            if torch.cuda.is_available() and str(device) != "cpu" else torch.from_numpy(np.ascontiguousarray(a)).to(dt)
        return {"code": t(self.code), "seqlens": t(self.seqlens), "img_pos": t(self.img_pos),
                "wp_coords": t(self.wp_coords, torch.float32), "wp_pos": t(self.wp_pos),
                "query_pos": t(self.query_pos.reshape(-1)), "loss_pos": t(self.loss_pos),
                "loss_labels": t(self.loss_labels)}


def build_plan(cfg: VLAConfig, ids, valid, loss_mask, placeholder_values, n_img: int | None = None) -> Plan:
    ids = np.asarray(ids.cpu() if isinstance(ids, torch.Tensor) else ids, dtype=np.int64)
    valid = np.asarray(valid.cpu() if isinstance(valid, torch.Tensor) else valid, dtype=bool)
    loss_mask = np.asarray(loss_mask.cpu() if isinstance(loss_mask, torch.Tensor) else loss_mask, dtype=bool)
    B, L = ids.shape
    NQ = cfg.n_queries
    S = L + NQ
    V = cfg.vocab
    n_img = cfg.img_tokens * B if n_img is None else n_img
    # language codes before replacement: embed_tokens(ids.clamp(0, V-1))  (adaptors.py:256)
    lang = _code(KIND_TOKEN, np.clip(ids, 0, V - 1))
    # 2a placeholders (internvl2_model.py:53-91): unique ids >= first added special id; first
    # occurrence per sample; pairs whose first occurrence is 0 are skipped (nonzero(), :78)
    special = sorted(set(ids[ids >= cfg.first_added_id].tolist()))
    wp_coords, wp_lang = [], []
    if special and placeholder_values:
        for b in range(B):
            for key in special:
                hit = np.nonzero(ids[b] == key)[0]
                first = int(hit[0]) if hit.size else 0
                if first == 0:
                    continue
                coords = np.asarray(placeholder_values[b][key], dtype=np.float32).reshape(-1, 2)
                for j in range(coords.shape[0]):
                    wp_lang.append((b, first + j))
                    wp_coords.append(coords[j])
                    lang[b, first + j] = _code(KIND_WP, len(wp_coords) - 1)
    # 2 merge image features (internvl2_model.py:119-131): IMG_CONTEXT positions in flattened order
    sel = (ids.reshape(-1) == cfg.img_context_id)
    n_sel = int(sel.sum())
    if n_sel > n_img:
        raise ValueError(f"{n_sel} <IMG_CONTEXT> tokens but only {n_img} image feature rows")
    flat = lang.reshape(-1)
    flat[sel] = _code(KIND_IMG, np.arange(n_sel))
    lang = flat.reshape(B, L)
    # AdaptorList.forward: concat [language | driving queries], stable valid-first permutation
    valid_cat = np.concatenate([valid, np.ones((B, NQ), dtype=bool)], axis=1)
    perm = np.argsort(~valid_cat, axis=1, kind="stable")
    inv = np.argsort(perm, axis=1, kind="stable")
    code = np.empty((B, S), dtype=np.int64)
    for b in range(B):
        i0 = int(perm[b, 0])
        for s in range(S):
            if s < L - i0:  # internvl2_model.py:139-142 copy of the replaced language embeddings
                code[b, s] = lang[b, i0 + s]
            else:
                p = int(perm[b, s])
                code[b, s] = _code(KIND_QUERY, p - L) if p >= L else _code(KIND_TOKEN, min(max(int(ids[b, p]), 0), V - 1))
    seqlens = valid_cat.sum(1).astype(np.int32)
    # positions of image / waypoint rows in the final sequence (for the backward gathers)
    flat_code = code.reshape(-1)
    kinds = flat_code >> 28
    idx = flat_code & ((1 << 28) - 1)
    img_pos = np.full(n_img, B * S, dtype=np.int32)
    m = kinds == KIND_IMG
    img_pos[idx[m]] = np.nonzero(m)[0]
    n_wp = len(wp_coords)
    wp_pos = np.full(n_wp, B * S, dtype=np.int32)
    m = kinds == KIND_WP
    wp_pos[idx[m]] = np.nonzero(m)[0]
    query_pos = (np.arange(B)[:, None] * S + inv[:, L:]).astype(np.int32)
    # LanguageAdaptor.compute_loss: logits[:, :-1] vs where(loss_mask, ids, -1)[:, 1:]
    labels = np.where(loss_mask, ids, -1)[:, 1:]
    bb, tt = np.nonzero(labels != -1)
    loss_pos = (bb * S + inv[bb, tt]).astype(np.int32)
    loss_labels = labels[bb, tt].astype(np.int32)
    return Plan(B=B, L=L, S=S, code=code.reshape(-1).astype(np.int32), seqlens=seqlens, n_img=n_img, img_pos=img_pos,
                wp_coords=np.asarray(wp_coords, dtype=np.float32).reshape(-1, 2), wp_pos=wp_pos,
                query_pos=query_pos, loss_pos=loss_pos, loss_labels=loss_labels,
                loss_bt=np.stack([bb, tt], 1).astype(np.int64), perm=perm.astype(np.int64))


def plan_from_example(cfg: VLAConfig, example, inference: bool = False) -> Plan:
    di = example.driving_input if hasattr(example, "driving_input") else example
    lab = di.prompt_inference if inference else di.prompt
    B = di.camera_images.shape[0]
    n_img = B * di.camera_images.shape[2] * cfg.img_tokens_per_tile
    return build_plan(cfg, lab.phrase_ids, lab.phrase_valid, lab.loss_masking, lab.placeholder_values, n_img)
