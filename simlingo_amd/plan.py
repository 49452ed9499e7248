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

    def to_device(self, device, extra: dict | None = None) -> dict:
        """Every index array (and the `extra` f32 host tensors, e.g. the step's labels) packed into ONE pinned staging
        slot and sent to the device in ONE non-blocking copy on the current stream; the returned dict holds views of
        that device buffer. No host<->device synchronisation: the slot is reused only after the copy that last read it
        has executed (a ring of events), so the host can build the next batch while the GPU runs this one."""
        i32 = lambda a: np.ascontiguousarray(a, dtype=np.int32).reshape(-1)
        f32 = lambda a: np.ascontiguousarray(a, dtype=np.float32).reshape(-1).view(np.int32)
        bt = self.loss_bt if self.loss_bt is not None else np.zeros((0, 2))
        parts = [("code", i32(self.code), None, False), ("seqlens", i32(self.seqlens), None, False),
                 ("img_pos", i32(self.img_pos), None, False), ("wp_coords", f32(self.wp_coords), (-1, 2), True),
                 ("wp_pos", i32(self.wp_pos), None, False), ("query_pos", i32(self.query_pos), None, False),
                 ("loss_pos", i32(self.loss_pos), None, False), ("loss_labels", i32(self.loss_labels), None, False),
                 ("loss_bt", i32(bt), (-1, 2), False)]
        for k, t in (extra or {}).items():
            a = t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)
            parts.append((k, f32(a), tuple(a.shape), True))
        return stage_to_device(parts, device)


class _PinnedRing:
    """Pinned int32 staging slots of one device, each guarded by the event of the H2D copy that last read it."""

    def __init__(self, depth: int = 4):
        self.slots = [None] * depth
        self.events = [None] * depth
        self.i = 0

    def take(self, n: int):
        s = self.i % len(self.slots)
        self.i += 1
        if self.events[s] is not None:
            self.events[s].synchronize()  # normally long done: that copy ran at the start of an earlier step
        buf = self.slots[s]
        if buf is None or buf.numel() < n:
            buf = self.slots[s] = torch.empty(max(n, 1 << 16), dtype=torch.int32).pin_memory()
        return s, buf


_rings: dict = {}


def stage_to_device(parts, device) -> dict:
    """parts: [(name, int32 words (f32 data viewed as int32), shape or None, is_f32)] -> {name: device view}: one pinned
    slot, one H2D copy on the current stream."""
    device = torch.device(device)
    if device.type != "cuda" or not torch.cuda.is_available():
        raise RuntimeError("the token plan is staged for the MI355X (HIP) path only; there is no CPU path")
    n = sum(a.size for _, a, _, _ in parts)
    ring = _rings.setdefault(device, _PinnedRing())
    s, host = ring.take(n)
    hv = host.numpy()
    off, spans = 0, []
    for name, a, shape, is_f32 in parts:
        hv[off:off + a.size] = a
        spans.append((name, off, a.size, shape, is_f32))
        off += a.size
    dev = torch.empty(max(n, 1), dtype=torch.int32, device=device)
    dev[:n].copy_(host[:n], non_blocking=True)
    ev = torch.cuda.Event()
    ev.record()
    ring.events[s] = ev
    out = {}
    for name, o, size, shape, is_f32 in spans:
        v = dev[o:o + size]
        if is_f32:
            v = v.view(torch.float32)
        out[name] = v.view(shape) if shape is not None else v
    return out


def language_codes(cfg: VLAConfig, ids: np.ndarray, placeholder_values, n_img: int):
    """[B, L] codes of the language rows after replace_placeholder_tokens (before the valid-first permutation), and the
    waypoint-encoder input coordinates in the reference's row order."""
    B, L = ids.shape
    V = cfg.vocab
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
    return lang, wp_coords


def build_plan(cfg: VLAConfig, ids, valid, loss_mask, placeholder_values, n_img: int | None = None) -> Plan:
    ids = np.asarray(ids.cpu() if isinstance(ids, torch.Tensor) else ids, dtype=np.int64)
    valid = np.asarray(valid.cpu() if isinstance(valid, torch.Tensor) else valid, dtype=bool)
    loss_mask = np.asarray(loss_mask.cpu() if isinstance(loss_mask, torch.Tensor) else loss_mask, dtype=bool)
    B, L = ids.shape
    NQ = cfg.n_queries
    S = L + NQ
    V = cfg.vocab
    n_img = cfg.img_tokens * B if n_img is None else n_img
    lang, wp_coords = language_codes(cfg, ids, placeholder_values, n_img)
    # AdaptorList.forward: concat [language | driving queries], stable valid-first permutation
    valid_cat = np.concatenate([valid, np.ones((B, NQ), dtype=bool)], axis=1)
    perm = np.argsort(~valid_cat, axis=1, kind="stable")
    inv = np.argsort(perm, axis=1, kind="stable")
    # internvl2_model.py:139-142: row s of sample b takes the replaced language embedding lang[b, i0 + s] while
    # s < L - i0 (i0 = the first valid position); the rest follow the permutation (driving queries, or the plain
    # token embedding of the trailing positions)
    i0 = perm[:, 0]
    s_idx = np.arange(S)[None, :]
    take_lang = s_idx < (L - i0)[:, None]
    src = np.minimum(i0[:, None] + s_idx, L - 1)
    from_lang = np.take_along_axis(lang, src, axis=1)
    p_ = perm
    tok = _code(KIND_TOKEN, np.clip(np.take_along_axis(ids, np.minimum(p_, L - 1), axis=1), 0, V - 1))
    code = np.where(take_lang, from_lang, np.where(p_ >= L, _code(KIND_QUERY, p_ - L), tok))
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
