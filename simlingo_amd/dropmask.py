"""Host mirror of the counter-based dropout mask used by the HIP kernels (common.h: hash_u32 / drop_keep).
Test helper: lets a PyTorch reference apply exactly the mask the kernels apply."""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def _hash_u32(x):
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def seed_mix(seed: int) -> np.uint64:
    s = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    inner = _hash_u32(np.asarray([(s >> np.uint64(32)) ^ np.uint64(0x9E3779B9)]))
    return _hash_u32(np.asarray([(s & M32) ^ inner[0]]))[0]


def keep_mask(seed: int, idx: np.ndarray, p: float) -> np.ndarray:
    """common.h drop_keep: one hash per index pair (idx >> 1), low / high 16 bits for even / odd idx."""
    idx = idx.astype(np.uint64)
    h = _hash_u32((idx >> np.uint64(1)) ^ seed_mix(seed))
    u = np.where((idx & np.uint64(1)) == 1, h >> np.uint64(16), h & np.uint64(0xFFFF))
    thr = np.uint64(int(p * 65536.0 + 0.5))
    return u >= thr


def keep_scale(seed: int, rows: int, cols: int, ldmask: int, p: float) -> np.ndarray:
    """[rows, cols] float32: 1/(1-p) where kept, 0 where dropped (index = row*ldmask + col)."""
    idx = np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(ldmask) + np.arange(cols, dtype=np.uint64)[None, :]
    return np.where(keep_mask(seed, idx, p), 1.0 / (1.0 - p), 0.0).astype(np.float32)


def keep_bits(seed: int, rows: int, cols: int, ldmask: int, p: float) -> np.ndarray:
    """[rows, cols // 32] uint32 keep bitmask as slx_lora_down writes it (bit c & 31 of word c >> 5)."""
    k = keep_scale(seed, rows, cols, ldmask, p) > 0
    w = k.reshape(rows, cols // 32, 32).astype(np.uint64) << np.arange(32, dtype=np.uint64)
    return w.sum(-1).astype(np.uint32)


def lora_site_seed(step_seed: int, layer: int, site_index: int) -> int:
    """Seed of the LoRA dropout mask of one (layer, site) in one training step (engine._lora_down)."""
    return step_seed * 1000003 + 131 * layer + 7 * site_index + 1


def lora_masks(cfg, rows: int, step_seed: int) -> dict:
    """{(layer, site): [rows, in_features] float32 keep-scale} — exactly the masks the engine's forward with
    this step_seed applies (rows = flat B*S LLM rows in the permuted order). Test helper for the oracle."""
    from .params import LORA_SITES, lora_io
    p = cfg.lora_dropout
    out = {}
    for i in range(cfg.llm_layers):
        for j, site in enumerate(LORA_SITES):
            kin = lora_io(cfg, site)[0]
            out[(i, site)] = keep_scale(lora_site_seed(step_seed, i, j), rows, kin, kin, p)
    return out
