"""Host mirror of the counter-based dropout mask used by the HIP kernels (common.h: hash_u32 /
uniform01). Test helper: lets a PyTorch reference apply exactly the mask the kernels apply."""
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


def uniform01(seed: int, idx: np.ndarray) -> np.ndarray:
    idx = idx.astype(np.uint64)
    seed = np.uint64(seed & 0xFFFFFFFFFFFFFFFF)
    lo = idx & M32
    hi = idx >> np.uint64(32)
    inner = _hash_u32((seed & M32) ^ ((hi * np.uint64(0x9E3779B9)) & M32))
    h = _hash_u32(lo ^ inner ^ (seed >> np.uint64(32)))
    return (h >> np.uint64(8)).astype(np.float64) * (1.0 / 16777216.0)


def keep_scale(seed: int, rows: int, cols: int, ldmask: int, p: float) -> np.ndarray:
    """[rows, cols] float32: 1/(1-p) where kept, 0 where dropped (index = row*ldmask + col)."""
    idx = np.arange(rows, dtype=np.uint64)[:, None] * np.uint64(ldmask) + np.arange(cols, dtype=np.uint64)[None, :]
    return np.where(uniform01(seed, idx) >= p, 1.0 / (1.0 - p), 0.0).astype(np.float32)


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
