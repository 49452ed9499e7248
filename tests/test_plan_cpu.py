"""Host token plan (simlingo_amd.plan): the vectorised row assembly equals the per-element restatement of
internvl2_model.py:139-142 + AdaptorList.forward's valid-first permutation (adaptors.py:322-325), on left-padded and
unpadded batches with placeholders, and it stays cheap at the config-3 size (B = 8, S = 798)."""
import time

import numpy as np
import pytest

from simlingo_amd.config import full_config, tiny_config
from simlingo_amd.plan import KIND_QUERY, KIND_TOKEN, _code, language_codes, plan_from_example
from simlingo_amd.synthetic import make_batch


def _loop_codes(cfg, ids, placeholder_values, n_img, perm):
    """The per-element loop the vectorised form replaces (the round-4 plan.py:91-98)."""
    B, L = ids.shape
    S = L + cfg.n_queries
    lang, _ = language_codes(cfg, ids, placeholder_values, n_img)
    out = np.empty((B, S), dtype=np.int64)
    for b in range(B):
        i0 = int(perm[b, 0])
        for s in range(S):
            if s < L - i0:
                out[b, s] = lang[b, i0 + s]
            else:
                p = int(perm[b, s])
                out[b, s] = _code(KIND_QUERY, p - L) if p >= L else _code(KIND_TOKEN, min(max(int(ids[b, p]), 0),
                                                                                           cfg.vocab - 1))
    return out


@pytest.mark.parametrize("pad", [[0, 0, 0, 0], [0, 3, 7, 1]])
def test_vectorised_plan_equals_loop(pad):
    cfg = tiny_config()
    ex = make_batch(cfg, B=4, s_text=24, n_loss=6, seed=11, pad=pad)
    plan = plan_from_example(cfg, ex)
    ids = ex.driving_input.prompt.phrase_ids.numpy()
    valid = ex.driving_input.prompt.phrase_valid.numpy()
    pv = ex.driving_input.prompt.placeholder_values
    np.testing.assert_array_equal(plan.code.reshape(plan.B, plan.S), _loop_codes(cfg, ids, pv, plan.n_img, plan.perm))
    # invariants: every image row and waypoint row lands exactly once; queries follow the valid rows
    kinds = plan.code >> 28
    assert (kinds == 1).sum() == (ids == cfg.img_context_id).sum()
    assert (plan.img_pos[: (kinds == 1).sum()] < plan.B * plan.S).all()
    assert np.array_equal((plan.query_pos.reshape(plan.B, -1) % plan.S).max(1) + 1, plan.seqlens)


def test_plan_build_cost_full_geometry():
    cfg = full_config()
    ex = make_batch(cfg, B=8, s_text=256, n_loss=16, seed=5, pad=[0, 2, 0, 5, 0, 0, 1, 0])
    plan_from_example(cfg, ex)
    ts = []
    for _ in range(5):  # the minimum over repeats: this shared host stalls for 10-100 ms at times
        t0 = time.perf_counter()
        plan = plan_from_example(cfg, ex)
        ts.append(time.perf_counter() - t0)
    dt = min(ts)
    assert plan.S == 798 and plan.loss_pos.shape[0] == 8 * 16
    assert dt < 50e-3, f"plan build {dt * 1e3:.2f} ms"
