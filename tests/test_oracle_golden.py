"""Pin the oracle (CPU fp32 restatement) against fixtures produced by the reference's own code."""
import numpy as np
import pytest
import torch

from golden_util import CASES, grad_entries, load_case
from oracle import vla_oracle as O


@pytest.mark.parametrize("case", CASES + ["full1"])
def test_oracle_matches_reference_fixture(case):
    """Tiny cases + `full1`: the InternVL2-1B widths (InternViT 1024/16 heads at T = 1025, GQA 14/2,
    FFN 4864, the 151,655-way CE, LoRA r32) with one layer of each stack, left-padded B = 2 at S_llm = 798, against
    the reference's own AdaptorList / replace_placeholder_tokens / summarise_losses on the transformers mirrors."""
    cfg, P, ex, z = load_case(case)
    out, grads = O.loss_and_grads(P, cfg, ex)
    for k in ("loss", "language_loss", "route_loss", "speed_wps_loss"):
        np.testing.assert_allclose(out[k].numpy(), z["out." + k], rtol=2e-5, atol=2e-5, err_msg=k)
    np.testing.assert_allclose(out["route_pred"].numpy(), z["out.route_pred"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["speed_pred"].numpy(), z["out.speed_pred"], rtol=1e-4, atol=1e-5)
    inp = out["inputs"].double()
    np.testing.assert_allclose([inp.sum().item(), inp.abs().sum().item()], z["out.inputs_sum"], rtol=1e-6)
    for name, g in grads.items():
        idx, want = grad_entries(z, name)
        got = g.reshape(-1)[torch.from_numpy(np.asarray(idx))].numpy()
        scale = np.abs(z["gs." + name][1]) / max(g.numel(), 1) + 1e-8
        np.testing.assert_allclose(got, want, rtol=2e-3, atol=2e-3 * scale + 1e-7, err_msg=name)
        gd = g.double()
        np.testing.assert_allclose(gd.pow(2).sum().item(), z["gs." + name][2], rtol=1e-3, atol=1e-12, err_msg=name)


def test_plan_matches_reference_assembly():
    """The host token plan reproduces the reference's permutation / placeholder / image merge."""
    from simlingo_amd.plan import plan_from_example, KIND_QUERY
    for case in CASES:
        cfg, P, ex, z = load_case(case)
        plan = plan_from_example(cfg, ex)
        perm = z["out.perm"]
        B, S = perm.shape
        assert plan.S == S
        np.testing.assert_array_equal(plan.seqlens, z["out.inputs_mask"].sum(1))
        kinds = (plan.code.reshape(B, S) >> 28)
        # queries sit exactly where the reference permutation put the driving tokens
        L = S - cfg.n_queries
        for b in range(B):
            for s in range(S):
                if perm[b, s] >= L and s >= (L - perm[b, 0]):
                    assert kinds[b, s] == KIND_QUERY
