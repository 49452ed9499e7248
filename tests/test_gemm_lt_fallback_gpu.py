"""The engine's hipBLASLt sites (engine.GEMM_LT: the Qwen2 down projection + residual and the gate/up data gradient on
slx_gemm_lt) against the same step on slx_gemm_bf16, and the switch-over when hipBLASLt refuses a shape: a warning,
GEMM_LT off for the process, the step completed on slx_gemm_bf16 with the same result."""
import pytest
import torch

from golden_util import load_case
from simlingo_amd import kernels as K

pytestmark = pytest.mark.gpu


def _step(case="nopad"):
    import simlingo_amd.engine as E
    from simlingo_amd.plan import plan_from_example
    cfg, P, ex, _ = load_case(case)
    dev = torch.device("cuda")
    eng = E.VLAEngine(cfg, dev, P)
    plan = plan_from_example(cfg, ex)
    lab = ex.driving_label
    out, _, _ = eng.forward(ex.driving_input.camera_images.to(dev), plan, plan.to_device(dev), lab.path.to(dev),
                            lab.waypoints.to(dev))
    eng.backward(None)
    torch.cuda.synchronize()
    return out.clone(), eng.grad.clone()


def test_lt_sites_match_slx_gemm(dev, monkeypatch):
    import simlingo_amd.engine as E
    monkeypatch.setattr(E, "GEMM_LT", True)
    out_lt, g_lt = _step()
    monkeypatch.setattr(E, "GEMM_LT", False)
    out_slx, g_slx = _step()
    # the two paths differ by f32 summation order only
    assert torch.allclose(out_lt, out_slx, rtol=1e-4, atol=1e-5), (out_lt, out_slx)
    err = ((g_lt - g_slx).norm() / g_slx.norm()).item()
    assert err < 1e-3, err


def test_refused_shape_switches_to_slx_gemm(dev, monkeypatch):
    import simlingo_amd.engine as E
    monkeypatch.setattr(E, "GEMM_LT", False)
    out_ref, g_ref = _step()
    monkeypatch.setattr(E, "GEMM_LT", True)
    calls = []

    def refuse(*a, **kw):
        calls.append(1)
        raise RuntimeError("slx_gemm_lt: no hipBLASLt algorithm (test)")

    monkeypatch.setattr(K, "mm_lt", refuse)
    with pytest.warns(UserWarning, match="slx_gemm_lt unavailable"):
        out, g = _step()
    assert calls and E.GEMM_LT is False
    assert torch.allclose(out, out_ref, rtol=1e-5, atol=1e-6)
    err = ((g - g_ref).norm() / g_ref.norm()).item()
    assert err < 1e-4, err  # same kernels; only f32 atomic orders differ
