"""Fused LM head + cross entropy (slx_lmhead_ce_fwd / _bwd, LanguageAdaptor.compute_loss adaptors.py:259-274 on the
gathered loss rows) against torch fp32 on the same bf16 operands: per-row CE and lse, ignored rows (-1), labels at
the vocabulary edges, V not a multiple of the 64/128-column tiles, and the bf16 dlogits of the backward (zero past V
and on ignored rows). Tolerances: CE / lse 2e-4 relative (f32 exp / log), dlogits bf16 rounding."""
import pytest
import torch

from simlingo_amd import kernels as K

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,V,D", [(37, 1000, 128), (5, 64, 64), (128, 151655, 896)])
def test_lmhead_ce_fused(dev, R, V, D):
    g = torch.Generator(device=dev).manual_seed(R + V)
    Vp = (V + 127) // 128 * 128
    feat = (torch.randn(R, D, device=dev, generator=g) * 2).bfloat16()
    W = torch.zeros(Vp, D, device=dev, dtype=torch.bfloat16)
    W[:V] = (torch.randn(V, D, device=dev, generator=g) * 0.5).bfloat16()
    lab = torch.randint(0, V, (R,), device=dev, generator=g, dtype=torch.int32)
    lab[0] = 0
    lab[-1] = V - 1
    if R > 2:
        lab[1] = -1
    loss = torch.empty(R, device=dev)
    lse = torch.empty(R, device=dev)
    nws = K.lib().slx_lmhead_ce_ws_floats(R, V)
    ws = torch.empty(nws, device=dev)
    K.call("slx_lmhead_ce_fwd", K.P(feat), D, K.P(W), D, K.P(lab), R, V, D, K.P(loss), K.P(lse), K.P(ws), nws,
           K.stream_ptr())
    logits = feat.float() @ W[:V].float().t()
    ref_lse = torch.logsumexp(logits, 1)
    ref = torch.nn.functional.cross_entropy(logits, lab.long(), ignore_index=-1, reduction="none")
    torch.testing.assert_close(lse, ref_lse, rtol=2e-4, atol=2e-4)
    torch.testing.assert_close(loss, ref, rtol=2e-4, atol=2e-4)
    gs = torch.tensor([0.37], device=dev)
    dlog = torch.full((R, Vp), float("nan"), device=dev, dtype=torch.bfloat16)
    K.call("slx_lmhead_ce_bwd", K.P(feat), D, K.P(W), D, K.P(lab), K.P(lse), R, V, D, K.P(gs), K.P(dlog), Vp,
           K.stream_ptr())
    sm = torch.softmax(logits, 1)
    valid = lab >= 0
    oh = torch.zeros_like(sm)
    oh[valid, lab[valid].long()] = 1.0
    want = (sm - oh) * 0.37 * valid[:, None]
    torch.testing.assert_close(dlog[:, :V].float(), want, atol=2e-3, rtol=1e-2)
    assert torch.all(dlog[:, V:] == 0)
