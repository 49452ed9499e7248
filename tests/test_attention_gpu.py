"""Flash-attention parity: HIP fwd/bwd vs a plain PyTorch fp32 attention of the same bf16 inputs.

Mask semantics follow the reference's call sites: InternViT is non-causal over all tokens; Qwen2 is
causal with a key-padding mask over a valid-first (right-padded) layout, so query row q may attend key
k iff k < len_b and k <= q (padded query rows attend all valid keys, as SDPA does).
"""
import math

import pytest
import torch

from simlingo_amd import kernels as K

pytestmark = pytest.mark.gpu


def ref_attn(q, k, v, B, S, Hq, Hkv, causal, lens):
    # q: [B*S, Hq*64] ... -> fp32 math
    q = q.float().view(B, S, Hq, 64).transpose(1, 2)
    k = k.float().view(B, S, Hkv, 64).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    v = v.float().view(B, S, Hkv, 64).transpose(1, 2).repeat_interleave(Hq // Hkv, 1)
    s = q @ k.transpose(-1, -2) / 8.0
    kk = torch.arange(S, device=q.device)
    allowed = kk[None, None, :] < torch.tensor(lens, device=q.device)[:, None, None]
    if causal:
        allowed = allowed & (kk[None, None, :] <= kk[None, :, None])
    s = s.masked_fill(~allowed[:, None], float("-inf"))
    o = torch.softmax(s, -1) @ v
    return o.transpose(1, 2).reshape(B * S, Hq * 64)


CASES = [
    # B, S, Hq, Hkv, causal, lens
    (2, 1025, 2, 2, False, None),
    # the row tail folded into the last whole block (S % 128 in 1..2): 129 = 1 block + 1, 258 = 2 blocks + 2; 1027
    # (3 rows: not folded) and 1024 (no tail) keep the plain layout
    (2, 129, 2, 2, False, None),
    (1, 258, 3, 3, False, None),
    (1, 1027, 2, 2, False, None),
    (1, 1024, 1, 1, False, None),
    (3, 200, 4, 4, False, None),
    (2, 150, 14, 2, True, [150, 97]),
    (1, 64, 2, 1, True, None),
    (2, 333, 7, 7, True, [300, 5]),
]


@pytest.mark.parametrize("B,S,Hq,Hkv,causal,lens", CASES)
def test_attention_fwd_bwd(dev, B, S, Hq, Hkv, causal, lens):
    torch.manual_seed(B * 1000 + S)
    lens = lens or [S] * B
    W = (Hq + 2 * Hkv) * 64
    qkv = (torch.randn(B * S, W, device=dev) * 1.5).bfloat16()
    q, k, v = qkv[:, : Hq * 64], qkv[:, Hq * 64: (Hq + Hkv) * 64], qkv[:, (Hq + Hkv) * 64:]
    seql = torch.tensor(lens, device=dev, dtype=torch.int32)
    o = torch.empty(B * S, Hq * 64, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * Hq * S, device=dev)
    K.attn_fwd(q, k, v, o, lse, B=B, S=S, Hq=Hq, Hkv=Hkv, causal=causal, seqlens=seql)
    qr, kr, vr = (t.detach().clone().float().requires_grad_() for t in (q, k, v))
    ref = ref_attn(qr, kr, vr, B, S, Hq, Hkv, causal, lens)
    err = (o.float() - ref).abs().max().item()
    assert err < 2e-2, f"fwd max err {err}"
    dout = torch.randn(B * S, Hq * 64, device=dev).bfloat16()
    ref.backward(dout.float())
    dqkv = torch.zeros_like(qkv)
    dq, dk, dv = dqkv[:, : Hq * 64], dqkv[:, Hq * 64: (Hq + Hkv) * 64], dqkv[:, (Hq + Hkv) * 64:]
    ws = K.attn_ws(B, S, Hq, Hkv, dev)
    # the q/k/v bias-gradient column sums ride along where dK/dV take the bf16 path (no GQA; RoPE is not used here)
    dbias = torch.full((3 * Hq * 64,), 0.25, device=dev) if Hq == Hkv else None
    K.attn_bwd(q, k, v, o, lse, dout, dq, dk, dv, ws, B=B, S=S, Hq=Hq, Hkv=Hkv, causal=causal, seqlens=seql,
               dbias=dbias)
    for name, got, want in (("dq", dq, qr.grad), ("dk", dk, kr.grad), ("dv", dv, vr.grad)):
        scale = want.abs().max().item() + 1e-6
        e = (got.float() - want).abs().max().item()
        assert e < 3e-2 * scale + 1e-2, f"{name}: max err {e} (scale {scale})"
    if dbias is not None:  # sums of the stored bf16 gradients over all B*S rows, f32 accumulation
        want = 0.25 + dqkv.float().sum(0)
        torch.testing.assert_close(dbias, want, atol=1e-3 * (B * S) ** 0.5, rtol=1e-4)


def test_rope_roundtrip_and_values(dev):
    B, S, H = 2, 40, 3
    x = torch.randn(B * S, H * 64, device=dev).bfloat16()
    cos, sin = K.rope_tables(S, 1e6, dev)
    y = x.clone()
    K.rope(y, B * S, S, H, cos, sin)
    # reference: rotate_half convention
    xf = x.float().view(B, S, H, 64)
    c = torch.cat([cos, cos], -1)[None, :, None, :]
    s = torch.cat([sin, sin], -1)[None, :, None, :]
    rot = torch.cat([-xf[..., 32:], xf[..., :32]], -1)
    ref = (xf * c + rot * s).view(B * S, H * 64)
    assert (y.float() - ref).abs().max().item() < 2e-2
    z = y.clone()
    K.rope(z, B * S, S, H, cos, sin, inverse=True)
    assert (z.float() - x.float()).abs().max().item() < 4e-2
