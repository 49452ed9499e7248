"""slx_adamw: the four-per-lane kernel (aligned bulk) and the scalar kernel (tail, unaligned slices) against the same
update written in torch f32 (decoupled weight decay, bias corrections, global-norm clip, bf16 working copy)."""
import pytest
import torch

from simlingo_amd import kernels as K

pytestmark = pytest.mark.gpu


def _ref(p, g, m, v, lr, b1, b2, eps, wd, step, max_norm, gscale):
    tn = torch.sqrt((g.double() ** 2).sum()).float() * gscale
    coef = gscale * min(1.0, max_norm / (tn.item() + 1e-6)) if max_norm > 0 else gscale
    gi = g * coef
    p = p * (1 - lr * wd)
    m = m + (1 - b1) * (gi - m)
    v = v * b2 + (1 - b2) * gi * gi
    den = torch.sqrt(v) / ((1 - b2 ** step) ** 0.5) + eps
    p = p - (lr / (1 - b1 ** step)) * m / den
    return p, m, v


@pytest.mark.parametrize("off,n", [(0, 4099), (1, 4099), (0, 3), (4, 1 << 20)])
def test_adamw(dev, off, n):
    gen = torch.Generator(device=dev).manual_seed(n + off)
    buf = [torch.randn(n + off, device=dev, generator=gen) for _ in range(4)]
    buf[3] = buf[3].abs()
    p, g, m, v = [b[off:] for b in buf]
    pbf_buf = torch.zeros(n + off, device=dev, dtype=torch.bfloat16)
    pbf = pbf_buf[off:]
    want = _ref(p.clone(), g.clone(), m.clone(), v.clone(), 1e-3, 0.9, 0.999, 1e-8, 0.1, 3, 0.5, 0.5)
    sumsq = (g.double() ** 2).sum().float().reshape(1)
    K.call("slx_adamw", K.P(p), K.P(g), K.P(m), K.P(v), K.P(pbf), n, 1e-3, 0.9, 0.999, 1e-8, 0.1, 3, K.P(sumsq),
           0.5, 0.5, K.stream_ptr())
    torch.cuda.synchronize()
    for got, ref in zip((p, m, v), want):
        torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)  # FMA contraction vs torch op order
    assert torch.equal(pbf, p.bfloat16())
