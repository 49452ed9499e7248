"""LoRA dropout: the hash mask applied while loading A (down-projection), while loading B (dA GEMM) and
in the DROPMASK epilogue (dx) is one function of (seed, row*ldmask + col); checked against a PyTorch
fp32 reference that applies the host mirror of the mask (simlingo_amd/dropmask.py)."""
import numpy as np
import pytest
import torch

from simlingo_amd import kernels as K
from simlingo_amd.dropmask import keep_scale

pytestmark = pytest.mark.gpu


def test_dropout_mask_consistency(dev):
    M, kin, r, p, seed = 300, 256, 32, 0.1, 987654321
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(M, kin, device=dev, generator=g).bfloat16()
    A = (torch.randn(r, kin, device=dev, generator=g) * 0.1).bfloat16()
    mask = torch.from_numpy(keep_scale(seed, M, kin, kin, p)).to(dev)
    assert 0.85 < (mask > 0).float().mean().item() < 0.95
    xd = (x.float() * mask).bfloat16().float()  # the kernels round the scaled, masked input to bf16
    # forward: t = drop(x) A^T  (mask on the A operand)
    t = torch.empty(M, r, device=dev, dtype=torch.float32)
    K.mm(x, A, t, drop_operand=1, seed=seed, drop_p=p, ldmask=kin)
    torch.testing.assert_close(t, xd @ A.float().t(), atol=2e-2, rtol=2e-2)
    # dA = dt^T drop(x)  (mask on the B operand, TN layout)
    dt = torch.randn(M, r, device=dev, generator=g).bfloat16()
    dA = torch.zeros(r, kin, device=dev)
    K.mm(dt, x, dA, ta=True, tb=False, drop_operand=2, seed=seed, drop_p=p, ldmask=kin, accumulate=True)
    torch.testing.assert_close(dA, dt.float().t() @ xd, atol=2e-2, rtol=1e-2)
    # dx += mask * (dt A)  (epilogue)
    dx = torch.ones(M, kin, device=dev)
    K.mm(dt, A, dx, tb=False, epi=K.EPI_DROPMASK, accumulate=True, seed=seed, drop_p=p, ldmask=kin)
    torch.testing.assert_close(dx, 1 + mask * (dt.float() @ A.float()), atol=2e-2, rtol=2e-2)
    # standalone dropout kernel agrees too
    y = torch.empty_like(x)
    K.call("slx_dropout", K.P(x), kin, K.P(y), kin, M, kin, seed, p, kin, K.stream_ptr())
    torch.testing.assert_close(y.float(), (x.float() * mask).bfloat16().float())
