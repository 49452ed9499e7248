"""The attention kernel forms behind the SLX_ATTN_* switches (read once per process, so each form runs in one child
process) against the same plain PyTorch fp32 attention as tests/test_attention_gpu.py, every case of its CASES:
  SLX_ATTN_DMA=0  the register-staged forward / dQ / dK-dV kernels (rounds 1-3),
  SLX_ATTN_PP=1   the ping-pong dQ pass (8 waves, MFMA / VALU phases alternating between two wave groups)."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, torch
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import test_attention_gpu as T
dev = torch.device("cuda:0")
for case in T.CASES:
    T.test_attention_fwd_bwd(dev, *case)
print("OK", len(T.CASES))
"""


@pytest.mark.parametrize("env", ["SLX_ATTN_DMA=0", "SLX_ATTN_PP=1"])
def test_attention_form(dev, env):
    k, v = env.split("=")
    code = CHILD.format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180,
                       env=dict(os.environ, **{k: v}))
    assert r.returncode == 0 and "OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])
