"""slx_dec_attn_o_split_ok (host function, no GPU): the split decode attention's cache-length limit follows
SLX_DEC_SPLIT_NS, so GreedyDecoder can fall back to slx_dec_attn + the O GEMV instead of failing the C argument check
(the Python guard used to assume the default split count)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = """
import sys
sys.path.insert(0, {root!r})
from simlingo_amd import kernels as K
import simlingo_amd.decode  # registers the decode entry points
print([int(K.lib().slx_dec_attn_o_split_ok(n)) for n in (1, 512, 513, 2048, 2049)])
"""


def _probe(ns):
    env = dict(os.environ)
    env.pop("SLX_DEC_SPLIT_NS", None)
    if ns is not None:
        env["SLX_DEC_SPLIT_NS"] = str(ns)
    out = subprocess.run([sys.executable, "-c", PROBE.format(root=ROOT)], env=env, capture_output=True, text=True,
                         timeout=120)
    assert out.returncode == 0, out.stderr
    return eval(out.stdout.strip().splitlines()[-1])


def test_split_limit_follows_split_count():
    assert _probe(None) == [1, 1, 1, 1, 0]   # 8 splits x 8 blocks of 32 keys: up to 2048 rows
    assert _probe(2) == [1, 1, 0, 0, 0]      # 2 splits: up to 512 rows
    assert _probe(0) == [0, 0, 0, 0, 0]      # an invalid count disables the split path
