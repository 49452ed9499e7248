"""Phase timing of GreedyDecoder.generate on the full geometry (real decode steps: eos = -1 never matches)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from simlingo_amd.config import full_config  # noqa: E402
from simlingo_amd.decode import GreedyDecoder  # noqa: E402
from simlingo_amd.engine import VLAEngine  # noqa: E402
from simlingo_amd.params import init_params  # noqa: E402

dev = torch.device("cuda", 0)
cfg = full_config()
eng = VLAEngine(cfg, dev, init_params(cfg, seed=0, lora_b_std=0.02, device=dev))
dec = GreedyDecoder(eng, max_len=1024, max_new_tokens=int(os.environ.get("NEW", "100")), eos_id=-7)
prefix = torch.randn(576, cfg.llm_dim, device=dev) * 0.02
for it in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    toks = dec.generate(prefix)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    print(f"generate {1e3*(t1-t0):.2f} ms n={len(toks)} timing={dec.last_timing}", flush=True)
