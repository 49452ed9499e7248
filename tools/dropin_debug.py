"""Drop-in loop per-step losses (bench.py dropin_line) for bisecting a bad loss: python tools/dropin_debug.py [steps]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 4
dl = bench.dropin_loader(steps=steps, warmup=1)
import torch  # noqa: E402
dev = torch.device("cuda", 0)
res = bench.dropin_line(dl, dev)
print(json.dumps(res))
