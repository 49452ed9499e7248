import sys, torch, numpy as np
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
from golden_util import load_case
from oracle import vla_oracle as O
from test_vla_parity_gpu import run_engine, engine_precision_params
dev = torch.device("cuda")
for case in ["nopad", "leftpad"]:
    cfg, P, ex, z = load_case(case)
    eng, out4, rp, sp = run_engine(cfg, P, ex, dev)
    ref, grads = O.loss_and_grads(engine_precision_params(eng, P), cfg, ex)
    rows = []
    for name, g in grads.items():
        e = eng.G[name].detach().float().cpu().reshape(-1); r = g.reshape(-1)
        if r.norm() < 1e-12: continue
        rows.append((torch.nn.functional.cosine_similarity(e, r, dim=0).item(), ((e - r).norm() / r.norm()).item(), name))
    rows.sort()
    print(case, [(round(a, 4), round(b, 4), n) for a, b, n in rows[:8]])
