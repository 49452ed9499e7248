import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import torch
from golden_util import load_case
from oracle import vla_oracle as O
from test_vla_parity_gpu import run_engine
for case in sys.argv[1:] or ["leftpad"]:
    cfg, P, ex, z = load_case(case)
    ref, grads = O.loss_and_grads(P, cfg, ex)
    eng, out4, rp, sp = run_engine(cfg, P, ex, "cuda")
    print(case, "losses", out4.tolist(), [ref[k].item() for k in ("loss", "language_loss", "route_loss", "speed_wps_loss")])
    print(" route maxdiff per sample", (rp - ref["route_pred"]).abs().amax((1, 2)).tolist())
    print(" speed maxdiff per sample", (sp - ref["speed_pred"]).abs().amax((1, 2)).tolist())
    for name, g in grads.items():
        e = eng.G[name].float().cpu().reshape(-1); r = g.reshape(-1)
        if r.norm() < 1e-12: continue
        cos = torch.nn.functional.cosine_similarity(e, r, dim=0).item(); rel = ((e - r).norm() / r.norm()).item()
        if cos < 0.995 or rel > 0.1: print(f"  {name:28s} cos {cos:.4f} rel {rel:.4f}")
