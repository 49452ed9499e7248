"""Drop-in NaN bisect: per batch, check the collated inputs and run the raw engine step on them."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dl = bench.dropin_loader(steps=4, warmup=1)
import torch  # noqa: E402
from simlingo_amd.engine import VLAEngine  # noqa: E402
from simlingo_amd.params import init_params  # noqa: E402
from simlingo_amd.plan import plan_from_example  # noqa: E402
dev = torch.device("cuda", 0)
cfg, col, it = dl["cfg"], dl["col"], dl["it"]
eng = VLAEngine(cfg, dev, init_params(cfg, seed=0, lora_b_std=0.02, device=dev))
mode = sys.argv[1] if len(sys.argv) > 1 else "fresh"
first = None
outs = []
for i in range(5):
    hb = next(it)
    ex = col.device(hb)
    if mode == "same":
        first = first or ex
        ex = first
    pix = ex.driving_input.camera_images
    plan = plan_from_example(cfg, ex)
    dplan = plan.to_device(dev, extra={"path": ex.driving_label.path, "waypoints": ex.driving_label.waypoints})
    out4, rp, sp = eng.forward(pix, plan, dplan, dplan["path"], dplan["waypoints"], training=True)
    eng.backward(None)
    if mode == "nosync":  # the bench's host-runs-ahead regime: no host synchronisation inside the loop
        outs.append(out4.clone())
        eng.adamw_step(1.2e-6, i + 1, betas=(0.95, 0.999), eps=cfg.eps, weight_decay=cfg.weight_decay,
                       max_norm=cfg.grad_clip)
        continue
    gn = torch.linalg.vector_norm(eng.grad).item()
    eng.adamw_step(1.2e-6, i + 1, betas=(0.95, 0.999), eps=cfg.eps, weight_decay=cfg.weight_decay, max_norm=cfg.grad_clip)
    torch.cuda.synchronize()
    print(i, "pix finite", bool(torch.isfinite(pix).all()), "pix absmax", pix.abs().max().item(), "loss", out4.tolist(),
          "grad norm", gn, "master finite", bool(torch.isfinite(eng.master).all()), "S", plan.S, "R", plan.loss_pos.shape[0],
          "nwp", plan.wp_coords.shape[0], "wp absmax", float(abs(plan.wp_coords).max()), flush=True)
torch.cuda.synchronize()
for i, o in enumerate(outs):
    print("nosync", i, o.tolist(), flush=True)
