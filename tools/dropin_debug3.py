"""Drop-in NaN bisect (host runs ahead, no per-step sync): which part of the DrivingModel loop breaks it.
modes: full | noautograd (engine.backward called directly) | rawopt (loss.backward, engine.adamw_step directly)"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dl = bench.dropin_loader(steps=4, warmup=1)
import torch  # noqa: E402
from simlingo_amd.driving import DrivingModel  # noqa: E402
from simlingo_amd.params import init_params  # noqa: E402

dev = torch.device("cuda", 0)
cfg, col, it = dl["cfg"], dl["col"], dl["it"]
mode = sys.argv[1] if len(sys.argv) > 1 else "full"
variant = {"variant": "OpenGVLab/InternVL2-1B"}
m = DrivingModel(vision_model=dict(variant), language_model=dict(variant, lora=True, lora_r=32, lora_alpha=64,
                                                                 lora_dropout=0.1),
                 lr=cfg.lr, init_params=init_params(cfg, seed=0, lora_b_std=0.02, device=dev))
m.max_steps = 10000
m.build_engine(dev)
conf = m.configure_optimizers()
opt, sched = conf["optimizer"], conf["lr_scheduler"]["scheduler"]
outs = []
diag = []
if os.environ.get('UPLOAD_SYNC') == '1':
    from simlingo_amd import frames as _fr
    _orig = _fr.FrameUploader.__call__
    def _sync_call(self, f):
        d = _orig(self, f)
        torch.cuda.synchronize()
        return d
    _fr.FrameUploader.__call__ = _sync_call
probe = []
if os.environ.get("PROBE") == "1":  # finiteness of the flat gradient after every parameter group's backward
    _eng = m.engine
    _gd = _eng._group_done
    def _probe_done(g, _gd=_gd, _eng=_eng):
        probe.append((len(outs), g, torch.isfinite(_eng.grad).all()))
        return _gd(g)
    _eng._group_done = _probe_done
SYNC_AT = os.environ.get("SYNC_AT", "")
def _sync(tag):
    if tag in SYNC_AT.split(","):
        torch.cuda.synchronize()
for i in range(5):
    _sync("pre")
    hb = next(it)
    _sync("next")
    ex = col.device(hb)
    _sync("col")
    if mode == "noautograd":
        o, _ = m.forward_loss(ex)
        loss = o.loss.detach()
        _sync("fwd")
        m.engine.backward(None)
        _sync("bwd")
    else:
        out = m.training_step(ex, 0)
        loss = out["loss"]
        loss.backward()
    if mode == "rawopt":
        m.engine.adamw_step(1.2e-6, i + 1, betas=(0.95, 0.999), eps=cfg.eps, weight_decay=cfg.weight_decay,
                            max_norm=cfg.grad_clip)
    else:
        opt.step()
        sched.step()
    _sync("opt")
    opt.zero_grad()
    e = m.engine
    diag.append(torch.stack([torch.isfinite(e.grad).all().float(), torch.linalg.vector_norm(e.grad.float()),
                             torch.isfinite(e.master).all().float(), torch.isfinite(e.wbf).all().float(),
                             torch.isfinite(ex.driving_input.camera_images).all().float()]))
    outs.append(loss)
    print(mode, i, "lr", opt.param_groups[0]["lr"], "betas", opt.param_groups[0]["betas"], flush=True)
torch.cuda.synchronize()
print(mode, "losses", [round(x.item(), 4) for x in outs], flush=True)
for i, d in enumerate(diag):
    print(mode, i, "grad finite, grad norm, master finite, wbf finite, pix finite", [round(v, 4) for v in d.tolist()],
          flush=True)
bad = {}
for st, g, f in probe:
    if not bool(f.item()) and st not in bad:
        bad[st] = g
print(mode, "first non-finite group per step", bad, "groups in order", [g for st, g, f in probe if st == 0][:6], flush=True)
