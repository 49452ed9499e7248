"""The drop-in training loop (bench.py `dropin` key) is the engine step and nothing else: DataLoader (Collate.host in
the loader) -> Collate.device (pinned-ring H2D + HIP frame kernel) -> DrivingModel.training_step -> loss.backward()
-> FusedAdamW.step -> OneCycleLR.step, against VLAEngine stepped directly on the same collated batches at the same
step seed and parameters (tiny geometry, LoRA dropout on). Run in deterministic-reduction mode (every cross-block f32
sum in a fixed order), so the two paths must agree BIT FOR BIT: each step's losses and its whole gradient buffer (the
optimizer call itself is pinned by test_driving_dropin_gpu / test_adamw_gpu)."""
import pytest
import torch

from simlingo_amd import kernels as K

from chat_util import build_tokenizer
from test_collate_cpu import _samples

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore::UserWarning")]


def test_dropin_loop_equals_engine_steps(dev):
    from torch.utils.data import DataLoader
    from simlingo_amd.collate import Collate
    from simlingo_amd.config import tiny_config
    from simlingo_amd.driving import DrivingModel
    from simlingo_amd.engine import VLAEngine
    from simlingo_amd.params import init_params
    cfg = tiny_config(lora_dropout=0.1)
    col = Collate(build_tokenizer(), num_image_tokens_per_patch=cfg.img_tokens_per_tile, num_image_patches=cfg.tiles,
                  device=dev, input_size=cfg.img_size)
    data = _samples(cfg, 12, seed=5)
    loader = DataLoader(data, batch_size=4, shuffle=False, num_workers=0, collate_fn=col.host)
    P = init_params(cfg, seed=3, lora_b_std=0.05, std=0.05)
    m = DrivingModel(vision_model={"variant": "tiny"}, language_model={"variant": "tiny", "lora_dropout": 0.1},
                     lr=1e-3, init_params=P)
    m.max_steps = 8
    m.build_engine(dev)
    conf = m.configure_optimizers()
    opt, sched = conf["optimizer"], conf["lr_scheduler"]["scheduler"]
    ref = VLAEngine(m.vla_cfg, dev, P)
    K.set_deterministic(True, dev)
    try:
        _run(m, ref, col, loader, opt, sched, dev)
    finally:
        K.set_deterministic(False)


def _run(m, ref, col, loader, opt, sched, dev):
    from simlingo_amd.plan import plan_from_example
    for i, hb in enumerate(loader):
        ex = col.device(hb)
        assert ex.driving_input.camera_images.is_cuda
        # the reference engine starts every step from the drop-in model's current parameters and step seed
        ref.master.copy_(m.engine.master)
        ref.wbf.copy_(m.engine.wbf)
        ref._refresh_derived()
        ref.step_seed = m.engine.step_seed
        out = m.training_step(ex, i)
        out["loss"].backward()
        plan = plan_from_example(m.vla_cfg, ex)
        lab = ex.driving_label
        out4, _, _ = ref.forward(ex.driving_input.camera_images, plan, plan.to_device(dev), lab.path.to(dev),
                                 lab.waypoints.to(dev), training=True)
        ref.backward(None)
        torch.cuda.synchronize()
        assert out["loss"].item() == out4[0].item(), (i, out["loss"].item(), out4[0].item())
        g, r = m.engine.grad, ref.grad
        assert torch.equal(g, r), (i, ((g - r).norm() / r.norm()).item())
        opt.step()
        sched.step()
        opt.zero_grad()
    assert i == 2 and opt.step_count == 3
