"""Drop-in SimLingo-Base surface (simlingo_amd.base_driving): the constructor contract and optimizer groups on
CPU; on the MI355X the Lightning-style step (training_step -> loss.backward() -> configure_optimizers() step)
reproduces the BaseEngine calls, and forward() returns the heads' predictions."""
import pytest
import torch

from simlingo_amd.base_driving import BaseFusedAdamW, DrivingModel, Llama, LLaVAnextEncoderModel


def _tiny(**kw):
    return DrivingModel(LLaVAnextEncoderModel("tiny", embed_dim=128, freeze=False), Llama("debug-tiny"), **kw)


def test_geometry_and_errors():
    m = DrivingModel(LLaVAnextEncoderModel("llava-hf/llava-v1.6-mistral-7b-hf", 512, False), Llama("tiny"),
                     lr=3e-5, vision_lr=3e-5)
    c = m.base_cfg
    assert (c.llm_layers, c.llm_dim, c.llm_heads, c.llm_ffn, c.vit_used) == (12, 512, 8, 2048, 23)
    assert c.img_tokens == 200 and c.seq == 233   # BASELINE.md config 2 (1024 x 359 frame)
    with pytest.raises(NotImplementedError):
        LLaVAnextEncoderModel("tiny", 128, freeze=True)
    with pytest.raises(ValueError):
        Llama("x-small")
    with pytest.raises(NotImplementedError):
        Llama("tiny", lora=True)
    with pytest.raises(NotImplementedError):
        _tiny(speed_wps_mode="1d")


def test_optimizer_groups_follow_configure_params_groups():
    m = _tiny(lr=1e-3, vision_lr=2e-3)
    opt = BaseFusedAdamW(m, lr=1e-3, vision_lr=2e-3, weight_decay=0.1)
    assert [(g["lr"], g["weight_decay"]) for g in opt.param_groups] == [(1e-3, 0.1), (1e-3, 0.0), (2e-3, 0.1),
                                                                        (2e-3, 0.0)]
    torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=[g["lr"] for g in opt.param_groups], total_steps=100,
                                        pct_start=0.05)
    assert opt.param_groups[2]["lr"] == pytest.approx(2 * opt.param_groups[0]["lr"])


@pytest.mark.gpu
def test_lightning_step_matches_engine(dev):
    from base_golden_util import load_base_case
    from simlingo_amd.base_engine import BaseEngine
    cfg, P, ex, _ = load_base_case()
    m = _tiny(lr=1e-3, vision_lr=2e-3, init_params=P)
    m.build_engine(dev)
    assert m.base_cfg == cfg.replace(lr=1e-3, vision_lr=2e-3)
    loss = m.training_step(ex)["loss"]
    loss.backward()
    opt = m.configure_optimizers()["optimizer"]
    opt.step()
    ref = BaseEngine(cfg, dev, P)
    di, dl = ex.driving_input, ex.driving_label
    out4, _, _ = ref.forward(di.camera_images.to(dev), di.vehicle_speed.to(dev), di.map_route.to(dev),
                             dl.route_adjusted.to(dev), dl.waypoints.to(dev), image_size=(cfg.frame_h, cfg.frame_w))
    ref.backward(None)
    g0, g2 = opt.param_groups[0], opt.param_groups[2]
    ref.adamw_step(g0["lr"], g2["lr"], 1, betas=g0["betas"], eps=g0["eps"], weight_decay=0.1, max_norm=1.0)
    torch.cuda.synchronize()
    assert abs(loss.item() - out4[0].item()) <= 1e-5 * abs(out4[0].item())
    torch.testing.assert_close(m.engine.master, ref.master, rtol=1e-5, atol=1e-6)
    sp, rp = m.forward(ex.driving_input)
    B = di.camera_images.shape[0]
    assert sp.shape == (B, cfg.n_speed, 2) and rp.shape == (B, cfg.n_route, 2)
    losses, preds = m.forward_loss(ex, per_sample=True)
    assert losses["route_loss"][0].shape == (B,) and preds["route_prediction"].shape == (B, cfg.n_route, 2)
