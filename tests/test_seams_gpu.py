"""Inner seams of the drop-in DrivingModel (SURVEY.md §8b 'Inner seams'), composed exactly as the reference's
DrivingModel.forward_loss / forward_model compose them (simlingo_training/models/driving.py:190-261):
    adaptor_dict = model.adaptors(example)                                   adaptors.py:301-331
    model.vision_model.image_encoder.replace_placeholder_tokens(adaptor_dict, pixel_values, placeholder_values, wp)
    out = model.language_model.model(attention_mask, position_ids, inputs_embeds, output_hidden_states, return_dict)
    loss_dict = model.adaptors.compute_loss(features, logits, adaptor_dict, example) -> summarise_losses
checked against the golden fixture the reference code produced (permutation, assembled-input checksum, losses) and
the CPU oracle (features, logits); plus LLM.greedy_sample teacher-forced against the oracle. Tolerances: the
bf16 gates of test_vla_parity_gpu.py (losses rel 1e-2)."""
import numpy as np
import pytest
import torch

from golden_util import load_case
from oracle import vla_oracle as O
from test_vla_parity_gpu import engine_precision_params

pytestmark = pytest.mark.gpu


def _model(P, cfg):
    from simlingo_amd.driving import DrivingModel
    return DrivingModel(vision_model={"variant": "tiny"}, language_model={"variant": "tiny", "lora_dropout": 0.0},
                        init_params=P)


@pytest.mark.parametrize("case", ["nopad", "leftpad"])
def test_reference_composition_of_seams(dev, case):
    cfg, P, ex, z = load_case(case)
    model = _model(P, cfg)
    model.build_engine(dev)
    ad = model.adaptors(ex)
    np.testing.assert_array_equal(ad["perm"].cpu().numpy(), z["out.perm"])
    np.testing.assert_array_equal(ad["inputs_mask"].cpu().numpy(), z["out.inputs_mask"])
    assert [int(x) for x in ad["split_sizes"]] == [ex.driving_input.prompt.phrase_ids.shape[1], cfg.n_queries]
    di = ex.driving_input
    res = model.vision_model.image_encoder.replace_placeholder_tokens(
        adaptor_dict=ad, pixel_values=di.camera_images, placeholder_values=di.prompt.placeholder_values,
        wp_encoder=None)
    assert res is ad
    x = ad["inputs"].double()
    np.testing.assert_allclose([x.sum().item(), x.abs().sum().item()], z["out.inputs_sum"], rtol=1e-2, atol=1e-2)
    out = model.language_model.model(attention_mask=ad["inputs_mask"], position_ids=None, inputs_embeds=ad["inputs"],
                                     output_hidden_states=True, return_dict=True)
    features, logits = out.hidden_states[-1], out[0]
    Pe = engine_precision_params(model.engine, P)
    ref_feat, ref_logits = O.llm_forward(Pe, cfg, ad["inputs"].cpu(), ad["inputs_mask"].cpu())
    mask = ad["inputs_mask"].cpu()
    fe = (features.cpu() - ref_feat)[mask]
    assert (fe.norm() / ref_feat[mask].norm()).item() < 2e-2
    le = (logits.cpu() - ref_logits)[mask]
    assert (le.norm() / ref_logits[mask].norm()).item() < 2e-2
    loss_dict = model.adaptors.compute_loss(features, logits, ad, ex)
    avg = {k: (loss_dict[k][0].sum() / loss_dict[k][1].sum()).item() for k in loss_dict if k.endswith("_loss")}
    assert set(avg) == {"language_loss", "route_loss", "speed_wps_loss"}
    total = sum(avg.values())
    np.testing.assert_allclose([total, avg["language_loss"], avg["route_loss"], avg["speed_wps_loss"]],
                               [float(z["out.loss"]), float(z["out.language_loss"]), float(z["out.route_loss"]),
                                float(z["out.speed_wps_loss"])], rtol=1e-2, atol=1e-4)
    assert loss_dict["route_prediction"].shape == (ex.driving_input.prompt.phrase_ids.shape[0], cfg.n_route, 2)
    with pytest.raises(NotImplementedError):  # masks must be valid-first, as AdaptorList.forward lays them out
        bad = ad["inputs_mask"].clone()
        bad[:, 0] = False
        bad[:, -1] = True
        model.language_model.model(attention_mask=bad, inputs_embeds=ad["inputs"])


def test_extract_feature_and_greedy_sample(dev):
    cfg, P, ex, z = load_case("nopad")
    model = _model(P, cfg)
    model.build_engine(dev)
    pix = ex.driving_input.camera_images
    vit = model.vision_model.image_encoder.extract_feature(pix)
    Pe = engine_precision_params(model.engine, P)
    ref = O.extract_feature(Pe, cfg, pix.reshape(-1, 3, cfg.img_size, cfg.img_size))
    assert vit.shape == ref.shape
    assert ((vit.cpu() - ref).norm() / ref.norm()).item() < 2e-2
    # greedy_sample on the first sample's valid prompt rows vs the oracle's literal re-run-the-prefix loop
    ad = model.adaptors(ex, inference=True)
    model.vision_model.image_encoder.replace_placeholder_tokens(ad, pix, ex.driving_input.prompt_inference
                                                                .placeholder_values, None)
    n0 = int(ad["inputs_mask"][0].sum()) - cfg.n_queries
    emb = ad["inputs"][:1, :n0]
    toks, embeds = model.language_model.greedy_sample(emb, max_new_tokens=6, eos_token_id=None)
    assert toks.shape == (1, 6) and embeds.shape[1] == n0 + 6
    # teacher-forced on the HIP tokens (test_decode_gpu.py's bf16 token gate): each chosen token's oracle logit is
    # within 3e-2 std of the oracle maximum, and identical wherever the oracle's top-2 margin exceeds 0.2 std
    x = torch.cat([emb[0].cpu(), Pe["llm.embed"][toks[0].cpu()]], 0)
    _, lg = O.llm_forward(Pe, cfg, x[None], torch.ones(1, x.shape[0], dtype=torch.bool))
    lg = lg[0, n0 - 1: n0 + 5]
    for i, t in enumerate(toks[0].tolist()):
        std, top2 = lg[i].std().item(), lg[i].topk(2).values
        assert (top2[0] - lg[i, t]).item() <= 3e-2 * std, (i, t)
        if (top2[0] - top2[1]).item() > 0.2 * std:
            assert t == int(lg[i].argmax()), i
    torch.testing.assert_close(embeds[0, n0:].cpu(), Pe["llm.embed"][toks[0].cpu()])


def test_replace_placeholder_tokens_honours_caller_values_and_encoder(dev):
    """internvl2_model.py:53-91 reads the caller's placeholder_values and calls the caller's wp_encoder: other
    coordinates move exactly the <TARGET_POINT> rows; a torch WaypointInputAdaptor holding the engine's weights
    reproduces the engine's own rows; every other row of `inputs` is untouched."""
    from torch import nn
    cfg, P, ex, _ = load_case("nopad")
    model = _model(P, cfg)
    model.build_engine(dev)
    enc = model.vision_model.image_encoder
    di = ex.driving_input
    base = model.adaptors(ex)
    enc.replace_placeholder_tokens(base, di.camera_images, di.prompt.placeholder_values, None)
    pv2 = [{k: np.asarray(v, dtype=np.float32) + 1.5 for k, v in d.items()} for d in di.prompt.placeholder_values]
    moved = model.adaptors(ex)
    enc.replace_placeholder_tokens(moved, di.camera_images, pv2, None)
    plan = moved["_plan"]
    B, S, d = plan.B, plan.S, cfg.llm_dim
    pos = torch.from_numpy(plan.wp_pos[plan.wp_pos < B * S].astype(np.int64))
    assert pos.numel() > 0
    xb, xm = base["inputs"].reshape(B * S, d).cpu(), moved["inputs"].reshape(B * S, d).cpu()
    other = torch.ones(B * S, dtype=torch.bool)
    other[pos] = False
    assert torch.equal(xb[other], xm[other])
    assert (xb[pos] - xm[pos]).abs().max().item() > 1e-3

    class WaypointInputAdaptor(nn.Module):  # adaptors.py:64-93 layout
        def __init__(self):
            super().__init__()
            self.mlp = nn.Sequential(nn.Linear(2, cfg.wp_hidden), nn.ReLU(True), nn.Linear(cfg.wp_hidden, cfg.wp_hidden2),
                                     nn.ReLU(True), nn.Linear(cfg.wp_hidden2, d))

        def forward(self, x):
            return self.mlp(x)
    wp = WaypointInputAdaptor().to(dev)
    with torch.no_grad():
        for i, j in ((0, 0), (1, 2), (2, 4)):
            wp.mlp[j].weight.copy_(model.engine.P[f"wp.{i}.w"].float())
            wp.mlp[j].bias.copy_(model.engine.P[f"wp.{i}.b"].float())
    ext = model.adaptors(ex)
    enc.replace_placeholder_tokens(ext, di.camera_images, pv2, wp)
    xe = ext["inputs"].reshape(B * S, d).cpu()
    assert torch.equal(xe[other], xm[other])
    torch.testing.assert_close(xe[pos], xm[pos], atol=1e-4, rtol=1e-4)
