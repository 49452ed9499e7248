"""Collate host path and the config-1 CPU plumbing.

* chat tokens / loss masks vs the reference's own get_chat_tokens / get_assistant_loss_mask (tests/golden/chat_tokens.npz,
  oracle/gen_golden_chat.py): exact;
* the internlm2-chat prompt restatement (conversation.py is a hub download absent from /root/reference: parity
  unpinned for the template text, checked here against its published structure);
* Collate -> DrivingExample -> host token plan -> oracle training step on the tiny geometry (config 1: the CPU side
  of the pipeline up to the engine boundary; the frame tiling is the HIP kernel's job and is stubbed here).
"""
import os

import numpy as np
import pytest
import torch

from chat_util import CONVERSATIONS, build_tokenizer, conversation
from golden_util import GOLDEN
from simlingo_amd import collate as C

pytestmark = pytest.mark.filterwarnings("ignore::UserWarning")


@pytest.fixture(scope="module")
def tok():
    return build_tokenizer()


@pytest.fixture(scope="module")
def z():
    return np.load(os.path.join(GOLDEN, "chat_tokens.npz"), allow_pickle=False)


def test_prompts_follow_the_internlm2_chat_template():
    convs, qs = C.custom_chat_prompts([conversation(q, a) for q, a in CONVERSATIONS], 8)
    img = "<img>" + "<IMG_CONTEXT>" * 8 + "</img>"
    for (q, a), pc, pq in zip(CONVERSATIONS, convs, qs):
        body = q.replace("<image>", img, 1) if "<image>" in q else f"{img}\n{q}"
        assert pc == f"<|im_start|>user\n{body}<|im_end|><|im_start|>assistant\n{a}<|im_end|>"
        assert pq == f"<|im_start|>user\n{body}<|im_end|><|im_start|>assistant\n"
        assert pc.count("<img>") == 1 and "system" not in pc
    with pytest.raises(AssertionError):
        C.custom_chat_prompts([[conversation("a", "b")[1], conversation("a", "b")[0]]], 8)
    with pytest.raises(ValueError):
        C.custom_chat_prompts([[conversation("a", "b")[0], {"role": "tool", "content": [{"text": "x"}]}]], 8)


def test_chat_tokens_match_reference(tok, z):
    convs, qs = C.custom_chat_prompts([conversation(q, a) for q, a in CONVERSATIONS], 8)
    assert list(z["conv.prompts"]) == convs and list(z["question.prompts"]) == qs
    for tag, prompts in (("conv", convs), ("question", qs)):
        d = C.chat_tokens(tok, prompts)
        for k in ("phrase_ids", "phrase_valid", "phrase_mask", "loss_masking"):
            np.testing.assert_array_equal(d[k].numpy(), z[f"{tag}.{k}"], err_msg=f"{tag}.{k}")
    # left padding; the question prompt ends at the assistant role, so its loss mask is the role tokens only
    ids = torch.from_numpy(z["question.phrase_ids"])
    assert (ids[:, -1] != tok.pad_token_id).all()
    assert (torch.from_numpy(z["question.loss_masking"]).sum(1) == len(tok(C.ROLES[1])["input_ids"])).all()


def test_multi_round_loss_mask(z):
    us = [[0, 10, 20], [3, 15]]
    as_ = [[5, 12, 25], [8, 29]]
    got = C.assistant_loss_mask(us, as_, torch.zeros(2, 30, dtype=torch.long))
    np.testing.assert_array_equal(got.numpy(), z["multi.loss_mask"])
    with pytest.raises(AssertionError):
        C.assistant_loss_mask([[5]], [[3]], torch.zeros(1, 8, dtype=torch.long))


def _samples(cfg, B, H=48, W=96, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for b in range(B):
        q, a = CONVERSATIONS[b % len(CONVERSATIONS)]
        out.append(C.DatasetOutput(
            image_ff=rng.integers(0, 256, size=(1, 3, H, W), dtype=np.uint8), image_ff_org_size=(H, W),
            conversation=conversation(q, a), answer=[conversation(q, a)[1]],
            placeholder_values={t: rng.normal(0, 10, size=(1, 2)).astype(np.float32)
                                for t in C.PLACEHOLDER_TOKENS if t in q},
            waypoints=np.cumsum(rng.normal((0.8, 0), 0.3, size=(cfg.n_speed, 2)), 0).astype(np.float32),
            path=np.cumsum(rng.normal((1.0, 0), 0.1, size=(cfg.n_route, 2)), 0).astype(np.float32),
            speed=np.float32([rng.uniform(0, 10)]), target_points=rng.normal(0, 10, size=(2,)).astype(np.float32),
            measurement_path=f"run_{b}/measurements/{b:04d}.json.gz"))
    return out


def test_collate_to_engine_boundary_config1(tok):
    """Config 1 plumbing on the CPU: collate -> DrivingExample -> token plan -> one oracle training step."""
    from oracle import vla_oracle as O
    from simlingo_amd.config import tiny_config
    from simlingo_amd.params import init_params
    from simlingo_amd.plan import plan_from_example
    cfg = tiny_config()
    calls = []

    def pixel_stub(frames_u8, max_num_grid):  # stands in for the HIP frame kernel (uint8 [B, 3, H, W])
        calls.append((tuple(frames_u8.shape), frames_u8.dtype, max_num_grid))
        g = torch.Generator().manual_seed(int(frames_u8.sum()))
        B = frames_u8.shape[0]
        return {"pixel_values": torch.randn(B, cfg.tiles, 3, cfg.img_size, cfg.img_size, generator=g),
                "image_sizes": torch.tensor([[frames_u8.shape[2], frames_u8.shape[3]]] * B)}

    col = C.Collate(tok, num_image_tokens_per_patch=cfg.img_tokens_per_tile, num_image_patches=cfg.tiles,
                    pixel_fn=pixel_stub)
    B = 4
    ex = col(_samples(cfg, B))
    assert calls == [((B, 3, 48, 96), torch.uint8, 2)]
    di, dl = ex.driving_input, ex.driving_label
    assert di.camera_images.shape == (B, 1, cfg.tiles, 3, cfg.img_size, cfg.img_size)
    assert di.camera_intrinsics.shape == (B, 3, 3) and di.camera_extrinsics.shape == (B, 4, 4)
    assert float(di.camera_intrinsics[0, 0, 2]) == 48.0 and float(di.camera_extrinsics[0, 0, 3]) == -1.5
    assert ex.run_id.shape == (B, 1000) and bytes(ex.run_id[1, :6].tolist()) == b"run_1/"
    assert dl.waypoints.shape == (B, cfg.n_speed, 2) and dl.path.shape == (B, cfg.n_route, 2)
    assert list(di.prompt.placeholder_values[1]) == [cfg.target_point_id]
    assert sorted(di.prompt.placeholder_values[3]) == [cfg.first_added_id, cfg.first_added_id + 5]  # WAYPOINTS, ROUTE
    ids = di.prompt.phrase_ids
    assert ((ids == cfg.img_context_id).sum(1) == cfg.img_tokens).all()
    plan = plan_from_example(cfg, ex)
    assert plan.B == B and plan.S == ids.shape[1] + cfg.n_queries
    P = init_params(cfg, seed=3, lora_b_std=0.05, std=0.05)
    out, grads = O.loss_and_grads(P, cfg, ex)
    assert torch.isfinite(out["loss"]) and out["language_loss"] > 0
    assert all(torch.isfinite(g).all() for g in grads.values())
    # the inference prompt (question only) collates and plans too
    assert plan_from_example(cfg, ex, inference=True).L == di.prompt_inference.phrase_ids.shape[1]


def test_collate_host_half_in_dataloader_workers(tok):
    """Collate.host is the CPU half that runs in DataLoader workers (datamodule.py:275-284): picklable, uint8 frames
    stacked as camera_images, the same token ids / masks / labels as the in-process call."""
    from torch.utils.data import DataLoader
    from simlingo_amd.config import tiny_config
    cfg = tiny_config()
    col = C.Collate(tok, num_image_tokens_per_patch=cfg.img_tokens_per_tile, num_image_patches=cfg.tiles)
    samples = _samples(cfg, 8, seed=3)
    want = [col.host(samples[:4]), col.host(samples[4:])]
    dl = DataLoader(samples, batch_size=4, shuffle=False, num_workers=2, collate_fn=col.host)
    got = list(dl)
    assert len(got) == 2
    for g, w in zip(got, want):
        assert g.driving_input.camera_images.dtype == torch.uint8 and g.driving_input.camera_images.shape == (4, 3, 48, 96)
        assert torch.equal(g.driving_input.camera_images, w.driving_input.camera_images)
        for k in ("phrase_ids", "phrase_valid", "loss_masking"):
            assert torch.equal(getattr(g.driving_input.prompt, k), getattr(w.driving_input.prompt, k))
        assert torch.equal(g.driving_label.path, w.driving_label.path)


def test_synthetic_samples_full_geometry():
    """simlingo_amd.synthetic.synthetic_samples + synthetic_tokenizer (InternVL2-1B id layout): the collated prompt is
    exactly s_text + img_tokens long with n_loss LM-loss tokens and two <TARGET_POINT> placeholders, so the plan has
    the config-3 sequence (S = 798)."""
    from simlingo_amd.config import full_config
    from simlingo_amd.plan import plan_from_example
    from simlingo_amd.synthetic import synthetic_samples, synthetic_tokenizer
    cfg = full_config()
    tk = synthetic_tokenizer(cfg)
    col = C.Collate(tk, num_image_tokens_per_patch=cfg.img_tokens_per_tile, num_image_patches=cfg.tiles)
    ex = col.host(synthetic_samples(cfg, 3, seed=2))
    p = ex.driving_input.prompt
    assert p.phrase_ids.shape == (3, 256 + cfg.img_tokens) and bool(p.phrase_valid.all())
    assert (p.loss_masking.sum(1) == 16).all()
    assert ex.driving_input.camera_images.shape == (3, 3, 359, 1024)
    plan = plan_from_example(cfg, ex)
    assert plan.S == 798 and plan.loss_pos.shape[0] == 3 * 16 and plan.wp_coords.shape == (6, 2)
