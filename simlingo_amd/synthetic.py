"""Seeded synthetic batches of the reference's shape (SURVEY.md §8d "Synthetic inputs").

There is no dataset or tokenizer offline; token ids are drawn around the fixed InternVL2 prompt
skeleton: text, <img>, img_tokens x <IMG_CONTEXT>, </img>, text with two consecutive <TARGET_POINT>
placeholders (coords N(0, 10) m, shape [2, 2]), text. The tokenizer is left-padded
(datamodule.py:138), so padded samples carry invalid tokens at the front.
"""
from __future__ import annotations

import numpy as np
import torch

from .config import VLAConfig
from .types import DrivingExample, DrivingInput, DrivingLabel, LanguageLabel

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def make_batch(cfg: VLAConfig, B: int, s_text: int, n_loss: int, seed: int = 0, pad: list[int] | None = None,
               device: str | torch.device = "cpu") -> DrivingExample:
    """B samples; each language sequence has L = s_text + img_tokens positions; the last `n_loss`
    tokens of every sample take part in the LM loss; pad[b] leading positions of sample b are padding."""
    rng = np.random.default_rng(seed)
    g = torch.Generator().manual_seed(seed)
    nimg = cfg.img_tokens
    L = s_text + nimg
    pad = pad or [0] * B
    text_hi = min(cfg.pad_id, cfg.vocab)  # ordinary text ids stay below the special tokens
    ids = np.zeros((B, L), dtype=np.int64)
    valid = np.ones((B, L), dtype=bool)
    loss_mask = np.zeros((B, L), dtype=bool)
    placeholders = []
    for b in range(B):
        p = pad[b]
        seq = list(rng.integers(0, text_hi, size=4))
        seq += [cfg.img_start_id] + [cfg.img_context_id] * nimg + [cfg.img_end_id]
        n_rest = L - p - len(seq)
        assert n_rest >= 8, "s_text too small for the prompt skeleton"
        tail = list(rng.integers(0, text_hi, size=n_rest))
        tp = max(0, min(3, n_rest - n_loss - 3))  # keep the placeholders out of the loss span
        tail[tp] = cfg.target_point_id
        tail[tp + 1] = cfg.target_point_id
        seq += tail
        ids[b, :p] = cfg.pad_id
        valid[b, :p] = False
        ids[b, p:] = np.asarray(seq)
        nl = min(n_loss, L - p - 1)
        loss_mask[b, L - nl:] = True
        placeholders.append({cfg.target_point_id: rng.normal(0.0, 10.0, size=(2, 2)).astype(np.float32)})
    prompt = LanguageLabel(
        phrase_ids=torch.from_numpy(ids), phrase_valid=torch.from_numpy(valid),
        phrase_mask=torch.from_numpy(valid.copy()), placeholder_values=placeholders,
        language_string=[""] * B, loss_masking=torch.from_numpy(loss_mask))
    # pixel tiles directly in the ImageNet-normalised distribution of uint8 uniform frames
    H = cfg.img_size
    u = torch.rand((B, 1, cfg.tiles, 3, H, H), generator=g)
    mean = torch.tensor(IMAGENET_MEAN).view(1, 1, 1, 3, 1, 1)
    std = torch.tensor(IMAGENET_STD).view(1, 1, 1, 3, 1, 1)
    pix = ((u - mean) / std).float()
    route = torch.cumsum(torch.tensor([1.0, 0.0]) + 0.1 * torch.randn((B, cfg.n_route, 2), generator=g), 1)
    speed = torch.cumsum(torch.tensor([0.8, 0.0]) + 0.3 * torch.randn((B, cfg.n_speed, cfg.speed_dims), generator=g), 1)
    di = DrivingInput(
        camera_images=pix.to(device), image_sizes=torch.tensor([[H * cfg.tiles, H]] * B),
        camera_intrinsics=torch.eye(3).repeat(B, 1, 1), camera_extrinsics=torch.eye(4).repeat(B, 1, 1),
        vehicle_speed=torch.zeros(B, 1), target_point=torch.zeros(B, 2), prompt=prompt, prompt_inference=prompt)
    dl = DrivingLabel(waypoints=speed.float().to(device), path=route.float().to(device), answer=None,
                      image_ff_org=torch.zeros(B, 2))
    return DrivingExample(driving_input=di, driving_label=dl, run_id=[f"synthetic-{seed}-{b}" for b in range(B)])


# ---- synthetic per-sample dataset outputs for the drop-in collate path (bench `dropin` key, config-1 test) --------
_ROLE_WORDS = ("user", "assistant", "system")


def synthetic_tokenizer(cfg: VLAConfig):
    """A word-level HF tokenizer with the InternVL2-1B id layout of `cfg` (the Qwen2 tokenizer is hub-only): ordinary
    words below pad_id, <|endoftext|> = pad, <|im_start|>, <|im_end|> = eos, <img>, </img>, <IMG_CONTEXT> at their
    ids, the SimLingo placeholders from first_added_id (datamodule.py:130-137), left padding (datamodule.py:138).
    Whitespace splits words, so one word is one token and prompt lengths are exact."""
    from tokenizers import Tokenizer, models, pre_tokenizers
    from transformers import PreTrainedTokenizerFast

    from .collate import PLACEHOLDER_TOKENS
    if not (cfg.img_start_id == cfg.pad_id + 3 and cfg.eos_id == cfg.pad_id + 2 and cfg.img_context_id == cfg.pad_id + 5
            and cfg.first_added_id == cfg.pad_id + 12):
        raise ValueError("synthetic_tokenizer follows the InternVL2-1B special-token layout (full_config)")
    vocab = {w: i for i, w in enumerate(_ROLE_WORDS)}
    for i in range(len(vocab), cfg.pad_id):
        vocab[f"w{i}"] = i
    specials = ["<|endoftext|>", "<|im_start|>", "<|im_end|>", "<img>", "</img>", "<IMG_CONTEXT>"]
    specials += [f"<spare{j}>" for j in range(cfg.first_added_id - cfg.pad_id - len(specials))]
    for j, t in enumerate(specials):
        vocab[t] = cfg.pad_id + j
    tk = Tokenizer(models.WordLevel(vocab=vocab, unk_token="<|endoftext|>"))
    tk.pre_tokenizer = pre_tokenizers.WhitespaceSplit()
    tok = PreTrainedTokenizerFast(tokenizer_object=tk, pad_token="<|endoftext|>", unk_token="<|endoftext|>",
                                  eos_token="<|im_end|>", additional_special_tokens=specials[1:])
    tok.add_special_tokens({"additional_special_tokens": specials[1:] + PLACEHOLDER_TOKENS})
    tok.padding_side = "left"
    assert tok.convert_tokens_to_ids("<TARGET_POINT>") == cfg.target_point_id
    assert tok.convert_tokens_to_ids("<IMG_CONTEXT>") == cfg.img_context_id
    return tok


def synthetic_samples(cfg: VLAConfig, B: int, s_text: int = 256, n_loss: int = 16, seed: int = 0,
                      frame_hw=(512, 1024)):
    """B per-sample `collate.DatasetOutput`s of the reference's shape: a 1024 x 512 RGB frame with the dataset's bottom
    crop applied (dataset_base.py:464-467 -> 359 rows, 2 tiles of 448^2), a [user, assistant] conversation whose
    chat-template token count is exactly s_text + img_tokens (so S_llm = s_text + img_tokens + n_queries, as in
    make_batch) with n_loss LM-loss tokens (the assistant span) and two <TARGET_POINT> placeholders, and the
    waypoint / path labels. Words come from synthetic_tokenizer's vocabulary."""
    from .collate import DatasetOutput
    from .frames import bottom_crop_rows
    rng = np.random.default_rng(seed)
    H0, W0 = frame_hw
    H = bottom_crop_rows(H0)
    n_ans = n_loss - 3                       # <|im_start|> assistant {answer} <|im_end|>: the assistant span
    n_q = s_text - 8 - n_ans                 # everything else but the image block and the role / separator tokens
    assert n_ans >= 1 and n_q >= 4, "s_text / n_loss too small for the chat template"
    words = lambda n: " ".join(f"w{int(i)}" for i in rng.integers(len(_ROLE_WORDS), cfg.pad_id, size=n))
    out = []
    for _ in range(B):
        q = words(2) + " <TARGET_POINT> <TARGET_POINT> " + words(n_q - 4)
        a = words(n_ans)
        conv = [{"role": "user", "content": [{"type": "text", "text": q}]},
                {"role": "assistant", "content": [{"type": "text", "text": a}]}]
        out.append(DatasetOutput(
            image_ff=rng.integers(0, 256, size=(1, 3, H, W0), dtype=np.uint8), image_ff_org_size=(H0, W0),
            conversation=conv, answer=[conv[1]],
            placeholder_values={"<TARGET_POINT>": rng.normal(0.0, 10.0, size=(2, 2)).astype(np.float32)},
            waypoints=np.cumsum(rng.normal((0.8, 0.0), 0.3, size=(cfg.n_speed, cfg.speed_dims)), 0).astype(np.float32),
            path=np.cumsum(rng.normal((1.0, 0.0), 0.1, size=(cfg.n_route, 2)), 0).astype(np.float32),
            speed=np.float32(rng.uniform(0, 10)), target_points=rng.normal(0, 10, size=(2,)).astype(np.float32),
            measurement_path=f"synthetic/route{int(rng.integers(1000))}/measurements/0000.json.gz"))
    return out
