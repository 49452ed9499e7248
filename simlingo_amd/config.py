"""Model geometry of the SimLingo VLA hot path.

Mirrors the reference's Hydra surface (simlingo_training/config.py:32-104; experiment
simlingo_seed1.yaml) plus the InternVL2-1B architecture constants that the reference pulls from the
hub config at run time (SURVEY.md §8 notation; InternViT-300M-448px + Qwen2-0.5B).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass, field


@dataclass
class VLAConfig:
    # ---- InternViT (remote InternVisionModel) ----
    img_size: int = 448
    patch: int = 14
    vit_dim: int = 1024
    vit_layers: int = 24
    vit_heads: int = 16
    vit_ffn: int = 4096
    vit_eps: float = 1e-6
    ls_init: float = 0.1
    tiles: int = 2                      # NUM_IMAGE_PATCHES (datamodule.py:110)
    # ---- mlp1 projector (downsample_ratio 0.5 -> pixel_shuffle) ----
    proj_eps: float = 1e-5
    # ---- Qwen2-0.5B (InternVL2-1B language half) ----
    llm_dim: int = 896
    llm_layers: int = 24
    llm_heads: int = 14
    llm_kv_heads: int = 2
    llm_ffn: int = 4864
    vocab: int = 151655
    rope_theta: float = 1e6
    rms_eps: float = 1e-6
    # ---- LoRA (llm.py:106-119; simlingo_seed1.yaml:21-24) ----
    lora: bool = True
    lora_r: int = 32
    lora_alpha: int = 64
    lora_dropout: float = 0.1
    # ---- vision_model.freeze (encoder/vlm.py:35-44): InternViT frozen, mlp1 still trained ----
    vit_freeze: bool = False
    # ---- driving adaptor (adaptors.py:96-136), wp_encoder (driving.py:91-96) ----
    n_route: int = 20
    n_speed: int = 10
    speed_dims: int = 2                 # speed_wps_mode '2d'
    head_mlp: int = 256
    wp_hidden: int = 256
    wp_hidden2: int = 512
    # ---- special token ids (InternVL2-1B tokenizer + SimLingo additions, datamodule.py:130-136) ----
    img_start_id: int = 151646
    img_end_id: int = 151647
    img_context_id: int = 151648
    first_added_id: int = 151655        # '<WAYPOINTS>' = tokenizer.additional_special_tokens_ids[0]
    target_point_id: int = 151662       # '<TARGET_POINT>'
    pad_id: int = 151643                # <|endoftext|>
    eos_id: int = 151645                # tokenizer.eos_token_id = <|im_end|> (driving.py:141) [third-party]
    # ---- optimisation (config.py:75-104, train.py:206) ----
    lr: float = 3e-5
    weight_decay: float = 0.1
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    pct_start: float = 0.05
    grad_clip: float = 0.3

    @property
    def vit_tokens(self) -> int:
        g = self.img_size // self.patch
        return g * g + 1

    @property
    def vit_grid(self) -> int:
        return self.img_size // self.patch

    @property
    def img_tokens_per_tile(self) -> int:
        return (self.vit_grid // 2) ** 2

    @property
    def img_tokens(self) -> int:
        return self.img_tokens_per_tile * self.tiles

    @property
    def n_queries(self) -> int:
        return self.n_route + self.n_speed

    @property
    def patch_k(self) -> int:
        return 3 * self.patch * self.patch

    @property
    def patch_kpad(self) -> int:
        return (self.patch_k + 63) // 64 * 64

    @property
    def lora_scale(self) -> float:
        return self.lora_alpha / self.lora_r

    def replace(self, **kw) -> "VLAConfig":
        return dataclasses.replace(self, **kw)


def full_config(**kw) -> VLAConfig:
    """InternVL2-1B geometry (BASELINE.json configs[2..4])."""
    return VLAConfig(**kw)


def tiny_config(**kw) -> VLAConfig:
    """Reduced geometry for parity tests: head_dim stays 64, every contiguous dim a multiple of 8."""
    base = dict(img_size=56, patch=14, vit_dim=128, vit_layers=2, vit_heads=2, vit_ffn=256,
                llm_dim=128, llm_layers=2, llm_heads=2, llm_kv_heads=1, llm_ffn=256, vocab=256,
                img_start_id=250, img_end_id=251, img_context_id=252, first_added_id=256,
                target_point_id=263, pad_id=249, eos_id=248, lora_dropout=0.0)
    base.update(kw)
    return VLAConfig(**base)
