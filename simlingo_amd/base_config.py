"""Geometry of the SimLingo-Base path (BASELINE.json configs[1]).

simlingo_base_training: LLaVAnextEncoderModel (models/encoder/llavanext.py:32-113) = the CLIP ViT-L/14-336
vision tower + 2-layer GELU projector of llava-hf/llava-v1.6-mistral-7b-hf, run by
LingoLlavaNextModel.forward_image (llavanext_model.py:45-178) on the anyres patches of one frame
(image_grid_pinpoints [[336, 672]] -> a 1 x 2 patch grid), hidden_states[-2] (vision_feature_layer -2,
CLS dropped), spatial_unpad + avg_pool2d(downsample_feature_grid_factor=2) + image_newline, then
Linear(4096 -> embed_dim) + temporal / camera encodings; speed (VectorInputAdaptor) and 2 target points
(WaypointInputAdaptor) tokens (driving.py:166-197); Llama CONFIGS['tiny'] (llama.py:46) over
[vision | speed | route | 20 route + 10 speed queries]; DrivingAdaptor heads with MSE (adaptors.py:96-232).
Constants of the hub checkpoints are [third-party; not verifiable offline] and match the transformers
defaults the oracle builds (CLIPVisionConfig / LlamaConfig).
"""
from __future__ import annotations

import dataclasses
from dataclasses import dataclass


@dataclass
class BaseConfig:
    # ---- CLIP ViT-L/14-336 ----
    img_size: int = 336
    patch: int = 14
    vit_dim: int = 1024
    vit_layers: int = 24            # tower depth; hidden_states[-2] uses the first vit_layers - 1
    vit_heads: int = 16
    vit_ffn: int = 4096
    vit_eps: float = 1e-5
    npatch_h: int = 1               # anyres grid for pinpoints [[336, 672]] (llavanext.py:63)
    npatch_w: int = 2
    # ---- projector + spatial merge ----
    proj_dim: int = 4096            # text hidden size of the LLaVA-NeXT checkpoint (linear_1 / linear_2)
    pool: int = 2                   # downsample_feature_grid_factor (simlingo_base_1.yaml:27)
    frame_h: int = 359              # image_sizes of the frame the processor sees: 1024 x 512 cropped to 359 rows
    frame_w: int = 1024             # (dataset_base.py:464-467, img_shift_augmentation True) -> 200 image tokens
    embed_dim: int = 512            # LLaVAnextEncoderConfig.embed_dim (config.py)
    # ---- Llama 'tiny' (llama.py:46) ----
    llm_dim: int = 512
    llm_layers: int = 12
    llm_heads: int = 8
    llm_ffn: int = 2048
    rope_theta: float = 1e4
    rms_eps: float = 1e-6
    # ---- input adaptors (driving.py:166-197) ----
    in_hidden: int = 256
    speed_min: float = 0.0          # NormZeroOne((0, 64/3.6)) (new_layer_norm_minmax False)
    speed_max: float = 64.0 / 3.6
    tp_min: float = -32.0           # NormZeroOne((-32, 32))
    tp_max: float = 32.0
    n_tp: int = 2                   # [target_point, next_target_point] (dataset_base.py:467-469)
    # ---- driving adaptor (adaptors.py:110-160) ----
    n_route: int = 20
    n_speed: int = 10
    speed_dims: int = 2
    head_mlp: int = 256
    # ---- optimisation (simlingo_base_1.yaml, train.py:189) ----
    lr: float = 3e-5
    vision_lr: float = 3e-5
    weight_decay: float = 0.1
    betas: tuple = (0.9, 0.999)
    eps: float = 1e-8
    pct_start: float = 0.05
    grad_clip: float = 1.0

    @property
    def vit_grid(self) -> int:
        return self.img_size // self.patch

    @property
    def vit_tokens(self) -> int:
        return self.vit_grid ** 2 + 1

    @property
    def vit_used(self) -> int:
        return self.vit_layers - 1

    @property
    def npatch(self) -> int:
        return self.npatch_h * self.npatch_w

    @property
    def patch_k(self) -> int:
        return 3 * self.patch * self.patch

    @property
    def patch_kpad(self) -> int:
        return (self.patch_k + 63) // 64 * 64

    def unpad(self) -> tuple[int, int, int, int]:
        """transformers unpad_image on the (npatch_h*g) x (npatch_w*g) grid -> (r0, hu, c0, wu)."""
        H, W = self.npatch_h * self.vit_grid, self.npatch_w * self.vit_grid
        oh, ow = self.frame_h, self.frame_w
        if ow / oh > W / H:
            new_h = int(round(oh * (W / ow), 7))
            pad = (H - new_h) // 2
            return pad, H - 2 * pad, 0, W
        new_w = int(round(ow * (H / oh), 7))
        pad = (W - new_w) // 2
        return 0, H, pad, W - 2 * pad

    @property
    def img_tokens(self) -> int:
        _, hu, _, wu = self.unpad()
        return (hu // self.pool) * (wu // self.pool + 1)

    @property
    def n_queries(self) -> int:
        return self.n_route + self.n_speed

    @property
    def seq(self) -> int:
        return self.img_tokens + 1 + self.n_tp + self.n_queries

    def replace(self, **kw) -> "BaseConfig":
        return dataclasses.replace(self, **kw)


def base_config(**kw) -> BaseConfig:
    return BaseConfig(**kw)


def base_tiny_config(**kw) -> BaseConfig:
    """Reduced geometry for parity tests (head_dim 64, every contiguous dim a multiple of 8)."""
    base = dict(img_size=112, patch=14, vit_dim=128, vit_layers=3, vit_heads=2, vit_ffn=256, proj_dim=192,
                frame_h=80, frame_w=256, embed_dim=128, llm_dim=128, llm_layers=2, llm_heads=2, llm_ffn=256,
                in_hidden=64, head_mlp=64)
    base.update(kw)
    return BaseConfig(**base)
