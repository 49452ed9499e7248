"""Hydra `_target_` stand-ins for the reference's encoder / language-model classes.

The reference instantiates these from config.py (VLMEncoderConfig._target_ :46, LanguageModelConfig
._target_ :71) inside DrivingModel.__init__ (driving.py:62-74). On the MI355X path the arithmetic
of both lives in VLAEngine, so these classes only carry (and validate) the same config keys.
"""
from __future__ import annotations

from torch import nn


class VLMEncoderModel(nn.Module):
    """simlingo_training/models/encoder/vlm.py:6-44 signature: (cfg_data_module, processor, cache_dir, **cfg)."""

    def __init__(self, cfg_data_module=None, processor=None, cache_dir=None, **cfg):
        super().__init__()
        for key, value in cfg.items():
            setattr(self, key, value)
        self.variant = cfg.get("variant", "OpenGVLab/InternVL2-1B")
        self.embed_dim = cfg.get("embed_dim", 512)
        self.freeze = cfg.get("freeze", False)
        if "internvl2" not in self.variant.lower() and self.variant != "tiny":
            raise ValueError(f"Unknown variant {self.variant}")


class LLM(nn.Module):
    """simlingo_training/models/language_model/llm.py:49-123 signature: (**cfg)."""

    def __init__(self, **cfg):
        super().__init__()
        for key, value in cfg.items():
            setattr(self, key, value)
        self.variant = cfg.get("variant", "OpenGVLab/InternVL2-1B")
        if "internvl" not in self.variant.lower() and self.variant != "tiny":
            raise ValueError(f"Carefull: Variant {self.variant} not tested.")
        self.lora = cfg.get("lora", True)
        self.lora_alpha = cfg.get("lora_alpha", 64)
        self.lora_r = cfg.get("lora_r", 32)
        self.lora_dropout = cfg.get("lora_dropout", 0.1)
