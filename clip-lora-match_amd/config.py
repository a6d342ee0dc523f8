"""Model shape descriptions for the CLIP+LoRA encode path.

Mirrors the shapes the reference reads from `config/clip_config.yaml:1-23` and
`config/lora_config.yaml:1-14` (model name, LoRA r/alpha/targets) and the
transformers `CLIPConfig` defaults it resolves to
(TF/models/clip/configuration_clip.py:47-64, 97-106).

Presets:
  * ``ViT-B/32``      -- openai/clip-vit-base-patch32 (BASELINE configs 0-2, 4)
  * ``ViT-L/14@336``  -- openai/clip-vit-large-patch14-336 (BASELINE config 3)
  * ``tiny``          -- a 2-layer toy used by fast parity tests
"""
from __future__ import annotations

from dataclasses import dataclass, field, replace
from typing import Tuple

# bit positions of LoRA targets, shared with include/clm.h (CLM_LORA_*)
LORA_TARGET_BITS = {"q_proj": 1, "k_proj": 2, "v_proj": 4, "out_proj": 8, "fc1": 16, "fc2": 32}

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)   # clip_config.yaml:11
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)    # clip_config.yaml:12


@dataclass(frozen=True)
class TowerConfig:
    hidden: int
    layers: int
    heads: int
    mlp: int

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


@dataclass(frozen=True)
class ModelConfig:
    name: str
    vision: TowerConfig
    text: TowerConfig
    patch: int
    image_size: int
    proj_dim: int
    vocab: int = 49408
    max_pos: int = 77
    channels: int = 3
    bos_token_id: int = 49406
    eos_token_id: int = 49407
    ln_eps: float = 1e-5
    lora_r: int = 8
    lora_alpha: float = 16.0
    lora_targets: Tuple[str, ...] = ("q_proj", "k_proj", "v_proj", "out_proj")
    mean: Tuple[float, float, float] = CLIP_MEAN
    std: Tuple[float, float, float] = CLIP_STD

    @property
    def grid(self) -> int:
        return self.image_size // self.patch

    @property
    def num_patches(self) -> int:
        return self.grid * self.grid

    @property
    def vision_seq(self) -> int:
        return self.num_patches + 1

    @property
    def lora_scaling(self) -> float:
        # PEFT LoRA: scaling = lora_alpha / r  (lora_adapter.py:36-37 -> 16/8 = 2.0)
        return self.lora_alpha / self.lora_r if self.lora_r > 0 else 0.0

    @property
    def lora_mask(self) -> int:
        m = 0
        for t in self.lora_targets:
            m |= LORA_TARGET_BITS[t]
        return m

    def with_lora(self, r: int, alpha: float, targets) -> "ModelConfig":
        return replace(self, lora_r=int(r), lora_alpha=float(alpha), lora_targets=tuple(targets))


PRESETS = {
    "ViT-B/32": ModelConfig(
        name="openai/clip-vit-base-patch32",
        vision=TowerConfig(hidden=768, layers=12, heads=12, mlp=3072),
        text=TowerConfig(hidden=512, layers=12, heads=8, mlp=2048),
        patch=32, image_size=224, proj_dim=512,
    ),
    "ViT-L/14@336": ModelConfig(
        name="openai/clip-vit-large-patch14-336",
        vision=TowerConfig(hidden=1024, layers=24, heads=16, mlp=4096),
        text=TowerConfig(hidden=768, layers=12, heads=12, mlp=3072),
        patch=14, image_size=336, proj_dim=768,
        lora_r=16, lora_alpha=32.0,
        lora_targets=("q_proj", "k_proj", "v_proj", "out_proj", "fc1", "fc2"),
    ),
    "tiny": ModelConfig(
        name="tiny",
        vision=TowerConfig(hidden=128, layers=2, heads=2, mlp=512),
        text=TowerConfig(hidden=128, layers=2, heads=2, mlp=512),
        patch=16, image_size=64, proj_dim=64, vocab=1000, max_pos=16,
        bos_token_id=998, eos_token_id=999,
    ),
}

# Hub names accepted by load_clip_model (clip_config.yaml:2)
NAME_TO_PRESET = {
    "openai/clip-vit-base-patch32": "ViT-B/32",
    "openai/clip-vit-large-patch14-336": "ViT-L/14@336",
    "tiny": "tiny",
}


def get_preset(name: str) -> ModelConfig:
    key = NAME_TO_PRESET.get(name, name)
    if key not in PRESETS:
        raise ValueError(f"unknown CLIP model '{name}' (known: {sorted(NAME_TO_PRESET)})")
    return PRESETS[key]
