"""clip_lora_match_amd -- MI355X-native CLIP+LoRA encode -> L2-normalise -> cosine top-k.

Drop-in for the reference's `models/clip_model.py`, `models/lora_adapter.py` and
`src/embedding/*` API; compute runs in hand-written gfx950 HIP kernels behind the
C-ABI library `libclm.so` (include/clm.h).
"""
from .config import ModelConfig, TowerConfig, PRESETS, get_preset  # noqa: F401

__all__ = ["ModelConfig", "TowerConfig", "PRESETS", "get_preset"]
