"""Drop-in for models/lora_adapter.py without peft.

  _load_lora_config    lora_adapter.py:13-18  FileNotFoundError if missing
  create_lora_config   lora_adapter.py:21-43  defaults r=8, alpha=16, dropout=0.1,
                                              bias="none", targets ["q_proj","v_proj"]
  attach_lora_to_clip  lora_adapter.py:46-56  wraps the model with adapters on every
                                              Linear whose name ends in a target
                                              (PEFT suffix matching: both towers)
PEFT initialises lora_B = 0, so a freshly attached adapter is an exact no-op;
init="synthetic" attaches the deterministic non-zero adapter instead. The adapters
are attached to the given model's own weights, in place (clm_set_lora on its
context), as get_peft_model does.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from pathlib import Path
from typing import List, Union

import numpy as np
import yaml

from . import weights as W
from .engine import ClipLoraModel


@dataclass
class LoraConfig:
    r: int = 8
    lora_alpha: float = 16
    lora_dropout: float = 0.1
    bias: str = "none"
    target_modules: List[str] = field(default_factory=lambda: ["q_proj", "v_proj"])
    task_type: str = "FEATURE_EXTRACTION"


def _load_lora_config(config_path: Union[str, Path]) -> dict:
    path = Path(config_path)
    if not path.exists():
        raise FileNotFoundError(f"LoRA config file not found: {path}")
    with open(path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f) or {}


def create_lora_config(config_path: Union[str, Path] = "config/lora_config.yaml") -> LoraConfig:
    cfg = _load_lora_config(config_path)
    lora_cfg = cfg.get("lora", {}) or {}
    model_cfg = cfg.get("model", {}) or {}
    return LoraConfig(
        r=lora_cfg.get("r", 8),
        lora_alpha=lora_cfg.get("alpha", 16),
        lora_dropout=lora_cfg.get("dropout", 0.1),
        bias=lora_cfg.get("bias", "none"),
        target_modules=list(model_cfg.get("target_modules", ["q_proj", "v_proj"])),
        task_type=lora_cfg.get("task_type", "FEATURE_EXTRACTION"),
    )


def attach_lora_to_clip(model: ClipLoraModel, lora_config: LoraConfig, init: str = "peft",
                        seed: int = 1) -> ClipLoraModel:
    """Wrap `model` -- its own loaded weights -- with adapters of `lora_config` on every Linear
    whose name ends in a target (lora_adapter.py:46-56; PEFT matches by suffix: both towers).
    Like get_peft_model the model is modified in place and returned.
    init="peft": lora_B = 0 (PEFT's initialisation: an exact no-op until trained weights are
    loaded); init="synthetic": the deterministic non-zero adapter."""
    cfg = model.cfg.with_lora(lora_config.r, lora_config.lora_alpha, lora_config.target_modules)
    if init == "synthetic":
        lora = W.synthetic_lora(cfg, seed)
    elif init == "peft":
        lora = {k: (v * 0.0 if ".lora_B." in k else v) for k, v in W.synthetic_lora(cfg, seed).items()}
    else:
        raise ValueError("init must be 'peft' or 'synthetic'")
    model.attach_lora(cfg.lora_r, cfg.lora_alpha, cfg.lora_targets, lora)
    trainable = W.lora_param_count(cfg)
    total = sum(int(np.prod(s)) for s in W.state_dict_shapes(cfg).values()) + trainable
    print(f"trainable params: {trainable:,d} || all params: {total:,d} || "
          f"trainable%: {100.0 * trainable / total:.4f}")
    return model
