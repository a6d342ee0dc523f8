"""Weights: deterministic synthetic CLIP/LoRA state dicts and on-disk loaders.

There is no network and no pretrained checkpoint in this environment, so the
encode path is exercised with a deterministic counter-hash generator
(splitmix64 over (seed, crc32(name), element index)). It does not depend on
any RNG library state, so numpy on any host produces bit-identical tensors.

Names follow the transformers CLIPModel state dict
(TF/models/clip/modeling_clip.py:138-218, 221-256, 280-384, 659-676) and the
PEFT adapter file format written by `PeftModel.save_pretrained`
(scripts/train_lora.py:247) and read by `PeftModel.from_pretrained`
(models/clip_model.py:78): ``base_model.model.<module path>.lora_{A,B}.weight``,
A: [r, in], B: [out, r].

PEFT initialises lora_B to zero, which would make LoRA a no-op and every
parity check vacuous; the synthetic adapter therefore has non-zero B.
"""
from __future__ import annotations

import json
import os
import zlib
from pathlib import Path
from typing import Dict, Iterator, Tuple

import numpy as np

from .config import ModelConfig

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix_u01(key: int, n: int) -> np.ndarray:
    """n uniforms in [0, 1) (24-bit resolution) from a 64-bit key."""
    i = np.arange(n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (i + np.uint64(key & 0xFFFFFFFFFFFFFFFF)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(40)).astype(np.float64) * (1.0 / 16777216.0)


def _uniform(seed: int, name: str, shape, lo: float, hi: float) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    key = (seed * 0x100000001B3 + zlib.crc32(name.encode())) * 0x9E3779B1
    u = _splitmix_u01(key, n)
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def _tower_layer_names(prefix: str, i: int, d: int, mlp: int) -> Iterator[Tuple[str, tuple]]:
    p = f"{prefix}.encoder.layers.{i}"
    for proj in ("k_proj", "v_proj", "q_proj", "out_proj"):
        yield f"{p}.self_attn.{proj}.weight", (d, d)
        yield f"{p}.self_attn.{proj}.bias", (d,)
    yield f"{p}.layer_norm1.weight", (d,)
    yield f"{p}.layer_norm1.bias", (d,)
    yield f"{p}.mlp.fc1.weight", (mlp, d)
    yield f"{p}.mlp.fc1.bias", (mlp,)
    yield f"{p}.mlp.fc2.weight", (d, mlp)
    yield f"{p}.mlp.fc2.bias", (d,)
    yield f"{p}.layer_norm2.weight", (d,)
    yield f"{p}.layer_norm2.bias", (d,)


def state_dict_shapes(cfg: ModelConfig) -> Dict[str, tuple]:
    """Every tensor of transformers.CLIPModel(cfg) that the encode path reads."""
    v, t = cfg.vision, cfg.text
    s: Dict[str, tuple] = {}
    s["text_model.embeddings.token_embedding.weight"] = (cfg.vocab, t.hidden)
    s["text_model.embeddings.position_embedding.weight"] = (cfg.max_pos, t.hidden)
    for i in range(t.layers):
        s.update(_tower_layer_names("text_model", i, t.hidden, t.mlp))
    s["text_model.final_layer_norm.weight"] = (t.hidden,)
    s["text_model.final_layer_norm.bias"] = (t.hidden,)
    s["vision_model.embeddings.class_embedding"] = (v.hidden,)
    s["vision_model.embeddings.patch_embedding.weight"] = (v.hidden, cfg.channels, cfg.patch, cfg.patch)
    s["vision_model.embeddings.position_embedding.weight"] = (cfg.vision_seq, v.hidden)
    s["vision_model.pre_layrnorm.weight"] = (v.hidden,)
    s["vision_model.pre_layrnorm.bias"] = (v.hidden,)
    for i in range(v.layers):
        s.update(_tower_layer_names("vision_model", i, v.hidden, v.mlp))
    s["vision_model.post_layernorm.weight"] = (v.hidden,)
    s["vision_model.post_layernorm.bias"] = (v.hidden,)
    s["visual_projection.weight"] = (cfg.proj_dim, v.hidden)
    s["text_projection.weight"] = (cfg.proj_dim, t.hidden)
    return s


def _init_range(name: str, shape: tuple) -> Tuple[float, float]:
    """Uniform range per tensor kind, chosen so activations keep CLIP-like scales
    and the pooled embeddings are not collinear."""
    if name.endswith("layer_norm1.weight") or name.endswith("layer_norm2.weight") \
            or name.endswith("layernorm.weight") or name.endswith("layrnorm.weight") \
            or name.endswith("final_layer_norm.weight"):
        return 0.8, 1.2
    if "norm" in name and name.endswith(".bias"):
        return -0.1, 0.1
    if name.endswith("token_embedding.weight"):
        return -0.05, 0.05
    if name.endswith("position_embedding.weight"):
        return -0.02, 0.02
    if name.endswith("class_embedding"):
        return -0.1, 0.1
    if name.endswith(".bias"):
        return -0.02, 0.02
    fan_in = int(np.prod(shape[1:]))
    a = 1.5 / np.sqrt(fan_in)
    return -a, a


def synthetic_state_dict(cfg: ModelConfig, seed: int = 0) -> Dict[str, np.ndarray]:
    out = {}
    for name, shape in state_dict_shapes(cfg).items():
        lo, hi = _init_range(name, shape)
        out[name] = _uniform(seed, name, shape, lo, hi)
    return out


def _target_module_paths(cfg: ModelConfig, targets) -> Iterator[Tuple[str, int, int]]:
    """(module path, in_features, out_features) of every Linear PEFT would wrap.

    PEFT matches `target_modules` by module-name suffix, so q/k/v/out_proj land in
    BOTH towers, all layers."""
    for prefix, tw in (("text_model", cfg.text), ("vision_model", cfg.vision)):
        for i in range(tw.layers):
            for tgt in targets:
                if tgt in ("q_proj", "k_proj", "v_proj", "out_proj"):
                    yield f"{prefix}.encoder.layers.{i}.self_attn.{tgt}", tw.hidden, tw.hidden
                elif tgt == "fc1":
                    yield f"{prefix}.encoder.layers.{i}.mlp.fc1", tw.hidden, tw.mlp
                elif tgt == "fc2":
                    yield f"{prefix}.encoder.layers.{i}.mlp.fc2", tw.mlp, tw.hidden


def lora_shapes(cfg: ModelConfig) -> Dict[str, tuple]:
    s = {}
    r = cfg.lora_r
    for path, fin, fout in _target_module_paths(cfg, cfg.lora_targets):
        s[f"base_model.model.{path}.lora_A.weight"] = (r, fin)
        s[f"base_model.model.{path}.lora_B.weight"] = (fout, r)
    return s


def synthetic_lora(cfg: ModelConfig, seed: int = 1, b_scale: float = 0.04) -> Dict[str, np.ndarray]:
    out = {}
    for name, shape in lora_shapes(cfg).items():
        if ".lora_A." in name:
            a = 1.0 / np.sqrt(shape[1])          # kaiming-uniform-like, as PEFT's A init
            out[name] = _uniform(seed, name, shape, -a, a)
        else:
            out[name] = _uniform(seed, name, shape, -b_scale, b_scale)   # non-zero B
    return out


def lora_param_count(cfg: ModelConfig) -> int:
    return int(sum(np.prod(s) for s in lora_shapes(cfg).values()))


# ---------------------------------------------------------------------------
# on-disk formats
# ---------------------------------------------------------------------------
def load_peft_adapter(path) -> Tuple[Dict[str, np.ndarray], dict]:
    """Read a PEFT adapter directory without peft: adapter_config.json +
    adapter_model.safetensors (or adapter_model.bin loaded weights_only)."""
    path = Path(path)
    cfg_file = path / "adapter_config.json"
    if not cfg_file.exists():
        raise FileNotFoundError(f"adapter_config.json not found in {path}")
    with open(cfg_file, "r", encoding="utf-8") as f:
        acfg = json.load(f)
    st = path / "adapter_model.safetensors"
    tensors: Dict[str, np.ndarray] = {}
    if st.exists():
        from safetensors.numpy import load_file
        raw = load_file(str(st))
        tensors = {k: v.astype(np.float32) for k, v in raw.items()}
    else:
        binf = path / "adapter_model.bin"
        if not binf.exists():
            raise FileNotFoundError(f"no adapter_model.safetensors/.bin in {path}")
        import torch
        raw = torch.load(str(binf), map_location="cpu", weights_only=True)
        tensors = {k: v.float().numpy() for k, v in raw.items()}
    # PEFT may keep the adapter name in the key ("...lora_A.default.weight")
    norm = {}
    for k, v in tensors.items():
        k2 = k.replace(".lora_A.default.weight", ".lora_A.weight").replace(
            ".lora_B.default.weight", ".lora_B.weight")
        if not k2.startswith("base_model.model."):
            k2 = "base_model.model." + k2
        norm[k2] = v
    return norm, acfg


def save_peft_adapter(path, tensors: Dict[str, np.ndarray], r: int, alpha: float, targets) -> None:
    """Write the PEFT on-disk adapter format (used by tests and tools)."""
    from safetensors.numpy import save_file
    path = Path(path)
    path.mkdir(parents=True, exist_ok=True)
    save_file({k: np.ascontiguousarray(v, dtype=np.float32) for k, v in tensors.items()},
              str(path / "adapter_model.safetensors"))
    with open(path / "adapter_config.json", "w", encoding="utf-8") as f:
        json.dump({"peft_type": "LORA", "r": int(r), "lora_alpha": float(alpha),
                   "lora_dropout": 0.1, "bias": "none", "target_modules": list(targets),
                   "task_type": "FEATURE_EXTRACTION"}, f)


def load_hf_checkpoint(path) -> Dict[str, np.ndarray]:
    """Read a local transformers CLIP checkpoint directory (model.safetensors or
    pytorch_model.bin via weights_only) into float32 numpy arrays."""
    path = Path(path)
    st = path / "model.safetensors"
    if st.exists():
        from safetensors.numpy import load_file
        return {k: v.astype(np.float32) for k, v in load_file(str(st)).items()}
    binf = path / "pytorch_model.bin"
    if binf.exists():
        import torch
        raw = torch.load(str(binf), map_location="cpu", weights_only=True)
        return {k: v.float().numpy() for k, v in raw.items()}
    raise FileNotFoundError(f"no model.safetensors / pytorch_model.bin in {path}")


def default_weight_cache_dir() -> str:
    return os.environ.get("CLM_WEIGHT_CACHE", "")
