"""Drop-in for the reference's models/clip_model.py (same names, arguments,
return types and error behaviour), running on the gfx950 HIP kernels.

  _load_clip_config   models/clip_model.py:15-20   FileNotFoundError if missing
  _get_device         models/clip_model.py:23-28
  _get_dtype          models/clip_model.py:31-34
  load_clip_model     models/clip_model.py:37-82   -> (model, processor, device)
  encode_image        models/clip_model.py:89-118  -> (D,) float32 CPU, unit norm
  encode_text         models/clip_model.py:121-150 -> (D,) float32 CPU, unit norm

Differences forced by the environment (no network, no peft, no CPU path):
  * CLIPModel.from_pretrained(name) fetches from the Hub, which is unreachable here, so the
    base weights come from a local transformers checkpoint directory: `model.weights_dir`
    in the YAML, the `weights_dir` argument or $CLM_WEIGHTS_DIR. The value "synthetic"
    selects the deterministic synthetic weights of weights.synthetic_state_dict (tests,
    benchmarks); with none of these set the load fails with OSError, as from_pretrained
    does offline -- never a silent substitute.
  * PeftModel.from_pretrained(dir) reads the PEFT on-disk adapter format directly
    (weights.load_peft_adapter); lora_weights_path="synthetic" attaches the deterministic
    non-zero synthetic adapter. A missing / unset LoRA path prints the reference's warning
    and continues without LoRA (models/clip_model.py:70-75); strict_lora=True (or
    $CLM_STRICT_LORA=1) raises instead, as the src/models/clip_model.py:54-59 variant does.
  * device "cpu" in the YAML (the shipped config) still runs on the GPU: this
    package has no CPU compute path.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Optional, Tuple, Union

import numpy as np
import torch
import yaml

from . import weights as W
from .config import get_preset
from .engine import ClipLoraModel
from .processor import ClipProcessor

ImagePath = Union[str, Path]


def _load_clip_config(config_path: Union[str, Path]) -> dict:
    path = Path(config_path)
    if not path.exists():
        raise FileNotFoundError(f"CLIP config file not found: {path}")
    with open(path, "r", encoding="utf-8") as f:
        return yaml.safe_load(f) or {}


def _get_device(device_str: Optional[str] = None) -> torch.device:
    if not torch.cuda.is_available():
        raise RuntimeError("clip_lora_match_amd runs on MI355X only; no HIP device is visible")
    if device_str is None or str(device_str).startswith("cpu"):
        return torch.device("cuda", torch.cuda.current_device())
    d = torch.device(device_str)
    return torch.device("cuda", d.index if d.index is not None else torch.cuda.current_device())


def _get_dtype(dtype_str: str, device: torch.device) -> str:
    """Compute dtype of the MFMA path. float16 -> fp16 operands; bfloat16 -> bf16;
    float32 (the reference's CPU dtype) -> fp16, the higher-precision 16-bit
    operand type (same MFMA rate), with fp32 accumulate / LayerNorm / softmax /
    residual stream everywhere. $CLM_COMPUTE_DTYPE overrides."""
    env = os.environ.get("CLM_COMPUTE_DTYPE")
    s = (env or dtype_str or "float32").lower()
    if s in ("bfloat16", "bf16"):
        return "bfloat16"
    return "float16"


def _base_weights(model_name: str, cfg, weights_dir, model_cfg: dict, seed: int):
    src = weights_dir or model_cfg.get("weights_dir") or os.environ.get("CLM_WEIGHTS_DIR")
    if src is None:
        raise OSError(
            f"no local checkpoint for '{model_name}': CLIPModel.from_pretrained needs the Hub, which is "
            "unreachable here. Point model.weights_dir (YAML), weights_dir= or $CLM_WEIGHTS_DIR at a "
            "transformers checkpoint directory, or set it to 'synthetic' for the deterministic synthetic weights")
    if str(src) == "synthetic":
        print(f"[clip_model] using deterministic synthetic weights for '{model_name}' (seed={seed})")
        return W.synthetic_state_dict(cfg, seed)
    if not Path(src).exists():
        raise FileNotFoundError(f"CLIP checkpoint directory not found: {src}")
    return W.load_hf_checkpoint(src)


def load_clip_model(
    config_path: Union[str, Path] = "config/clip_config.yaml",
    use_lora: bool = False,
    lora_weights_path: Optional[Union[str, Path]] = None,
    *,
    weights_dir: Optional[Union[str, Path]] = None,
    max_batch: int = 256,
    lora_mode: str = "merged",
    compute_dtype: Optional[str] = None,
    seed: int = 0,
    strict_lora: Optional[bool] = None,
) -> Tuple[ClipLoraModel, ClipProcessor, torch.device]:
    """Load CLIP (+ optional LoRA) onto the GPU; returns (model, processor, device)."""
    config = _load_clip_config(config_path)
    model_cfg = config.get("model", {}) or {}
    model_name = model_cfg.get("name", "openai/clip-vit-base-patch32")
    device = _get_device(model_cfg.get("device"))
    dtype = compute_dtype or _get_dtype(model_cfg.get("dtype", "float16"), device)
    cfg = get_preset(model_name)
    if strict_lora is None:
        strict_lora = os.environ.get("CLM_STRICT_LORA", "0") not in ("", "0")

    print(f"[clip_model] Loading CLIP model '{model_name}' on device: {device} (dtype={dtype})")
    sd = _base_weights(model_name, cfg, weights_dir, model_cfg, seed)

    lora = None
    if use_lora:
        paths_cfg = config.get("paths", {}) or {}
        if lora_weights_path is None:
            lora_weights_path = paths_cfg.get("lora_weights_dir")
        if lora_weights_path is None:
            if strict_lora:
                raise ValueError("use_lora=True but lora_weights_path is not set")
            print("[clip_model] use_lora=True tetapi lora_weights_path tidak diset, lanjut tanpa LoRA.")
        elif str(lora_weights_path) == "synthetic":
            lora = W.synthetic_lora(cfg, seed + 1)
            print("[clip_model] Attaching deterministic synthetic LoRA adapter")
        else:
            lora_path = Path(lora_weights_path)
            if not lora_path.exists():
                if strict_lora:
                    raise FileNotFoundError(f"LoRA weights not found: {lora_path}")
                print(f"[clip_model] LoRA weights tidak ditemukan di: {lora_path}, lanjut tanpa LoRA.")
            else:
                print(f"[clip_model] Loading LoRA weights from: {lora_path}")
                lora, acfg = W.load_peft_adapter(lora_path)
                targets = acfg.get("target_modules") or ["q_proj", "v_proj"]
                if isinstance(targets, str):
                    targets = [targets]
                cfg = cfg.with_lora(acfg.get("r", 8), acfg.get("lora_alpha", 16), targets)
    if lora is None:
        cfg = cfg.with_lora(0, 0.0, ())

    model = ClipLoraModel(cfg, device=device, compute_dtype=dtype, lora_mode=lora_mode, max_batch=max_batch)
    model.load_tensors(sd)
    if lora is not None:
        model.load_tensors(lora)
    model.finalize()
    processor = ClipProcessor(cfg, tokenizer_dir=model_cfg.get("tokenizer_dir"))
    model.eval()
    return model, processor, device


def _encode_images(images, model: ClipLoraModel, processor: ClipProcessor, normalize: bool) -> torch.Tensor:
    """host decode -> GPU resize + centre crop (clm_resize_crop) -> GPU encode (uint8 path:
    rescale / normalise fused in patchify)."""
    return model.encode_pixels(processor.images_u8(images, model.device), normalize=normalize)


def encode_image(
    image_path: ImagePath,
    model: ClipLoraModel,
    processor: ClipProcessor,
    device: torch.device,
) -> torch.Tensor:
    """One image -> unit-norm (D,) float32 CPU embedding (models/clip_model.py:89-118)."""
    image_path = Path(image_path)
    if not image_path.exists():
        raise FileNotFoundError(f"Image not found: {image_path}")
    feats = _encode_images([image_path], model, processor, normalize=True)
    return feats.squeeze(0).to("cpu", torch.float32)


def encode_text(
    text,
    model: ClipLoraModel,
    processor: ClipProcessor,
    device: torch.device,
) -> torch.Tensor:
    """One caption (str, or its CLIP token ids) -> unit-norm (D,) float32 CPU embedding
    (models/clip_model.py:121-150)."""
    ids = processor.token_ids(text if not isinstance(text, str) else [text])
    feats = model.encode_ids(ids.to(model.device), normalize=True)
    return feats.squeeze(0).to("cpu", torch.float32)


__all__ = ["load_clip_model", "encode_image", "encode_text", "_load_clip_config", "_get_device", "_get_dtype"]
