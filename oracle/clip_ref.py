"""ORACLE -- test infrastructure only. Never imported by the product path.

CPU fp32 (numpy) restatement of the reference's encode path so the HIP kernels
can be checked on identical inputs. Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.

What it restates (file:line into /root/reference unless prefixed TF/ =
/usr/local/lib/python3.10/dist-packages/transformers/):
  * image preprocessing for 224^2 (or image_size^2) uint8 input:
    CLIPImageProcessor resize/crop are identities, leaving
    `x * (1/255)` then `(x - mean) / std` (config/clip_config.yaml:7-13,
    TF/models/clip/image_processing_clip.py:23-39)                   -> preprocess_u8
  * CLIPVisionEmbeddings.forward  TF/models/clip/modeling_clip.py:202-218
  * CLIPTextEmbeddings.forward    TF/models/clip/modeling_clip.py:232-256
  * CLIPAttention + eager_attention_forward  modeling_clip.py:259-335
  * CLIPMLP + QuickGELU  modeling_clip.py:346-350, TF/activations.py:117-123
  * CLIPEncoderLayer     modeling_clip.py:362-384
  * CLIPTextModel.forward pooled EOS  modeling_clip.py:541-582
  * CLIPVisionModel.forward pooled CLS  modeling_clip.py:641-651
  * get_image_features / get_text_features projections  modeling_clip.py:712-713, 750-751
  * PEFT LoRA Linear at eval: y = x W^T + b + (alpha/r) * (x A^T) B^T
    (dropout is identity in eval; wired at models/clip_model.py:78,
    configured at models/lora_adapter.py:33-41)
  * L2 normalise  models/clip_model.py:116,148 (encode_image/encode_text)

Parity status: pinned against goldens produced by transformers 5.15.0
CLIPModel (the reference's own arithmetic) with the same synthetic weights --
see tests/golden/make_golden.py and tests/test_oracle.py.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

Array = np.ndarray


def preprocess_u8(images_hwc: Array, mean, std) -> Array:
    """uint8 [B,H,W,3] -> float32 [B,3,H,W] exactly as CLIPImageProcessor for
    inputs already at image_size^2 (rescale by 1/255, then normalise)."""
    # TF/image_transforms.py rescale: float64 multiply, downcast to float32;
    # normalize: (x - mean) / std in float32
    x = (images_hwc.astype(np.float64) * (1.0 / 255.0)).astype(np.float32)
    x = (x - np.asarray(mean, np.float32)) / np.asarray(std, np.float32)
    return np.ascontiguousarray(x.transpose(0, 3, 1, 2))


def layer_norm(x: Array, g: Array, b: Array, eps: float) -> Array:
    mu = x.mean(-1, keepdims=True, dtype=np.float32)
    var = ((x - mu) ** 2).mean(-1, keepdims=True, dtype=np.float32)
    return ((x - mu) / np.sqrt(var + np.float32(eps))) * g + b


def quick_gelu(x: Array) -> Array:
    # TF/activations.py:123  x * sigmoid(1.702 * x)
    return x * (1.0 / (1.0 + np.exp(-np.float32(1.702) * x)))


class _Linear:
    """nn.Linear with an optional PEFT LoRA side branch (unmerged, as PEFT runs)."""

    def __init__(self, W: Dict[str, Array], path: str, lora: Optional[Dict[str, Array]], scaling: float):
        self.w = W[path + ".weight"]
        self.b = W.get(path + ".bias")
        self.a = self.bb = None
        if lora is not None:
            ka = f"base_model.model.{path}.lora_A.weight"
            if ka in lora:
                self.a = lora[ka]
                self.bb = lora[f"base_model.model.{path}.lora_B.weight"]
        self.s = np.float32(scaling)

    def __call__(self, x: Array) -> Array:
        y = x @ self.w.T
        if self.b is not None:
            y = y + self.b
        if self.a is not None:
            y = y + self.s * ((x @ self.a.T) @ self.bb.T)
        return y


def _encoder(W, lora, scaling, prefix: str, h: Array, layers: int, heads: int, eps: float,
             causal: bool) -> Array:
    B, T, d = h.shape
    hd = d // heads
    scale = np.float32(hd ** -0.5)
    mask = None
    if causal:
        mask = np.triu(np.full((T, T), -np.inf, np.float32), 1)
    for i in range(layers):
        p = f"{prefix}.encoder.layers.{i}"
        res = h
        x = layer_norm(h, W[p + ".layer_norm1.weight"], W[p + ".layer_norm1.bias"], eps)
        q = _Linear(W, p + ".self_attn.q_proj", lora, scaling)(x)
        k = _Linear(W, p + ".self_attn.k_proj", lora, scaling)(x)
        v = _Linear(W, p + ".self_attn.v_proj", lora, scaling)(x)
        q = q.reshape(B, T, heads, hd).transpose(0, 2, 1, 3)
        k = k.reshape(B, T, heads, hd).transpose(0, 2, 1, 3)
        v = v.reshape(B, T, heads, hd).transpose(0, 2, 1, 3)
        s = (q @ k.transpose(0, 1, 3, 2)) * scale
        if mask is not None:
            s = s + mask
        s = s - s.max(-1, keepdims=True)
        e = np.exp(s)
        pr = e / e.sum(-1, keepdims=True)
        o = (pr @ v).transpose(0, 2, 1, 3).reshape(B, T, d)
        o = _Linear(W, p + ".self_attn.out_proj", lora, scaling)(o)
        h = res + o
        res = h
        x = layer_norm(h, W[p + ".layer_norm2.weight"], W[p + ".layer_norm2.bias"], eps)
        x = _Linear(W, p + ".mlp.fc1", lora, scaling)(x)
        x = quick_gelu(x)
        x = _Linear(W, p + ".mlp.fc2", lora, scaling)(x)
        h = res + x
    return h


def image_features(W, cfg, pixel_values: Array, lora=None, normalize: bool = True) -> Array:
    """pixel_values float32 [B,3,S,S] -> [B, proj_dim] (unit-norm if normalize)."""
    B = pixel_values.shape[0]
    p, g, d = cfg.patch, cfg.grid, cfg.vision.hidden
    # conv2d(k=s=p, no bias) == patchify + matmul (modeling_clip.py:148-154, 209)
    x = pixel_values.reshape(B, cfg.channels, g, p, g, p).transpose(0, 2, 4, 1, 3, 5)
    x = x.reshape(B, g * g, cfg.channels * p * p)
    wp = W["vision_model.embeddings.patch_embedding.weight"].reshape(d, -1)
    pe = x @ wp.T
    cls = np.broadcast_to(W["vision_model.embeddings.class_embedding"], (B, 1, d))
    h = np.concatenate([cls, pe], axis=1) + W["vision_model.embeddings.position_embedding.weight"][None]
    h = layer_norm(h, W["vision_model.pre_layrnorm.weight"], W["vision_model.pre_layrnorm.bias"], cfg.ln_eps)
    h = _encoder(W, lora, cfg.lora_scaling, "vision_model", h.astype(np.float32), cfg.vision.layers,
                 cfg.vision.heads, cfg.ln_eps, causal=False)
    pooled = layer_norm(h[:, 0, :], W["vision_model.post_layernorm.weight"],
                        W["vision_model.post_layernorm.bias"], cfg.ln_eps)
    f = pooled @ W["visual_projection.weight"].T
    if normalize:
        f = f / np.linalg.norm(f, axis=-1, keepdims=True)
    return f.astype(np.float32)


def eos_positions(ids: Array, eos_token_id: int) -> Array:
    """modeling_clip.py:561-582: first index of eos (== argmax(ids) when eos is
    the largest id, the legacy eos_token_id==2 rule)."""
    if eos_token_id == 2:
        return ids.argmax(-1)
    return (ids == eos_token_id).astype(np.int32).argmax(-1)


def text_features(W, cfg, ids: Array, lora=None, normalize: bool = True) -> Array:
    """ids int [B,L] (L<=max_pos) -> [B, proj_dim]."""
    B, L = ids.shape
    h = W["text_model.embeddings.token_embedding.weight"][ids] + \
        W["text_model.embeddings.position_embedding.weight"][:L][None]
    h = _encoder(W, lora, cfg.lora_scaling, "text_model", h.astype(np.float32), cfg.text.layers,
                 cfg.text.heads, cfg.ln_eps, causal=True)
    pos = eos_positions(ids, cfg.eos_token_id)
    pooled = h[np.arange(B), pos]
    pooled = layer_norm(pooled, W["text_model.final_layer_norm.weight"],
                        W["text_model.final_layer_norm.bias"], cfg.ln_eps)
    f = pooled @ W["text_projection.weight"].T
    if normalize:
        f = f / np.linalg.norm(f, axis=-1, keepdims=True)
    return f.astype(np.float32)
