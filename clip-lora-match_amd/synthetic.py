"""Seeded synthetic inputs of the benchmark shapes.

* images: uint8 HWC image_size^2 x 3, uniform [0,255], numpy PCG64 seed base+i
* captions: int32 [N, L]: ids[:,0]=BOS, per-row length L_i ~ U[8, L],
  ids[:,1:L_i-1] ~ U[0, eos-2], ids[:,L_i-1]=EOS, padded with EOS
  (the CLIP tokenizer pads with the EOS id, as models/clip_model.py:133-138
  produces with padding=True)
* index rows / queries: normalised Gaussian, optionally fp16-rounded
"""
from __future__ import annotations

import numpy as np


def images_u8(n: int, size: int, seed: int = 1234) -> np.ndarray:
    out = np.empty((n, size, size, 3), np.uint8)
    for i in range(n):
        out[i] = np.random.Generator(np.random.PCG64(seed + i)).integers(
            0, 256, size=(size, size, 3), dtype=np.uint8)
    return out


def captions(n: int, L: int, bos: int, eos: int, seed: int = 99, min_len: int = 8) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    ids = np.full((n, L), eos, np.int32)
    ids[:, 0] = bos
    lens = rng.integers(min(min_len, L), L + 1, size=n)
    for i in range(n):
        li = int(lens[i])
        ids[i, 1:li - 1] = rng.integers(0, eos - 1, size=li - 2)
        ids[i, li - 1] = eos
    return ids


def gaussian_rows(n: int, dim: int, seed: int, fp16: bool = True) -> np.ndarray:
    rng = np.random.Generator(np.random.PCG64(seed))
    x = rng.standard_normal((n, dim), dtype=np.float32)
    x /= np.linalg.norm(x, axis=-1, keepdims=True)
    if fp16:
        x = x.astype(np.float16)
    return x
