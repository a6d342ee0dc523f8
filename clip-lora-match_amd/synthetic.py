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


# (H, W) of the odd-size image set: tiny, one pixel, square off by one, both aspect orientations,
# an extreme strip whose resized long edge is 34,458 pixels, and camera-like sizes
ODD_SIZES = ((46, 36), (1, 1), (2, 7), (225, 225), (260, 300), (224, 500), (500, 224), (13, 2000),
             (999, 1001), (480, 640), (1599, 899))


def odd_images(seed: int = 4242, sizes=ODD_SIZES) -> list:
    """uint8 [H, W, 3] images at sizes other than 224^2: smooth colour gradients + noise, so the
    bicubic resample sees both edges and texture (numpy PCG64 seed + i)."""
    out = []
    for i, (h, w) in enumerate(sizes):
        rng = np.random.Generator(np.random.PCG64(seed + i))
        y = np.linspace(0.0, 1.0, h)[:, None, None]
        x = np.linspace(0.0, 1.0, w)[None, :, None]
        phase = rng.uniform(0, 2 * np.pi, size=(1, 1, 3))
        base = 127.5 + 100.0 * np.sin(6.0 * x + 4.0 * y + phase)
        noise = rng.normal(0.0, 30.0, size=(h, w, 3))
        out.append(np.clip(np.rint(base + noise), 0, 255).astype(np.uint8))
    return out


class DeviceImages:
    """n synthetic uint8 [S, S, 3] images generated on the device batch by batch
    (clm_synth_images): image i's pixels are a hash of (seed, i) only, so any shard / batch split
    of the index build (BASELINE configs[2]) sees the same images. Sequence-like: len() and
    batch(start, stop) -> uint8 device tensor [stop - start, S, S, 3]."""

    def __init__(self, n: int, size: int, seed: int = 1234, device=None):
        import torch
        self.n, self.size, self.seed = int(n), int(size), int(seed)
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())

    def __len__(self) -> int:
        return self.n

    def batch(self, start: int, stop: int, out=None):
        import torch
        from . import _capi as C
        start, stop = max(0, int(start)), min(self.n, int(stop))
        n = max(stop - start, 0)
        if out is None:
            out = torch.empty((n, self.size, self.size, 3), dtype=torch.uint8, device=self.device)
        C.check(C.lib().clm_synth_images(self.device.index, self.seed, start, n, self.size, C.ptr(out),
                                         C.stream_of(self.device)), "clm_synth_images")
        return out[:n]


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


def clustered_rows(n_centers: int, per: int, dim: int, noise: float, seed: int, noise_seed=None) -> np.ndarray:
    """Unit rows in tight clusters (center + Gaussian noise of norm ~`noise`), rows of one
    cluster contiguous. Top-k scores of a query near a center differ by ~1e-5..1e-4, below
    the fp16 operand rounding: only an exact re-score orders them like fp32 arithmetic.
    noise_seed: draw the noise from a separate stream (same centers, fresh noise)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    c = rng.standard_normal((n_centers, dim)).astype(np.float32)
    c /= np.linalg.norm(c, axis=-1, keepdims=True)
    if noise_seed is not None:
        rng = np.random.Generator(np.random.PCG64(noise_seed))
    x = np.repeat(c, per, axis=0) + rng.standard_normal((n_centers * per, dim)).astype(np.float32) * \
        np.float32(noise / np.sqrt(dim))
    return (x / np.linalg.norm(x, axis=-1, keepdims=True)).astype(np.float32)


def fp32_search_inputs():
    """The fp32 search fixture inputs (tests/golden/search_fp32.npz holds the reference's outputs
    on them): Gaussian rows [4096, 512] / queries [64, 512], and 64 tight clusters of 64 rows with
    one query near each center -- all fp32, not fp16-representable."""
    dim = 512
    return (gaussian_rows(4096, dim, seed=27, fp16=False), gaussian_rows(64, dim, seed=28, fp16=False),
            clustered_rows(64, 64, dim, 0.05, seed=29), clustered_rows(64, 1, dim, 0.05, seed=29, noise_seed=30))
