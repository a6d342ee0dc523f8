"""ORACLE -- test infrastructure only. Never imported by the product path.

numpy restatement of the image half of the reference's CLIPProcessor for images of ANY size,
so the HIP resize + centre-crop kernel (csrc/k_image.hip) can be checked bit for bit.

The reference path (models/clip_model.py:105-112, src/embedding/embed_image.py:13-19,36-41):
PIL `Image.open(path).convert("RGB")` -> CLIPProcessor(images=...) with the openai/clip-vit-base-patch32
preprocessor settings (config/clip_config.yaml:7-13): resize shortest edge to 224 with BICUBIC,
centre-crop 224 x 224, rescale 1/255, normalise by the CLIP mean / std. transformers 5.15 runs that
through its PIL backend when torchvision is absent (it is, here and on the GPU box), which is the
transformers 4.x "slow" CLIPImageProcessor the reference was written against:
  * output size      TF/image_transforms.py:296-299 get_resize_output_image_size
                     (short -> S, long -> int(S * long / short), default_to_square=False)
  * resize           TF/image_transforms.py:361-381 -> PIL Image.resize((w, h), BICUBIC, reducing_gap=None)
  * centre crop      TF/image_transforms.py:488-503 top = (h - S) // 2, left = (w - S) // 2
  * rescale/normalise as oracle.clip_ref.preprocess_u8 (TF/image_transforms.py:118-122, 419-439)
(TF/ = /usr/local/lib/python3.10/dist-packages/transformers/.)

PIL's BICUBIC resize is a third-party algorithm absent from /root/reference: Pillow 12.2.0 (the
version installed here and on the GPU box; the reference's requirements.txt leaves Pillow unpinned),
src/libImaging/Resample.c. Its published algorithm, restated below:
  * separable, horizontal pass first into a uint8 intermediate, then the vertical pass
    (ImagingResampleInner); a pass whose size does not change is an exact copy either way;
  * per output coordinate xx (precompute_coeffs): scale = in / out, filterscale = max(scale, 1),
    support = 2 * filterscale, center = (xx + 0.5) * scale, taps [xmin, xmin + n) with
    xmin = max(0, (int)(center - support + 0.5)), xmax = min(in, (int)(center + support + 0.5)),
    w_j = cubic((j + xmin - center + 0.5) / filterscale), a = -0.5 (bicubic_filter), normalised by
    their sequential sum;
  * weights to fixed point with 22 fraction bits (normalize_coeffs_8bpc: round half away from
    zero), accumulation from 1 << 21 in 32-bit integers, output clip8 = clamp(acc >> 22, 0, 255).

Pinned: equal bit for bit to PIL's Image.resize and to transformers' CLIPImageProcessor on the
reference's 17 committed images and on random sizes (tests/golden/make_image_golden.py,
tests/test_oracle.py).
"""
from __future__ import annotations

import numpy as np

PRECISION_BITS = 22


def cubic(x: np.ndarray) -> np.ndarray:
    """bicubic_filter, a = -0.5, evaluated in Resample.c's operation order."""
    a = -0.5
    x = np.abs(x)
    near = ((a + 2.0) * x - (a + 3.0)) * x * x + 1.0
    far = (((x - 5.0) * x + 8.0) * x - 4.0) * a
    return np.where(x < 1.0, near, np.where(x < 2.0, far, 0.0))


def coeffs(in_size: int, out_size: int):
    """(xmin [out], n [out], fixed-point weights int64 [out, ksize]) for every output coordinate."""
    scale = float(in_size) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(np.ceil(support)) * 2 + 1
    xx = np.arange(out_size, dtype=np.float64)
    center = (xx + 0.5) * scale
    ss = 1.0 / filterscale
    xmin = np.trunc(center - support + 0.5).astype(np.int64)
    xmin = np.maximum(xmin, 0)
    xmax = np.trunc(center + support + 0.5).astype(np.int64)
    xmax = np.minimum(xmax, in_size)
    n = xmax - xmin
    j = np.arange(ksize, dtype=np.int64)
    w = cubic(((j[None, :] + xmin[:, None]).astype(np.float64) - center[:, None] + 0.5) * ss)
    w = np.where(j[None, :] < n[:, None], w, 0.0)
    ww = np.zeros(out_size, np.float64)
    for t in range(ksize):               # sequential sum, as the C loop
        ww = ww + w[:, t]
    w = np.where(ww[:, None] != 0.0, w / np.where(ww == 0.0, 1.0, ww)[:, None], w)
    one = float(1 << PRECISION_BITS)
    k = np.where(w < 0, np.trunc(-0.5 + w * one), np.trunc(0.5 + w * one)).astype(np.int64)
    return xmin, n, k


def _clip8(acc: np.ndarray) -> np.ndarray:
    return np.clip(acc >> PRECISION_BITS, 0, 255).astype(np.uint8)


def _pass(img: np.ndarray, axis: int, xmin, n, k) -> np.ndarray:
    """one separable pass along `axis` (0 rows, 1 columns) of a uint8 [H, W, C] image."""
    src = np.moveaxis(img.astype(np.int64), axis, 0)     # [in, other, C]
    acc = np.full((len(xmin),) + src.shape[1:], 1 << (PRECISION_BITS - 1), np.int64)
    last = src.shape[0] - 1
    for t in range(k.shape[1]):
        idx = np.minimum(xmin + t, last)
        wt = np.where(t < n, k[:, t], 0)
        acc += src[idx] * wt[:, None, None]
    return np.moveaxis(_clip8(acc), 0, axis)


def resize_bicubic(img: np.ndarray, out_w: int, out_h: int) -> np.ndarray:
    """PIL Image.resize((out_w, out_h), BICUBIC) of a uint8 [H, W, 3] RGB array."""
    H, W = img.shape[:2]
    out = img
    if out_w != W:
        out = _pass(out, 1, *coeffs(W, out_w))
    if out_h != H:
        out = _pass(out, 0, *coeffs(H, out_h))
    return out


def shortest_edge_size(h: int, w: int, S: int):
    """(new_h, new_w) of get_resize_output_image_size(default_to_square=False)."""
    short, long = (w, h) if w <= h else (h, w)
    new_short, new_long = S, int(S * long / short)
    return (new_long, new_short) if w <= h else (new_short, new_long)


def resize_crop_u8(img: np.ndarray, S: int) -> np.ndarray:
    """uint8 [H, W, 3] -> uint8 [S, S, 3]: shortest-edge bicubic resize + centre crop."""
    H, W = img.shape[:2]
    nh, nw = shortest_edge_size(H, W, S)
    r = resize_bicubic(img, nw, nh)
    top, left = (nh - S) // 2, (nw - S) // 2
    return np.ascontiguousarray(r[top:top + S, left:left + S])


def resize_crop_u8_window(img: np.ndarray, S: int) -> np.ndarray:
    """The same crop computed only on the window the crop keeps (the HIP kernel's schedule):
    horizontal taps of the S kept columns over the source rows the S kept rows need, then the
    vertical taps. Equal to resize_crop_u8 (each output pixel depends only on its taps)."""
    H, W = img.shape[:2]
    nh, nw = shortest_edge_size(H, W, S)
    top, left = (nh - S) // 2, (nw - S) // 2
    xmin, xn, xk = coeffs(W, nw)
    ymin, yn, yk = coeffs(H, nh)
    xmin, xn, xk = xmin[left:left + S], xn[left:left + S], xk[left:left + S]
    ymin, yn, yk = ymin[top:top + S], yn[top:top + S], yk[top:top + S]
    r0, r1 = int(ymin[0]), int((ymin + yn).max())
    tmp = _pass(img[r0:r1], 1, xmin, xn, xk)
    return _pass(tmp, 0, ymin - r0, yn, yk)
