"""Host-side CLIPProcessor replacement (the `processor` load_clip_model returns).

Image side (CLIPImageProcessor with the reference's settings, config/clip_config.yaml:7-13;
models/clip_model.py:105-110, src/embedding/embed_image.py:13-19,36-41): the host only decodes
(PIL `Image.open(path).convert("RGB")`, the reference's own loader); everything after runs on the
GPU. Images already image_size^2 go straight to the encoder as uint8 (resize and crop are
identities); any other size goes through clm_resize_crop (csrc/k_image.hip): shortest-edge
BICUBIC resize + centre crop with PIL's 8-bit resampling arithmetic, bit-identical to
CLIPImageProcessor's resize + center_crop. Rescale / normalise then run fused in the encoder's
patchify kernel (a 3 x 256 float32 LUT, bit-identical to the processor's float64-rescale +
float32-normalise, see oracle/clip_ref.py:preprocess_u8). transformers is not imported.

Text side: tokenizer.ClipBPETokenizer (CLIP byte-level BPE, host-side) over a local
vocab.json + merges.txt given via `tokenizer_dir` / $CLM_TOKENIZER_DIR (the CLIP
vocabulary is not shipped in this environment); without one, callers
pass token ids directly (list[int] / [n, L] tensor), BOS ... EOS padded with EOS
exactly as CLIPTokenizer(padding=True) produces.
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path
from typing import List, Optional, Sequence, Union

import numpy as np
import torch

from .config import ModelConfig

ImageLike = Union[str, Path, "PIL.Image.Image", np.ndarray]  # noqa: F821


class TokenizerUnavailable(RuntimeError):
    pass


class ClipProcessor:
    def __init__(self, cfg: ModelConfig, tokenizer_dir: Optional[str] = None):
        self.cfg = cfg
        self.image_size = cfg.image_size
        self.mean = cfg.mean
        self.std = cfg.std
        self._hf_image = None
        self._pin = None                     # pinned staging of images_u8 (grow-only)
        self._pin_lock = threading.Lock()
        self.tokenizer = None
        tdir = tokenizer_dir or os.environ.get("CLM_TOKENIZER_DIR")
        if tdir and Path(tdir, "vocab.json").exists() and Path(tdir, "merges.txt").exists():
            from .tokenizer import ClipBPETokenizer
            self.tokenizer = ClipBPETokenizer.from_dir(tdir, model_max_length=cfg.max_pos)

    # ------------------------------------------------------------- images --
    @staticmethod
    def load_image(image: ImageLike):
        """PIL RGB image: the reference's _load_image (embed_image.py:13-19; clip_model.py:102-105)."""
        from PIL import Image
        if isinstance(image, Image.Image):
            return image.convert("RGB")
        if isinstance(image, np.ndarray):
            return Image.fromarray(image).convert("RGB")
        p = Path(image)
        if not p.exists():
            raise FileNotFoundError(f"Image not found: {p}")
        return Image.open(p).convert("RGB")

    @classmethod
    def decode(cls, image: ImageLike) -> np.ndarray:
        """uint8 [H, W, 3] RGB pixels of one image (host decode only)."""
        if isinstance(image, np.ndarray) and image.dtype == np.uint8 and image.ndim == 3 and image.shape[2] == 3:
            return np.ascontiguousarray(image)
        return np.asarray(cls.load_image(image), dtype=np.uint8)

    def images_u8(self, images: Sequence[ImageLike], device) -> torch.Tensor:
        """uint8 [n, S, S, 3] on `device`: the CLIPImageProcessor resize + centre crop of every
        image (clm_resize_crop for sizes other than S x S), ready for encode_pixels."""
        from . import _capi
        S = self.image_size
        device = torch.device(device)
        arrs = [self.decode(im) for im in images]
        if all(a.shape[:2] == (S, S) for a in arrs):
            if not arrs:
                return torch.zeros((0, S, S, 3), dtype=torch.uint8, device=device)
            return torch.from_numpy(np.stack(arrs)).to(device)
        _capi.require_gpu()
        sizes = np.array([a.shape[0] * a.shape[1] * 3 for a in arrs], np.int64)
        offs = np.zeros(len(arrs), np.int64)
        offs[1:] = np.cumsum(sizes)[:-1]
        total = int(sizes.sum())
        hw = np.array([a.shape[:2] for a in arrs], np.int32).reshape(-1)
        out = torch.empty((len(arrs), S, S, 3), dtype=torch.uint8, device=device)
        # one grow-only pinned staging buffer per processor (no pinned allocation per
        # call); it is free again when clm_resize_crop returns (that call drains the stream)
        with self._pin_lock:
            if self._pin is None or self._pin.numel() < total:
                self._pin = torch.empty(max(total, 1 << 20), dtype=torch.uint8, pin_memory=True)
            flat = self._pin[:total]
            fv = flat.numpy()
            for a, o, n in zip(arrs, offs, sizes):
                fv[o:o + n] = a.reshape(-1)
            src = flat.to(device, non_blocking=True)
            _capi.check(_capi.lib().clm_resize_crop(
                device.index if device.index is not None else torch.cuda.current_device(), _capi.ptr(src),
                offs.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), hw.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                len(arrs), S, _capi.ptr(out), _capi.stream_of(device)), "resize_crop")
        return out

    def normalize_lut(self) -> np.ndarray:
        """float32 [3, 256]: pixel value v of channel c -> float32(float64(v) * (1/255)) then
        (x - mean[c]) / std[c] in float32, i.e. CLIPImageProcessor's rescale + normalise
        (TF/image_transforms.py:118-122, 419-439) tabulated per byte value."""
        x = (np.arange(256, dtype=np.float64) * (1 / 255)).astype(np.float32)
        m = np.asarray(self.mean, np.float32)[:, None]
        s = np.asarray(self.std, np.float32)[:, None]
        return ((x[None, :] - m) / s).astype(np.float32)

    def pixel_values(self, images: Sequence[ImageLike], device=None) -> torch.Tensor:
        """float32 [n, 3, S, S] exactly as CLIPImageProcessor (resize shortest edge, centre crop,
        rescale, normalise); computed on the GPU, returned on the CPU."""
        from . import _capi
        _capi.require_gpu()
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        u8 = self.images_u8(images, dev).permute(0, 3, 1, 2).long()      # [n, 3, S, S]
        lut = torch.from_numpy(self.normalize_lut()).to(dev)
        ch = torch.arange(3, device=dev).view(1, 3, 1, 1) * 256
        return lut.view(-1)[u8 + ch].cpu()

    # --------------------------------------------------------------- text --
    def token_ids(self, text: Union[str, Sequence[str], Sequence[int], Sequence[Sequence[int]], torch.Tensor],
                  max_length: Optional[int] = None) -> torch.Tensor:
        """int32 [n, L] padded with EOS (CLIPTokenizer padding=True, truncation=True)."""
        L = max_length or self.cfg.max_pos
        eos = self.cfg.eos_token_id
        if isinstance(text, torch.Tensor):
            t = text if text.dim() == 2 else text.unsqueeze(0)
            return t.to(torch.int32)
        if isinstance(text, np.ndarray):
            t = torch.from_numpy(np.atleast_2d(text))
            return t.to(torch.int32)
        if isinstance(text, str) or (isinstance(text, (list, tuple)) and text and isinstance(text[0], str)):
            texts = [text] if isinstance(text, str) else list(text)
            if self.tokenizer is None:
                raise TokenizerUnavailable(
                    "the CLIP BPE vocabulary is not available offline; set CLM_TOKENIZER_DIR to a directory "
                    "with vocab.json + merges.txt, or pass token ids")
            enc = self.tokenizer(texts, padding=True, truncation=True, max_length=L, return_tensors="pt")
            ids = enc["input_ids"].to(torch.int32)
            if (ids >= self.cfg.vocab).any():
                raise ValueError(f"tokenizer produced ids >= the model's vocabulary size {self.cfg.vocab}")
            return ids
        rows: List[List[int]] = [list(text)] if (text and isinstance(text[0], (int, np.integer))) else \
            [list(r) for r in text]
        rows = [r[:L] if len(r) <= L else r[:L - 1] + [eos] for r in rows]
        width = max(len(r) for r in rows) if rows else 1
        out = torch.full((len(rows), width), eos, dtype=torch.int32)
        for i, r in enumerate(rows):
            out[i, :len(r)] = torch.tensor(r, dtype=torch.int32)
        return out

    def __call__(self, images=None, text=None, return_tensors: str = "pt", padding=True, truncation=True,
                 max_length=None, **kw):
        out = {}
        if images is not None:
            imgs = images if isinstance(images, (list, tuple)) else [images]
            out["pixel_values"] = self.pixel_values(imgs)
        if text is not None:
            ids = self.token_ids(text, max_length)
            out["input_ids"] = ids.long()
            out["attention_mask"] = (torch.cumsum((ids == self.cfg.eos_token_id).int(), 1) <= 1).long()
        return out
