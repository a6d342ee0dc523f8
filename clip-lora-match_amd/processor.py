"""Host-side CLIPProcessor replacement (the `processor` load_clip_model returns).

Image side (CLIPImageProcessor, config/clip_config.yaml:7-13): for RGB images
already at image_size^2 the resize and centre-crop are identities, so the raw
uint8 pixels go to the GPU and rescale/normalise run fused in the patchify
kernel (bit-identical to the processor's float64-rescale + float32-normalise,
see oracle/clip_ref.py:preprocess_u8). Any other size is resized/cropped on
the host by transformers' own CLIPImageProcessor when importable, else by a
PIL bicubic shortest-edge resize + centre crop, and handed over as float32
pixel_values.

Text side: tokenizer.ClipBPETokenizer (CLIP byte-level BPE, host-side) over a local
vocab.json + merges.txt given via `tokenizer_dir` / $CLM_TOKENIZER_DIR (the CLIP
vocabulary is not shipped in this environment); without one, callers
pass token ids directly (list[int] / [n, L] tensor), BOS ... EOS padded with EOS
exactly as CLIPTokenizer(padding=True) produces.
"""
from __future__ import annotations

import os
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
        self.tokenizer = None
        tdir = tokenizer_dir or os.environ.get("CLM_TOKENIZER_DIR")
        if tdir and Path(tdir, "vocab.json").exists() and Path(tdir, "merges.txt").exists():
            from .tokenizer import ClipBPETokenizer
            self.tokenizer = ClipBPETokenizer.from_dir(tdir, model_max_length=cfg.max_pos)

    # ------------------------------------------------------------- images --
    @staticmethod
    def load_image(image: ImageLike):
        from PIL import Image
        if isinstance(image, Image.Image):
            return image.convert("RGB")
        if isinstance(image, np.ndarray):
            return Image.fromarray(image).convert("RGB")
        p = Path(image)
        if not p.exists():
            raise FileNotFoundError(f"Image not found: {p}")
        return Image.open(p).convert("RGB")

    def images_u8(self, images: Sequence[ImageLike]) -> Optional[np.ndarray]:
        """uint8 [n,S,S,3] when every image is already S x S (fast path), else None."""
        S = self.image_size
        out = []
        for im in images:
            if isinstance(im, np.ndarray) and im.dtype == np.uint8 and im.shape == (S, S, 3):
                out.append(im)
                continue
            pil = self.load_image(im)
            if pil.size != (S, S):
                return None
            out.append(np.asarray(pil, dtype=np.uint8))
        return np.stack(out) if out else np.zeros((0, S, S, 3), np.uint8)

    def pixel_values(self, images: Sequence[ImageLike]) -> np.ndarray:
        """float32 [n,3,S,S] exactly as CLIPImageProcessor (resize shortest edge, centre crop,
        rescale, normalise)."""
        pils = [self.load_image(im) for im in images]
        S = self.image_size
        try:
            if self._hf_image is None:
                from transformers import CLIPImageProcessor
                self._hf_image = CLIPImageProcessor(size={"shortest_edge": S},
                                                    crop_size={"height": S, "width": S},
                                                    image_mean=list(self.mean), image_std=list(self.std))
            return np.asarray(self._hf_image(images=pils, return_tensors="np")["pixel_values"], np.float32)
        except ImportError:
            pass
        from PIL import Image
        out = []
        for im in pils:
            w, h = im.size
            if w <= h:
                nw, nh = S, int(S * h / w)
            else:
                nw, nh = int(S * w / h), S
            im = im.resize((nw, nh), Image.BICUBIC)
            left, top = (nw - S) // 2, (nh - S) // 2
            im = im.crop((left, top, left + S, top + S))
            x = (np.asarray(im, np.float64) * (1.0 / 255.0)).astype(np.float32)
            x = (x - np.asarray(self.mean, np.float32)) / np.asarray(self.std, np.float32)
            out.append(x.transpose(2, 0, 1))
        return np.stack(out).astype(np.float32)

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
            out["pixel_values"] = torch.from_numpy(self.pixel_values(imgs))
        if text is not None:
            ids = self.token_ids(text, max_length)
            out["input_ids"] = ids.long()
            out["attention_mask"] = (torch.cumsum((ids == self.cfg.eos_token_id).int(), 1) <= 1).long()
        return out
