"""Query fusion and item search: the hot-path part of src/embedding/seeker_service.py.

  fuse_query_embeddings   seeker_service.py:148-157  v = w_text*t + w_image*i; v / ||v||, batched
                          over [n, D] rows in one gfx950 kernel (clm_fuse_queries)
  build_query_embedding   seeker_service.py:84-157   text and/or image query -> (D,) f32 CPU
  search_items            seeker_service.py:159-186  query embedding -> List[SearchResult]

SeekerService re-reads the .pt index from disk on every query (:183); here the index
stays resident in HBM (a TextSearchIndex passed in by the caller). The YOLO crop step
(:120-138) is outside the encode/search path and is not part of this module.
"""
from __future__ import annotations

from pathlib import Path
from typing import List, Optional, Union

import torch

from . import _capi as C
from .clip_model import encode_image, encode_text
from .search import SearchResult, TextSearchIndex


def _rows(x: torch.Tensor, name: str) -> torch.Tensor:
    t = torch.as_tensor(x)
    if t.dim() == 1:
        t = t.unsqueeze(0)
    if t.dim() != 2:
        raise ValueError(f"{name} must be (D,) or (n, D), got {tuple(t.shape)}")
    return t


def fuse_query_embeddings(text_emb: Optional[torch.Tensor], image_emb: Optional[torch.Tensor],
                          w_text: float = 0.5, w_image: float = 0.5) -> torch.Tensor:
    """Row-wise weighted fusion + L2 normalise (seeker_service.py:148-157).

    One side None: that side alone, renormalised (:149-152). Both: w_text*text + w_image*image,
    renormalised (:155-156). Inputs (D,) or (n, D); the result has the inputs' shape, dtype
    float32, on the inputs' device. Raises ValueError when both are None (:101-102).
    """
    if text_emb is None and image_emb is None:
        raise ValueError("Minimal harus ada query_text atau query_image_path.")
    C.require_gpu()
    first = text_emb if text_emb is not None else image_emb
    one_d = torch.as_tensor(first).dim() == 1
    out_dev = torch.as_tensor(first).device
    dev = torch.device("cuda", torch.cuda.current_device())
    a = _rows(first, "query embedding").to(dev, torch.float32).contiguous()
    b = None
    if text_emb is not None and image_emb is not None:
        b = _rows(image_emb, "image embedding").to(dev, torch.float32).contiguous()
        if b.shape != a.shape:
            raise ValueError(f"text {tuple(a.shape)} and image {tuple(b.shape)} embeddings differ in shape")
    wa = float(w_text) if b is not None else 1.0
    out = torch.empty_like(a)
    C.check(C.lib().clm_fuse_queries(dev.index, C.ptr(a), wa, C.ptr(b) if b is not None else None,
                                     float(w_image), a.shape[0], a.shape[1], C.ptr(out), C.stream_of(dev)),
            "clm_fuse_queries")
    out = out.to(out_dev)
    return out.squeeze(0) if one_d else out


def build_query_embedding(query_text, query_image_path: Optional[Union[str, Path]], model, processor, device,
                          w_text: float = 0.5, w_image: float = 0.5) -> torch.Tensor:
    """Text-only, image-only or text+image query -> unit-norm (D,) f32 CPU (seeker_service.py:84-157).

    `query_text` is a caption (needs the local CLIP tokenizer) or its token ids; an empty or
    whitespace-only string counts as absent (:98).
    """
    if isinstance(query_text, str):
        have_text = query_text.strip() != ""
    else:
        have_text = query_text is not None and len(query_text) > 0
    have_image = query_image_path is not None
    if not have_text and not have_image:
        raise ValueError("Minimal harus ada query_text atau query_image_path.")
    t = encode_text(query_text, model, processor, device) if have_text else None
    i = encode_image(query_image_path, model, processor, device) if have_image else None
    return fuse_query_embeddings(t, i, w_text, w_image).to("cpu", torch.float32)


def search_items(index: TextSearchIndex, model, processor, device, query_text=None,
                 query_image_path: Optional[Union[str, Path]] = None, top_k: int = 5,
                 root_dir: Optional[Union[str, Path]] = None) -> List[SearchResult]:
    """SeekerService.search_items (seeker_service.py:159-186) against a resident index.

    A relative `query_image_path` is resolved under `root_dir` (the service's root, :173);
    a missing image raises FileNotFoundError (:174-175).
    """
    img_path = None
    if query_image_path:
        p = Path(query_image_path)
        img_path = ((Path(root_dir) / p) if root_dir is not None else p).resolve()
        if not img_path.exists():
            raise FileNotFoundError(f"Query image not found: {img_path}")
    q = build_query_embedding(query_text, img_path, model, processor, device)
    return index.search_with_embedding(q, top_k=top_k)


__all__ = ["fuse_query_embeddings", "build_query_embedding", "search_items"]
