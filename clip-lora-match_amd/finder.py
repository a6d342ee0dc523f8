"""The finder's report flow (src/embedding/finder_service.py:41-216) on a resident index.

FinderService.report_item copies the uploaded image, encodes the item's *description text*
(+ ", ditemukan di <location>", :158-161) with CLIP+LoRA, re-normalises it (:165-169), then
re-loads the whole .pt index, torch.cat's one row onto it and re-saves the whole file on every
report (:171-185), and inserts a Postgres row (:187-204). Here:

* the index stays resident (TextSearchIndex: fp32 host mirror in a capacity-doubling buffer +
  the HBM index): one report appends in amortised O(1), and a search right after a report
  sees the new row without a reload;
* persistence keeps the reference .pt format ({"embeddings", "image_paths", "texts"},
  :93-103) and is decoupled from the append: `save_every=1` re-saves after every report as the
  reference does, `save_every=n` after every n-th, `save_every=0` only on `flush()`;
* reports can be batched (`report_items`): one encoder launch sequence for many descriptions;
* the Postgres insert and the YOLO crop (:140-156, off by default in the API, main.py:34) are
  outside the encode/search path and are not part of this module: the returned record carries
  the index row number where the reference returns the database id.
"""
from __future__ import annotations

import shutil
from datetime import datetime
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Union

import torch

from .clip_model import encode_text
from .search import TextSearchIndex

PathLike = Union[str, Path]


def _full_text(description: str, location: Optional[str]) -> str:
    # finder_service.py:159-161
    return f"{description}, ditemukan di {location}" if location else description


class FinderIndex:
    """Resident index + report flow. `index_path` need not exist yet (a new index, :86-91)."""

    def __init__(self, model, processor, device, index_path: PathLike, root_dir: PathLike,
                 upload_dir: PathLike, save_every: int = 1, dim: Optional[int] = None):
        self.model, self.processor, self.device = model, processor, device
        self.index_path = Path(index_path)
        self.root_dir = Path(root_dir).resolve()
        self.upload_dir = Path(upload_dir)
        self.upload_dir.mkdir(parents=True, exist_ok=True)
        if save_every < 0:
            raise ValueError("save_every must be >= 0")
        self.save_every = int(save_every)
        self._unsaved = 0
        if self.index_path.exists():
            self.index = TextSearchIndex(self.index_path, device=device)
        else:
            d = int(dim if dim is not None else model.cfg.proj_dim)
            self.index = TextSearchIndex(embeddings=torch.empty((0, d)), image_paths=[], texts=[], device=device)

    def _store_image(self, src_image_path: PathLike) -> str:
        src = Path(src_image_path).resolve()
        if not src.exists():
            raise FileNotFoundError(f"Source image not found: {src}")
        dest = (self.upload_dir / src.name).resolve()
        if src != dest:
            shutil.copy2(src, dest)
        return str(dest.relative_to(self.root_dir)).replace("\\", "/")

    def report_items(self, src_image_paths: Sequence[PathLike], descriptions: Sequence,
                     locations: Optional[Sequence[Optional[str]]] = None,
                     reporters: Optional[Sequence[Optional[str]]] = None,
                     found_at: Optional[Sequence[Optional[datetime]]] = None) -> List[Dict]:
        """Report n items at once: n descriptions encoded in one batch, n rows appended."""
        n = len(descriptions)
        if len(src_image_paths) != n:
            raise ValueError(f"{len(src_image_paths)} images vs {n} descriptions")
        locations = list(locations) if locations is not None else [None] * n
        reporters = list(reporters) if reporters is not None else [None] * n
        found_at = list(found_at) if found_at is not None else [None] * n
        # checked before any image is copied: token-id descriptions have no text to append a
        # location to (finder_service.py:123-131 builds "<description>, ditemukan di <location>"),
        # and one batch is either all strings or all token ids
        is_str = [isinstance(d, str) for d in descriptions]
        if any(is_str) and not all(is_str):
            raise ValueError("descriptions must be all strings or all token-id lists, not a mix")
        if not all(is_str) and any(loc for loc in locations):
            raise ValueError("a location needs a string description (token ids cannot carry it)")
        rel_paths = [self._store_image(p) for p in src_image_paths]
        texts = []
        for d, loc in zip(descriptions, locations):
            texts.append(_full_text(d, loc) if isinstance(d, str) else d)
        if n == 0:
            return []
        if all(isinstance(t, str) for t in texts) or n == 1:
            ids = self.processor.token_ids(texts if n > 1 or isinstance(texts[0], str) else texts[0])
        else:
            ids = self.processor.token_ids(texts)
        emb = self.model.encode_ids(ids.to(self.model.device), normalize=True).to("cpu", torch.float32)
        first = self.index.num_items
        self.index.append(emb, rel_paths, [t if isinstance(t, str) else "" for t in texts])
        self._unsaved += n
        if self.save_every and self._unsaved >= self.save_every:
            self.flush()
        out = []
        for j in range(n):
            ts = found_at[j] or datetime.now()
            out.append({"id": first + j, "image_path": rel_paths[j],
                        "description": texts[j] if isinstance(texts[j], str) else "",
                        "location": locations[j], "found_at": ts.isoformat(), "reporter": reporters[j]})
        return out

    def report_item(self, src_image_path: PathLike, description, location: Optional[str] = None,
                    reporter: Optional[str] = None, found_at: Optional[datetime] = None) -> Dict:
        """finder_service.py:107-216 (without the database insert)."""
        return self.report_items([src_image_path], [description], [location], [reporter], [found_at])[0]

    def flush(self) -> None:
        """Write the index in the reference .pt format (finder_service.py:93-103)."""
        self.index.save(self.index_path)
        self._unsaved = 0
        print(f"[FinderService] Index updated and saved to: {self.index_path}")

    def search(self, query_emb: torch.Tensor, top_k: int = 5):
        return self.index.search_with_embedding(query_emb, top_k=top_k)


__all__ = ["FinderIndex"]
