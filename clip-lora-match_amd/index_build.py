"""Index build: scripts/rebuild_index.py:28-115 on the gfx950 encode path, batched and
optionally sharded over the GPUs of one node.

The reference encodes each item's description one at a time (:64-77: encode_text, then
a second `/ norm`), concatenates the rows and writes
{"embeddings": [N, D] f32, "image_paths": [...], "texts": [...]} with torch.save (:86-93).
Here one call encodes `batch_size` captions (or images) per launch sequence, the rows
stay on the device until the save, and under torch.distributed each rank encodes its
shard_range of the items and one all_gather assembles the index in item order
(distributed.build_index_sharded). The file format is the reference's, so
TextSearchIndex (ours or the reference's) loads it unchanged.

The database query (:46-52) is the caller's: pass the items' descriptions / image paths.
"""
from __future__ import annotations

from pathlib import Path
from typing import Optional, Sequence, Union

import torch
import torch.distributed as dist

from . import _capi as C


def _renormalize(rows: torch.Tensor) -> torch.Tensor:
    """The reference's second `text_emb / text_emb.norm(...)` (rebuild_index.py:72), on the device."""
    rows = rows.float().contiguous()
    if rows.shape[0]:
        C.check(C.lib().clm_l2_normalize(rows.device.index, C.ptr(rows), rows.shape[0], rows.shape[1],
                                         C.stream_of(rows.device)), "clm_l2_normalize")
    return rows


def encode_items(model, processor, texts: Optional[Sequence] = None, images=None,
                 batch_size: int = 256, group=None) -> torch.Tensor:
    """[N, D] f32 unit rows on the model's device, in item order, for N captions (str or token ids)
    or N images. Images: a sequence of paths / PIL images / uint8 arrays (decoded on the host,
    resized on the GPU), a uint8 tensor [N, S, S, 3] (host or device), or a source with len() and
    batch(start, stop) -> uint8 device tensor (e.g. synthetic.DeviceImages). Sharded over the
    ranks of `group` when torch.distributed is up."""
    if (texts is None) == (images is None):
        raise ValueError("pass exactly one of texts / images")
    pixel_source = images is not None and (hasattr(images, "batch") or isinstance(images, torch.Tensor))
    items = images if pixel_source else list(texts if texts is not None else images)
    n = len(items)
    D = model.cfg.proj_dim

    def encode_rows(start: int, stop: int) -> torch.Tensor:
        if stop <= start:
            return torch.empty((0, D), dtype=torch.float32, device=model.device)
        if pixel_source:
            px = items.batch(start, stop) if hasattr(items, "batch") else items[start:stop]
            return _renormalize(model.encode_pixels(px.to(model.device), normalize=True))
        chunk = items[start:stop]
        if texts is not None:
            ids = processor.token_ids(chunk)
            out = model.encode_ids(ids.to(model.device), normalize=True)
        else:
            from .clip_model import _encode_images
            out = _encode_images(chunk, model, processor, normalize=True)
        return _renormalize(out)

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        from .distributed import build_index_sharded
        return build_index_sharded(encode_rows, n, batch_size, group)
    outs = [encode_rows(s, min(s + batch_size, n)) for s in range(0, n, batch_size)]
    return torch.cat(outs, 0) if outs else encode_rows(0, 0)


def _save_index(rows: torch.Tensor, descriptions: Sequence, image_paths: Sequence, index_path) -> None:
    """torch.save in the reference's format (rebuild_index.py:86-93), to a temporary name renamed
    into place so readers never see a partial file."""
    index_path = Path(index_path)
    index_path.parent.mkdir(parents=True, exist_ok=True)
    texts = [d if isinstance(d, str) else "" for d in descriptions]
    tmp = index_path.with_name(index_path.name + ".tmp")
    torch.save({"embeddings": rows, "image_paths": [str(p) for p in image_paths], "texts": texts}, tmp)
    tmp.replace(index_path)


def rebuild_index(model, processor, descriptions: Sequence, image_paths: Sequence[str],
                  index_path: Union[str, Path], batch_size: int = 256, from_images: bool = False,
                  group=None, images=None) -> torch.Tensor:
    """rebuild_index.py:28-115: embed every item (its description by default, as the reference
    does; its image with from_images=True -- the files at image_paths, or `images`: any image
    source encode_items takes, e.g. pixels already on the device), save the .pt index, return the
    [N, D] CPU rows. Under torch.distributed only rank 0 writes the file (to a temporary name,
    renamed into place); its outcome is broadcast, so every rank returns after the file exists or
    raises if rank 0's write failed (no rank is left waiting). No items: nothing is written (:54-56)."""
    if len(descriptions) != len(image_paths):
        raise ValueError(f"{len(descriptions)} descriptions vs {len(image_paths)} image paths")
    if images is not None and len(images) != len(image_paths):
        raise ValueError(f"{len(images)} images vs {len(image_paths)} image paths")
    if len(descriptions) == 0:
        return torch.empty((0, model.cfg.proj_dim), dtype=torch.float32)
    if from_images:
        src = images if images is not None else list(image_paths)
        rows = encode_items(model, processor, images=src, batch_size=batch_size, group=group)
    else:
        rows = encode_items(model, processor, texts=list(descriptions), batch_size=batch_size, group=group)
    rows = rows.cpu()
    distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    err = None
    if not distributed or dist.get_rank(group) == 0:
        try:
            _save_index(rows, descriptions, image_paths, index_path)
        except Exception as e:   # re-raised below on every rank
            if not distributed:
                raise
            err = f"rank 0 failed to write {index_path}: {e!r}"
    if distributed:
        status = [err]
        dist.broadcast_object_list(status, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                   group=group)
        if status[0] is not None:
            raise RuntimeError(status[0])
    return rows


__all__ = ["encode_items", "rebuild_index"]
