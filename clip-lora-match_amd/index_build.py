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


EXCHANGES = ("fp32", "fp16")


def _f16_exchange(rows: torch.Tensor) -> torch.Tensor:
    """Unit fp32 rows -> fp16 (RNE): the form the rows cross the links in with exchange="fp16"."""
    return rows.to(torch.float16)


def _f16_restore(rows: torch.Tensor) -> torch.Tensor:
    """fp16 rows -> fp32, re-normalised (clm_l2_normalize): the rows every rank keeps."""
    return _renormalize(rows.float())


def fold_sha256(rows: torch.Tensor) -> str:
    """Checksum of checksums of an [N, D] fp32 index: a column-weighted fold of each row's bits
    (sum_j bits[i, j] * (2j + 1), int64, on the rows' device), then sha256 of the N folds (first 16
    hex digits). Equal for two indexes iff (with overwhelming probability) every row is bit-equal;
    compared across world sizes by the bench and tests (configs[2])."""
    import hashlib
    bits = rows.contiguous().view(torch.int32).to(torch.int64)
    fold = (bits * (torch.arange(bits.shape[1], device=bits.device, dtype=torch.int64) * 2 + 1)).sum(1)
    return hashlib.sha256(fold.cpu().numpy().tobytes()).hexdigest()[:16]


def encode_items(model, processor, texts: Optional[Sequence] = None, images=None,
                 batch_size: int = 256, group=None, exchange: str = "fp32") -> torch.Tensor:
    """[N, D] f32 unit rows on the model's device, in item order, for N captions (str or token ids)
    or N images. Images: a sequence of paths / PIL images / uint8 arrays (decoded on the host,
    resized on the GPU), a uint8 tensor [N, S, S, 3] (host or device), or a source with len() and
    batch(start, stop) -> uint8 device tensor (e.g. synthetic.DeviceImages). Sharded over the
    ranks of `group` when torch.distributed is up.

    exchange: "fp32" (default) gathers the fp32 rows as encoded (4 B per value over the links);
    "fp16" gathers them rounded to fp16 and re-normalises the gathered rows in fp32 (half the
    all_gather bytes: 1.02 GB instead of 2.05 GB for 1 M x 512). The fp16 round trip is applied at
    every world size, world 1 included, so the rows do not depend on the number of ranks; it moves
    a unit row by at most ~2^-12 relative per component (cosines by < 5e-4), inside the path's 1e-3
    score bar, and is not the reference's fp32 .pt content -- hence opt-in."""
    if exchange not in EXCHANGES:
        raise ValueError(f"exchange must be one of {EXCHANGES}, got {exchange!r}")
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

    f16 = exchange == "fp16"
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        from .distributed import build_index_sharded
        return build_index_sharded(encode_rows, n, batch_size, group, exchange=_f16_exchange if f16 else None,
                                   restore=_f16_restore if f16 else None)
    outs = [encode_rows(s, min(s + batch_size, n)) for s in range(0, n, batch_size)]
    rows = torch.cat(outs, 0) if outs else encode_rows(0, 0)
    return _f16_restore(_f16_exchange(rows)) if f16 else rows


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
                  group=None, images=None, exchange: str = "fp32",
                  host_rows: bool = True) -> torch.Tensor:
    """rebuild_index.py:28-115: embed every item (its description by default, as the reference
    does; its image with from_images=True -- the files at image_paths, or `images`: any image
    source encode_items takes, e.g. pixels already on the device), save the .pt index, return the
    [N, D] rows. Under torch.distributed only rank 0 writes the file (to a temporary name,
    renamed into place); its outcome is broadcast, so every rank returns after the file exists or
    raises if rank 0's write failed (no rank is left waiting). No items: nothing is written (:54-56).

    Every rank returns the CPU rows by default (host_rows=True, the reference's return type);
    host_rows=False returns the gathered rows on each rank's device instead, so only the writing
    process copies them to the host (2 GB of D2H per rank saved at 1 M rows). exchange: see
    encode_items."""
    if len(descriptions) != len(image_paths):
        raise ValueError(f"{len(descriptions)} descriptions vs {len(image_paths)} image paths")
    if images is not None and len(images) != len(image_paths):
        raise ValueError(f"{len(images)} images vs {len(image_paths)} image paths")
    if len(descriptions) == 0:
        return torch.empty((0, model.cfg.proj_dim), dtype=torch.float32)
    if from_images:
        src = images if images is not None else list(image_paths)
        rows = encode_items(model, processor, images=src, batch_size=batch_size, group=group, exchange=exchange)
    else:
        rows = encode_items(model, processor, texts=list(descriptions), batch_size=batch_size, group=group,
                            exchange=exchange)
    distributed = dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    writer = not distributed or dist.get_rank(group) == 0
    dev_rows = rows
    if writer:
        rows = rows.cpu()
    err = None
    if writer:
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
    if host_rows:
        return rows if writer else dev_rows.cpu()
    return dev_rows


__all__ = ["encode_items", "rebuild_index", "fold_sha256"]
