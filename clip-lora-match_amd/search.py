"""Drop-in for src/embedding/search.py: SearchResult + TextSearchIndex, backed by
an HBM-resident fp16 index (libclm clm_index_*) and the gfx950 cosine GEMM +
exact top-k kernels.

  SearchResult                       search.py:14-20
  TextSearchIndex.__init__           search.py:24-68  (key variants :41-56, re-normalise :68)
  .search_with_embedding             search.py:70-115 (shape checks :80-90, safe metadata :103-105)
  .search_by_text / .search_by_image search.py:117-151
New: .append / .save keep the index resident with amortised
O(1) append instead of FinderService's torch.cat + full re-save per report
(finder_service.py:93-103,172-185; the report flow itself is finder.py), and
.search_batch serves many queries per launch. .save_shard / .load_shard persist the HBM
index itself (SURVEY §5 checkpoint row): a raw shard of the fp16 MFMA operands, their fp32
inverse norms and the fp32 rows, streamed back to HBM without re-normalising or re-rounding
anything (the .pt reload of search.py:29-36,68 costs torch.load + an fp32 normalise of every
row + the fp16 rounding), bit-identical in search.

Scores are the exact cosines of the stored fp32 rows (fp64 arithmetic, rounded
once): the fp16 MFMA pass only bounds the candidates (clm_index_search). Top-k
order is (score desc, index asc); CPU torch.topk leaves exact ties in arbitrary
order (SURVEY §7 hard part 2).
"""
from __future__ import annotations

import ctypes
import json
import struct
from dataclasses import dataclass
from pathlib import Path
from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from . import _capi as C


@dataclass
class SearchResult:
    """Satu hasil pencarian."""
    index: int
    score: float
    image_path: str
    text: str


def _pad_dim(x: torch.Tensor, dim_p: int) -> torch.Tensor:
    if x.shape[-1] == dim_p:
        return x
    return torch.nn.functional.pad(x, (0, dim_p - x.shape[-1]))


class CosineIndex:
    """GPU index of fp16 rows + fp32 inverse norms (score = q.row / (|q| |row|))."""

    def __init__(self, dim: int, capacity: int = 1024, device=None):
        C.require_gpu()
        self.dim = int(dim)
        self.dim_p = (self.dim + 63) // 64 * 64          # GEMM K granule; zero padding keeps dots/norms
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None
                                   else (torch.device(device).index or 0))
        h = ctypes.c_void_p()
        C.check(C.lib().clm_index_create(self.device.index, max(int(capacity), 1), self.dim_p, ctypes.byref(h)),
                "clm_index_create")
        self._h = h

    def __len__(self) -> int:
        return int(C.lib().clm_index_size(self._h))

    def append(self, rows) -> None:
        t = torch.as_tensor(rows)
        if t.dim() == 1:
            t = t.unsqueeze(0)
        if t.dim() != 2 or t.shape[1] != self.dim:
            raise ValueError(f"rows must be [n, {self.dim}], got {tuple(t.shape)}")
        if t.dtype not in (torch.float32, torch.float16):
            t = t.float()
        t = _pad_dim(t.to(self.device), self.dim_p).contiguous()
        code = C.CLM_F32 if t.dtype == torch.float32 else C.CLM_F16
        C.check(C.lib().clm_index_append(self._h, C.ptr(t), code, t.shape[0], C.stream_of(self.device)),
                "clm_index_append")

    def reset(self) -> None:
        C.check(C.lib().clm_index_reset(self._h))

    def set_offset(self, offset: int) -> None:
        C.check(C.lib().clm_index_set_offset(self._h, int(offset)))

    def read(self, start: int = 0, n: Optional[int] = None) -> torch.Tensor:
        n = len(self) - start if n is None else n
        out = torch.empty((n, self.dim_p), dtype=torch.float32)
        C.check(C.lib().clm_index_read(self._h, start, n, C.ptr(out), C.stream_of(self.device)), "clm_index_read")
        return out[:, :self.dim]

    def search(self, queries, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
        """queries [nq, dim] (f32/f16, any device) -> (scores [nq,k] f32, idx [nq,k] i64) on the GPU."""
        q = torch.as_tensor(queries)
        if q.dim() == 1:
            q = q.unsqueeze(0)
        if q.dim() != 2 or q.shape[1] != self.dim:
            raise ValueError(f"queries must be [nq, {self.dim}], got {tuple(q.shape)}")
        if q.dtype not in (torch.float32, torch.float16):
            q = q.float()
        q = _pad_dim(q.to(self.device), self.dim_p).contiguous()
        nq = q.shape[0]
        s = torch.empty((nq, k), dtype=torch.float32, device=self.device)
        i = torch.empty((nq, k), dtype=torch.int64, device=self.device)
        code = C.CLM_F32 if q.dtype == torch.float32 else C.CLM_F16
        C.check(C.lib().clm_index_search(self._h, C.ptr(q), code, nq, int(k), C.ptr(s), C.ptr(i),
                                         C.stream_of(self.device)), "clm_index_search")
        return s, i

    # ------------------------------------------------------------ shard file --
    def save_shard(self, path: Union[str, Path], meta: Optional[dict] = None, chunk_rows: int = 1 << 20) -> None:
        """Write the index's internal state (fp16 operands, fp32 inverse norms, the fp32 rows if
        kept) to a shard file (format: _SHARD_MAGIC, u64 header length, JSON header, then the
        sections at 4 KiB boundaries), streamed through a pinned host buffer; atomic rename."""
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        n = len(self)
        has32 = int(C.lib().clm_index_has_f32(self._h)) == 1
        header = {"format": "clm-index-shard", "version": 1, "dim": self.dim, "dim_p": self.dim_p, "n": n,
                  "has_f32": has32, "meta": meta or {}}
        hb = json.dumps(header).encode()
        tmp = path.with_name(path.name + ".tmp")
        chunk = max(1, min(int(chunk_rows), max(n, 1)))
        b16 = torch.empty((chunk, self.dim_p), dtype=torch.float16, pin_memory=True)
        binv = torch.empty((chunk,), dtype=torch.float32, pin_memory=True)
        b32 = torch.empty((chunk, self.dim_p), dtype=torch.float32, pin_memory=True) if has32 else None
        secs = _shard_sections(len(hb), n, self.dim_p, has32)
        with open(tmp, "wb") as f:
            f.write(_SHARD_MAGIC + struct.pack("<Q", len(hb)) + hb)
            for r0 in range(0, n, chunk):
                m = min(chunk, n - r0)
                C.check(C.lib().clm_index_export(self._h, r0, m, C.ptr(b16), C.ptr(binv),
                                                 C.ptr(b32) if b32 is not None else None,
                                                 C.stream_of(self.device)), "clm_index_export")
                for name, buf in (("rows16", b16), ("inv", binv), ("rows32", b32)):
                    if buf is None:
                        continue
                    f.seek(secs[name][0] + r0 * buf[0].numel() * buf.element_size())
                    f.write(memoryview(buf[:m].numpy()).cast("B"))
            f.truncate(_shard_size(secs))
        tmp.replace(path)

    @classmethod
    def load_shard(cls, path: Union[str, Path], device=None, capacity: Optional[int] = None,
                   chunk_rows: int = 1 << 20) -> Tuple["CosineIndex", dict]:
        """(index, header) from a shard file: the sections are read chunk by chunk into a pinned
        buffer and imported into HBM as they are (clm_index_import)."""
        path = Path(path)
        if not path.exists():
            raise FileNotFoundError(f"Index shard not found: {path}")
        header, secs = read_shard_header(path)
        n, dim_p = header["n"], header["dim_p"]
        idx = cls(header["dim"], capacity=max(capacity or n, 1), device=device)
        if idx.dim_p != dim_p:
            raise ValueError(f"shard dim_p {dim_p} does not match dim {header['dim']}")
        chunk = max(1, min(int(chunk_rows), max(n, 1)))
        b16 = torch.empty((chunk, dim_p), dtype=torch.float16, pin_memory=True)
        binv = torch.empty((chunk,), dtype=torch.float32, pin_memory=True)
        b32 = torch.empty((chunk, dim_p), dtype=torch.float32, pin_memory=True) if header["has_f32"] else None
        with open(path, "rb", buffering=0) as f:
            for r0 in range(0, n, chunk):
                m = min(chunk, n - r0)
                for name, buf in (("rows16", b16), ("inv", binv), ("rows32", b32)):
                    if buf is None:
                        continue
                    row_bytes = buf[0].numel() * buf.element_size()
                    f.seek(secs[name][0] + r0 * row_bytes)
                    view = memoryview(buf.numpy()).cast("B")[: m * row_bytes]
                    if f.readinto(view) != m * row_bytes:
                        raise ValueError(f"truncated index shard {path} (section {name})")
                d16 = b16[:m].to(idx.device, non_blocking=True)
                dinv = binv[:m].to(idx.device, non_blocking=True)
                d32 = b32[:m].to(idx.device, non_blocking=True) if b32 is not None else None
                C.check(C.lib().clm_index_import(idx._h, C.ptr(d16), C.ptr(dinv), C.ptr(d32) if d32 is not None else None,
                                                 m, C.stream_of(idx.device)), "clm_index_import")
        return idx, header

    def stats(self) -> dict:
        """queries served by the sampled single-pass bounded search (`filtered`), the bounded
        search with a chunked fp16 scan as its first step (`scan_bounded`), the full exact
        scan (`full_exact`), their sum `exact`, overflow re-runs, and the queries whose filter
        pass ran on the G2 256 x 192 tiles (`filter_g2`) or, in blocks whose sampled candidate
        windows mostly exceed the list capacity, on gemm_kernel 256 x 256 (`filter_dense`)
        (include/clm.h), and the small batches (nq <= 16) served by the one-pass streaming search
        (`small_scan`)"""
        v = (ctypes.c_int64 * 7)()
        C.check(C.lib().clm_index_stats2(self._h, v, 7))
        return {"filtered": v[0], "scan_bounded": v[1], "full_exact": v[2], "exact": v[1] + v[2],
                "overflow": v[3], "filter_g2": v[4], "filter_dense": v[5], "small_scan": v[6]}

    def close(self) -> None:
        if getattr(self, "_h", None):
            C.lib().clm_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_SHARD_MAGIC = b"CLMIDX01"


def _shard_sections(header_len: int, n: int, dim_p: int, has32: bool) -> dict:
    """byte offset and length of each section, every one at a 4 KiB boundary"""
    def up(x):
        return (x + 4095) // 4096 * 4096
    off = up(len(_SHARD_MAGIC) + 8 + header_len)
    secs = {}
    for name, nbytes in (("rows16", n * dim_p * 2), ("inv", n * 4), ("rows32", n * dim_p * 4 if has32 else 0)):
        if nbytes or name != "rows32":
            secs[name] = (off, nbytes)
            off = up(off + nbytes)
    return secs


def _shard_size(secs: dict) -> int:
    return max(o + b for o, b in secs.values())


def read_shard_header(path: Union[str, Path]) -> Tuple[dict, dict]:
    """(header, sections) of a shard file; ValueError if it is not one"""
    with open(path, "rb") as f:
        magic = f.read(len(_SHARD_MAGIC))
        if magic != _SHARD_MAGIC:
            raise ValueError(f"{path} is not a clm index shard")
        (hl,) = struct.unpack("<Q", f.read(8))
        header = json.loads(f.read(hl).decode())
    if header.get("format") != "clm-index-shard" or header.get("version") != 1:
        raise ValueError(f"{path}: unsupported shard header {header.get('format')} v{header.get('version')}")
    secs = _shard_sections(hl, header["n"], header["dim_p"], header["has_f32"])
    if Path(path).stat().st_size < _shard_size(secs):
        raise ValueError(f"truncated index shard {path}")
    return header, secs


class TextSearchIndex:
    def __init__(self, index_path: Union[str, Path, None] = None, *, embeddings=None, image_paths=None,
                 texts=None, device=None):
        if index_path is not None:
            index_path = Path(index_path)
            if not index_path.exists():
                raise FileNotFoundError(f"Index file not found: {index_path}")
            obj = torch.load(index_path, map_location="cpu", weights_only=True)
        else:
            obj = {"embeddings": embeddings, "image_paths": image_paths, "texts": texts}

        embs = obj.get("embeddings")
        if embs is None:
            raise ValueError("Index file does not contain 'embeddings'")
        self.embeddings: torch.Tensor = torch.as_tensor(embs).float().cpu()
        if self.embeddings.dim() == 1:
            self.embeddings = self.embeddings.unsqueeze(0)

        images = obj.get("image_paths")
        if images is None:
            images = obj.get("image_path")
        if images is None:
            images = []
        self.image_paths: list = list(images)

        texts_ = obj.get("texts")
        if texts_ is None:
            texts_ = obj.get("text")
        if texts_ is None:
            texts_ = []
        self.texts: list = list(texts_)

        if self.embeddings.size(0) != len(self.image_paths):
            print(f"[TextSearchIndex] WARNING: embeddings rows ({self.embeddings.size(0)}) "
                  f"!= len(image_paths) ({len(self.image_paths)})")

        self.num_items, self.dim = self.embeddings.shape
        print(f"[TextSearchIndex] Loaded {self.num_items} items with dim={self.dim}")

        # Pastikan normalized (search.py:68) -- fp32 on the host, as the reference does; the GPU
        # index keeps these fp32 rows for its exact re-score
        self.embeddings = self.embeddings / self.embeddings.norm(dim=-1, keepdim=True)
        self._gpu = CosineIndex(self.dim, capacity=max(self.num_items, 1024), device=device)
        if self.num_items:
            self._gpu.append(self.embeddings)

    @classmethod
    def from_gpu_index(cls, index: "CosineIndex", image_paths: Sequence[str] = (),
                       texts: Sequence[str] = ()) -> "TextSearchIndex":
        """Wrap an HBM-resident CosineIndex (e.g. one built by index_build or load_shard) as a
        TextSearchIndex without a host copy of its rows: searches go straight to the GPU index;
        the host mirror (`embeddings`, used by save / append) is read back from HBM on first use."""
        self = cls.__new__(cls)
        self._gpu = index
        n = len(index)
        self._host, self._n = None, n
        self.num_items, self.dim = n, index.dim
        self.image_paths, self.texts = list(image_paths), list(texts)
        return self

    # host mirror of the rows: a capacity-doubling buffer, so append is amortised O(1) (the
    # reference's FinderService torch.cat's the whole index per report, finder_service.py:180)
    @property
    def embeddings(self) -> torch.Tensor:
        if self._host is None:   # from_gpu_index: the rows as the index keeps them, fetched once
            self._host = self._gpu.read(0, self._n).float()[:, : self.dim].contiguous()
        return self._host[: self._n]

    @embeddings.setter
    def embeddings(self, value) -> None:
        t = torch.as_tensor(value).float().cpu()
        self._host = t.contiguous() if t.dim() == 2 else t
        self._n = self._host.shape[0] if self._host.dim() >= 1 else 0

    # --------------------------------------------------------------- search --
    def search_batch(self, queries, top_k: int = 5) -> Tuple[torch.Tensor, torch.Tensor]:
        """[nq, d] queries -> (scores [nq, k], indices [nq, k]) on the GPU, k = min(top_k, num_items)."""
        k = min(int(top_k), self.num_items)
        if k < 0:
            raise RuntimeError("selected index k out of range")
        if k == 0:
            q = torch.as_tensor(queries)
            nq = 1 if q.dim() == 1 else q.shape[0]
            return torch.empty((nq, 0)), torch.empty((nq, 0), dtype=torch.int64)
        return self._gpu.search(queries, k)

    def search_with_embedding(self, query_emb: torch.Tensor, top_k: int = 5) -> List[SearchResult]:
        """query_emb: shape (d,) atau (1, d)."""
        query_emb = torch.as_tensor(query_emb)
        if query_emb.ndim == 1:
            query_emb = query_emb.unsqueeze(0)
        elif query_emb.ndim != 2 or query_emb.shape[0] != 1:
            raise ValueError(f"query_emb must be shape (d,) or (1, d), got {tuple(query_emb.shape)}")
        if query_emb.shape[-1] != self.dim:
            raise ValueError(f"query_emb dim {query_emb.shape[-1]} != index dim {self.dim}")
        scores, indices = self.search_batch(query_emb, top_k)
        results: List[SearchResult] = []
        for idx, score in zip(indices[0].tolist(), scores[0].tolist()):
            img = self.image_paths[idx] if idx < len(self.image_paths) else ""
            txt = self.texts[idx] if idx < len(self.texts) else ""
            results.append(SearchResult(index=idx, score=float(score), image_path=img, text=txt))
        return results

    def search_by_text(self, query, model, processor, device, top_k: int = 5) -> List[SearchResult]:
        from .clip_model import encode_text
        return self.search_with_embedding(encode_text(query, model, processor, device), top_k=top_k)

    def search_by_image(self, image_path, model, processor, device, top_k: int = 5) -> List[SearchResult]:
        from .clip_model import encode_image
        return self.search_with_embedding(encode_image(image_path, model, processor, device), top_k=top_k)

    # ------------------------------------------------------- resident append --
    def append(self, embeddings, image_paths: Sequence[str] = (), texts: Sequence[str] = ()) -> None:
        """Add rows (re-normalised in fp32, as finder_service.py:169 does) and their metadata:
        amortised O(1) per row on the host and in HBM."""
        e = torch.as_tensor(embeddings).float().cpu()
        if e.dim() == 1:
            e = e.unsqueeze(0)
        if e.dim() != 2 or e.shape[1] != self.dim:
            raise ValueError(f"embedding dim {e.shape[-1]} != index dim {self.dim}")
        e = e / e.norm(dim=-1, keepdim=True)
        if self._host is None:
            self.embeddings   # noqa: B018 -- materialise the host mirror before growing it
        n_new = self._n + e.shape[0]
        if n_new > self._host.shape[0]:
            cap = max(n_new, 2 * self._host.shape[0], 1024)
            buf = torch.empty((cap, self.dim), dtype=torch.float32)
            buf[: self._n] = self._host[: self._n]
            self._host = buf
        self._host[self._n: n_new] = e
        self._gpu.append(e)
        self._n = n_new
        self.image_paths.extend(image_paths)
        self.texts.extend(texts)
        self.num_items = n_new

    def save(self, path: Union[str, Path]) -> None:
        """The reference .pt format ({"embeddings": [N, D] f32, "image_paths", "texts"},
        finder_service.py:93-103), written to a temporary file and renamed into place."""
        path = Path(path)
        path.parent.mkdir(parents=True, exist_ok=True)
        tmp = path.with_name(path.name + ".tmp")
        torch.save({"embeddings": self.embeddings.clone(), "image_paths": list(self.image_paths),
                    "texts": list(self.texts)}, tmp)
        tmp.replace(path)

    # ------------------------------------------------------------ shard file --
    def save_shard(self, path: Union[str, Path]) -> None:
        """The HBM index as a raw shard (CosineIndex.save_shard) with this index's metadata; the
        reference .pt stays available through .save."""
        self._gpu.save_shard(path, meta={"image_paths": [str(p) for p in self.image_paths],
                                         "texts": [str(t) for t in self.texts]})

    @classmethod
    def load_shard(cls, path: Union[str, Path], device=None) -> "TextSearchIndex":
        """Reload a save_shard file straight into HBM (no torch.load, no re-normalisation): the
        same rows, metadata and search results, bit for bit, as the index that was saved."""
        gpu, header = CosineIndex.load_shard(path, device=device, capacity=max(header_n(path), 1024))
        self = cls.__new__(cls)
        n, dim, dim_p = header["n"], header["dim"], header["dim_p"]
        _, secs = read_shard_header(path)
        if n == 0:   # an empty index has no data sections to map (mmap refuses 0 bytes at EOF)
            host = torch.empty((0, dim), dtype=torch.float32)
        else:
            if header["has_f32"]:   # the host mirror: the fp32 rows, paged in lazily (copy-on-write map)
                host = np.memmap(path, dtype=np.float32, mode="c", offset=secs["rows32"][0], shape=(n, dim_p))
            else:
                host = np.memmap(path, dtype=np.float16, mode="r", offset=secs["rows16"][0], shape=(n, dim_p))
            host = torch.from_numpy(np.ascontiguousarray(host[:, :dim]) if dim != dim_p or not header["has_f32"]
                                    else host).float()
        self._host, self._n = host, n
        self.image_paths = list(header["meta"].get("image_paths", []))
        self.texts = list(header["meta"].get("texts", []))
        self.num_items, self.dim = n, dim
        self._gpu = gpu
        print(f"[TextSearchIndex] Loaded {n} items with dim={dim} (shard)")
        return self


def header_n(path) -> int:
    return read_shard_header(path)[0]["n"]
