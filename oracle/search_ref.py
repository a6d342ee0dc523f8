"""ORACLE -- test infrastructure only. Never imported by the product path.

CPU restatement of the reference's cosine search:
  * TextSearchIndex.__init__ row re-normalisation  src/embedding/search.py:36,68
  * search_with_embedding: query normalise :93, sims = q @ E^T :96,
    topk(min(k, N), largest, sorted) :98-99
  * similarity.cosine_similarity / top_k_similar    src/embedding/similarity.py:10-58
  * SeekerService._build_query_embedding fusion      src/embedding/seeker_service.py:148-157
    (restated only: the service module imports its DB / YOLO stack, so this
    3-line rule is parity-unpinned by reference-produced vectors)
with the tie rule the build defines (score desc, index asc) -- CPU torch.topk
leaves exact ties unordered (SURVEY §7 hard part 2).

Pinned by tests/golden/search_gauss.npz and custom_index_top3.npz, produced by
the reference's own similarity.py (tests/golden/make_golden.py).
"""
from __future__ import annotations

import numpy as np


def normalize_rows(x: np.ndarray) -> np.ndarray:
    x = np.asarray(x, np.float32)
    return x / np.linalg.norm(x, axis=-1, keepdims=True)


def cosine_scores(q: np.ndarray, E: np.ndarray, dtype=np.float64) -> np.ndarray:
    """normalise(q) . normalise(E)^T computed in `dtype` (fp64 for tie analysis)."""
    q = np.atleast_2d(np.asarray(q, dtype))
    E = np.asarray(E, dtype)
    q = q / np.linalg.norm(q, axis=-1, keepdims=True)
    E = E / np.linalg.norm(E, axis=-1, keepdims=True)
    return q @ E.T


def fuse_query(text_emb, image_emb, w_text: float = 0.5, w_image: float = 0.5) -> np.ndarray:
    """seeker_service.py:148-157: one modality -> e / ||e||; both -> (w_t*t + w_i*i) / ||.||,
    fp32 products and sum as torch evaluates `sum(w * e for e, w in embs)` (0 + w_t*t + w_i*i)."""
    if text_emb is None and image_emb is None:
        raise ValueError("need a text or an image embedding")
    if text_emb is None or image_emb is None:
        e = np.asarray(text_emb if text_emb is not None else image_emb, np.float32)
        return (e / np.linalg.norm(e.astype(np.float64), axis=-1, keepdims=True)).astype(np.float32)
    t = np.asarray(text_emb, np.float32)
    i = np.asarray(image_emb, np.float32)
    v = (np.float32(w_text) * t) + (np.float32(w_image) * i)
    return (v / np.linalg.norm(v.astype(np.float64), axis=-1, keepdims=True)).astype(np.float32)


def topk(scores: np.ndarray, k: int):
    """Row-wise top-k by (score desc, index asc) -> (values, indices)."""
    scores = np.atleast_2d(scores)
    n = scores.shape[1]
    k = min(k, n)
    idx = np.lexsort((np.broadcast_to(np.arange(n), scores.shape), -scores), axis=-1)[:, :k]
    return np.take_along_axis(scores, idx, axis=-1), idx


def search(q: np.ndarray, E: np.ndarray, k: int):
    return topk(cosine_scores(q, E), k)


def same_topk_up_to_ties(idx_a: np.ndarray, idx_b: np.ndarray, exact_scores: np.ndarray, eps: float) -> bool:
    """True if two top-k index lists of one query agree, except where the exact
    (fp64) scores of the differing entries are within eps of each other (near-ties
    that fp32 summation order may legitimately swap)."""
    idx_a = np.asarray(idx_a)
    idx_b = np.asarray(idx_b)
    if np.array_equal(idx_a, idx_b):
        return True
    sa = exact_scores[idx_a]
    sb = exact_scores[idx_b]
    # position-wise the scores must agree within eps, and the sets may differ only
    # in elements whose score is within eps of the boundary
    if np.max(np.abs(sa - sb)) > eps:
        return False
    diff = set(idx_a.tolist()) ^ set(idx_b.tolist())
    if not diff:
        return True
    boundary = min(sa[-1], sb[-1])
    return all(abs(exact_scores[i] - boundary) <= eps for i in diff)
