"""GPU parity of the cosine top-k search (through the C-ABI) against the
reference's own similarity.top_k_similar goldens and the CPU oracle.

Bar: top-k indices identical to the reference except inside near-tie groups
whose exact (fp64) scores differ by < 2e-6 (fp32 summation order can swap
those; DESIGN.md §Search parity); scores within 1e-5 (fp16-representable
inputs) / 1e-3 (fp32 inputs rounded to fp16 operands).
"""
import numpy as np
import pytest
import torch

from conftest import GOLDEN, golden

from clip_lora_match_amd import synthetic as syn
from clip_lora_match_amd.search import CosineIndex, TextSearchIndex
from clip_lora_match_amd.similarity import cosine_similarity, top_k_similar
from oracle import search_ref as S

pytestmark = pytest.mark.gpu
EPS_TIE = 2e-6


def _agree(gi, ri, exact, eps=EPS_TIE):
    for q in range(gi.shape[0]):
        assert S.same_topk_up_to_ties(gi[q], ri[q], exact[q], eps), (q, gi[q], ri[q])


@pytest.mark.parametrize("k", [1, 5, 10, 50])
def test_index_vs_reference_golden(k):
    g = golden("search_gauss.npz")
    rows = syn.gaussian_rows(int(g["n"]), int(g["dim"]), int(g["row_seed"]))
    qs = syn.gaussian_rows(int(g["nq"]), int(g["dim"]), int(g["q_seed"]))
    idx = CosineIndex(int(g["dim"]))
    idx.append(torch.from_numpy(rows))
    s, i = idx.search(torch.from_numpy(qs), k)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    _agree(i, g[f"idx_k{k}"], exact)
    assert np.max(np.abs(s - g[f"vals_k{k}"])) < 1e-5
    # our order is exactly (score desc, index asc) on the exact scores, up to ties
    _, oi = S.topk(exact, k)
    _agree(i, oi, exact)


def test_multi_chunk_and_fp32_queries():
    """N > one score chunk (exercise the chunk merge), fp32 queries, k at the limit."""
    n, dim, nq = 300_000, 512, 8
    rows = syn.gaussian_rows(n, dim, 17)
    qs = syn.gaussian_rows(nq, dim, 18, fp16=False)
    idx = CosineIndex(dim, capacity=n)
    idx.append(torch.from_numpy(rows).cuda())
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    for k in (7, 1024):
        s, i = idx.search(torch.from_numpy(qs).cuda(), k)
        _, oi = S.topk(exact, k)
        # fp32 queries are rounded to fp16 operands: near-ties up to ~1e-4 may swap
        _agree(i.cpu().numpy(), oi, exact, eps=2e-4)
        assert np.max(np.abs(s.cpu().numpy() - np.take_along_axis(exact, oi, 1))) < 1e-3


def test_ties_are_index_ascending_and_k_beyond_n():
    dim = 128
    base = syn.gaussian_rows(4, dim, 3)
    rows = np.concatenate([base[[1, 0, 1, 2, 1, 3]]], 0)   # rows 0, 2, 4 identical
    idx = CosineIndex(dim)
    idx.append(torch.from_numpy(rows))
    s, i = idx.search(torch.from_numpy(base[1:2]), 10)
    i = i.cpu().numpy()[0]
    s = s.cpu().numpy()[0]
    assert list(i[:3]) == [0, 2, 4]
    assert list(i[6:]) == [-1] * 4 and np.all(np.isneginf(s[6:]))


def test_empty_index_and_offset():
    idx = CosineIndex(64)
    s, i = idx.search(torch.ones((2, 64)), 3)
    assert (i.cpu() == -1).all()
    rows = syn.gaussian_rows(100, 64, 4)
    idx.append(torch.from_numpy(rows))
    idx.set_offset(1000)
    _, i = idx.search(torch.from_numpy(rows[42:43]), 1)
    assert int(i[0, 0]) == 1042
    back = idx.read(40, 5).numpy()
    assert np.array_equal(back, rows[40:45].astype(np.float32))


def test_text_search_index_custom_golden(tmp_path):
    """The reference's committed index (.pt, plural keys): self-queries give the
    reference's top-3 ([[0,1,2],[1,2,0],[2,1,5],...], 0.828312 / 0.818218)."""
    g = golden("custom_index_top3.npz")
    ix = TextSearchIndex(f"{GOLDEN}/custom_items_index.pt")
    assert ix.num_items == 6 and ix.dim == 512 and len(ix.texts) == 6
    for q in range(6):
        res = ix.search_with_embedding(ix.embeddings[q], top_k=3)
        assert [r.index for r in res] == g["idx"][q].tolist()
        assert np.allclose([r.score for r in res], g["vals"][q], atol=1e-3)
        assert res[0].text == ix.texts[res[0].index]
    res = ix.search_with_embedding(ix.embeddings[2].unsqueeze(0), top_k=3)
    assert abs(res[1].score - 0.828312) < 1e-3 and abs(res[2].score - 0.818218) < 1e-3
    # k > N clamps to N (search.py:98); shape errors are ValueError (search.py:80-90)
    assert len(ix.search_with_embedding(ix.embeddings[0], top_k=50)) == 6
    with pytest.raises(ValueError):
        ix.search_with_embedding(torch.zeros(2, 512))
    with pytest.raises(ValueError):
        ix.search_with_embedding(torch.zeros(511))


def test_text_search_index_singular_keys_append_save(tmp_path):
    rows = syn.gaussian_rows(5, 512, 9, fp16=False)
    p = tmp_path / "idx.pt"
    torch.save({"embeddings": torch.from_numpy(rows), "image_path": ["a", "b", "c", "d", "e"],
                "text": ["ta", "tb", "tc", "td", "te"]}, p)
    ix = TextSearchIndex(p)
    assert ix.image_paths[3] == "d" and ix.texts[4] == "te"
    new = syn.gaussian_rows(1, 512, 10, fp16=False)
    ix.append(torch.from_numpy(new), ["f"], ["tf"])
    res = ix.search_with_embedding(torch.from_numpy(new[0]), top_k=1)
    assert res[0].index == 5 and res[0].image_path == "f"
    ix.save(tmp_path / "out.pt")
    ix2 = TextSearchIndex(tmp_path / "out.pt")
    assert ix2.num_items == 6 and ix2.texts[-1] == "tf"
    with pytest.raises(FileNotFoundError):
        TextSearchIndex(tmp_path / "missing.pt")
    torch.save({"foo": 1}, tmp_path / "bad.pt")
    with pytest.raises(ValueError):
        TextSearchIndex(tmp_path / "bad.pt")


def test_similarity_functions_vs_reference_golden():
    g = golden("search_gauss.npz")
    rows = syn.gaussian_rows(int(g["n"]), int(g["dim"]), int(g["row_seed"]))
    qs = syn.gaussian_rows(int(g["nq"]), int(g["dim"]), int(g["q_seed"]))
    E = torch.from_numpy(rows.astype(np.float32))
    cs = cosine_similarity(torch.from_numpy(qs[0].astype(np.float32)), E)
    assert cs.shape == (int(g["n"]),) and cs.device.type == "cpu"
    assert np.max(np.abs(cs.numpy() - g["cos_q0"])) < 1e-5
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    for q in range(8):
        v, i = top_k_similar(torch.from_numpy(qs[q].astype(np.float32)), E, 10)
        assert S.same_topk_up_to_ties(i.numpy(), g["idx_k10"][q], exact[q], EPS_TIE)
        assert np.max(np.abs(v.numpy() - g["vals_k10"][q])) < 1e-5


def test_large_index_property():
    """BASELINE-shaped property at 2M rows: a planted copy of each query is its top-1
    with score 1, and the rest of the list is sorted and within (-1, 1)."""
    n, dim, nq = 2_000_000, 512, 64
    g = torch.Generator(device="cuda").manual_seed(5)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    rows = (rows / rows.norm(dim=-1, keepdim=True)).half()
    plant = torch.randint(0, n, (nq,), generator=g, device="cuda")
    q = rows[plant].clone()
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows)
    s, i = idx.search(q, 16)
    assert torch.equal(i[:, 0], plant)
    assert torch.all(torch.abs(s[:, 0] - 1) < 1e-3)
    assert torch.all(s[:, 1:] <= s[:, :-1])


@pytest.mark.parametrize("k", [1, 5, 16, 48])
def test_filtered_path_equals_exact_path(k, monkeypatch):
    """The single-pass threshold-filter search returns exactly what the exact chunked path
    returns (same scores bit for bit, same indices), and reports which path served."""
    n, dim, nq = 1_000_000, 512, 96
    g = torch.Generator(device="cuda").manual_seed(k)
    rows = torch.randn((n, dim), generator=g, device="cuda").half()
    q = torch.randn((nq, dim), generator=g, device="cuda").half()
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows)
    s1, i1 = idx.search(q, k)
    st = idx.stats()
    assert st["filtered"] == nq and st["exact"] == 0
    monkeypatch.setenv("CLM_SEARCH_EXACT", "1")
    s2, i2 = idx.search(q, k)
    assert idx.stats()["exact"] == nq
    assert torch.equal(i1, i2) and torch.equal(s1, s2)
    monkeypatch.delenv("CLM_SEARCH_EXACT")
    idx.search(q, 256)                    # k*N/256 > N/4: sampling would not pay -> exact path
    assert idx.stats()["exact"] == 2 * nq


def test_filtered_path_overflow_falls_back():
    """300k identical rows make every one of them a candidate (> capacity): those queries
    are redone exactly and return the k smallest indices of the tie group."""
    n, dim = 1_000_000, 128
    g = torch.Generator(device="cuda").manual_seed(3)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    dup = torch.randn((dim,), generator=g, device="cuda")
    pos = torch.randperm(n, generator=g, device="cuda")[:300_000].sort().values
    rows[pos] = dup
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows.half())
    q = torch.stack([dup, torch.randn((dim,), generator=g, device="cuda")]).half()
    s, i = idx.search(q, 8)
    assert idx.stats()["overflow"] >= 1
    assert torch.equal(i[0], pos[:8])
    assert torch.all(s[0] > 0.999)
