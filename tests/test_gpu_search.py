"""GPU parity of the cosine top-k search (through the C-ABI) against the
reference's own similarity.top_k_similar goldens and the CPU oracle.

Bar: top-k indices identical to the reference except inside near-tie groups
whose exact (fp64) scores differ by < 2e-6 (the reference's fp32 summation order
can swap those; DESIGN.md §Search parity); scores within 1e-6 of the reference's
fp32 scores -- ours are the exact cosines of the stored fp32 rows rounded once, the
reference's carry its own fp32 summation error (~1e-7). This holds on fp32 data
that fp16 cannot represent (search_fp32.npz), because the fp16 MFMA pass only
bounds the candidates and they are re-scored exactly.
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
    assert np.max(np.abs(s - g[f"vals_k{k}"])) < 1e-6
    # our order is exactly (score desc, index asc) on the exact scores, up to ties
    _, oi = S.topk(exact, k)
    _agree(i, oi, exact)


def test_multi_chunk_and_fp32_queries():
    """N > one score chunk (exercise the chunk merge), fp32 queries, k at the limit: exact
    scores, exact order."""
    n, dim, nq = 300_000, 512, 8
    rows = syn.gaussian_rows(n, dim, 17)
    qs = syn.gaussian_rows(nq, dim, 18, fp16=False)
    idx = CosineIndex(dim, capacity=n)
    idx.append(torch.from_numpy(rows).cuda())
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    for k in (7, 1024):
        s, i = idx.search(torch.from_numpy(qs).cuda(), k)
        _, oi = S.topk(exact, k)
        _agree(i.cpu().numpy(), oi, exact)
        assert np.max(np.abs(s.cpu().numpy() - np.take_along_axis(exact, oi, 1))) < 1e-6


PATHS = {"full": {"CLM_SEARCH_FULL": "1"}, "bounded_scan": {"CLM_SEARCH_BOUNDED": "1", "CLM_SEARCH_EXACT": "1"},
         "bounded": {"CLM_SEARCH_BOUNDED": "1"}}


@pytest.mark.parametrize("path", sorted(PATHS))
@pytest.mark.parametrize("name", ["gauss", "clus"])
def test_fp32_rows_vs_reference_golden(name, path, monkeypatch):
    """fp32 rows and queries fp16 cannot represent, through every search path (full exact scan,
    fp16-scan-bounded + re-score, and the sampled bounded path where it applies) vs the
    reference's own top_k_similar: indices equal up to 2e-6 near-ties, scores within 1e-6.
    The clustered set's top-k scores lie 1e-5..1e-4 apart: fp16-rounded ranking alone would
    misorder them; the exact re-score does not."""
    g = golden("search_fp32.npz")
    gr, gq, cr, cq = syn.fp32_search_inputs()
    rows, qs = (gr, gq) if name == "gauss" else (cr, cq)
    for kv in PATHS[path].items():
        monkeypatch.setenv(*kv)
    idx = CosineIndex(512, capacity=rows.shape[0])
    idx.append(torch.from_numpy(rows))
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    for k in (1, 5, 10, 50):
        s, i = idx.search(torch.from_numpy(qs), k)
        s, i = s.cpu().numpy(), i.cpu().numpy()
        _agree(i, g[f"{name}_idx_k{k}"], exact)
        assert np.max(np.abs(s - g[f"{name}_vals_k{k}"])) < 1e-6
        _, oi = S.topk(exact, k)
        _agree(i, oi, exact)
    st = idx.stats()
    assert st["full_exact" if path == "full" else "scan_bounded" if path == "bounded_scan" else "exact"] > 0 \
        or st["filtered"] > 0


def test_all_paths_agree_bit_for_bit(monkeypatch):
    """The full exact scan, the fp16-scan-bounded search and the sampled bounded search return
    the same indices and the same scores bit for bit (one device routine scores every
    (query, row) pair), on fp32 rows with a fp32 copy kept for the re-score."""
    n, dim, nq = 1_200_000, 512, 40
    g = torch.Generator(device="cuda").manual_seed(11)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    q = torch.randn((nq, dim), generator=g, device="cuda")
    q[:8] = rows[torch.arange(8, device="cuda") * 1000] + 0.01 * q[:8]   # near-duplicates
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows)
    res = {}
    for path in ("full", "bounded_scan", "bounded"):
        for kv in PATHS[path].items():
            monkeypatch.setenv(*kv)
        res[path] = idx.search(q, 12)
        for kv in PATHS[path]:
            monkeypatch.delenv(kv)
    st = idx.stats()
    # every query on its intended path; on failure the message carries every path counter (a
    # round-5 scratch run once saw 7 of 40 sampled queries overflow here)
    assert st["full_exact"] == nq and st["scan_bounded"] == nq and st["filtered"] == nq, st
    for path in ("bounded_scan", "bounded"):
        assert torch.equal(res[path][1], res["full"][1]), path
        assert torch.equal(res[path][0], res["full"][0]), path
    assert torch.equal(res["full"][1][:8, 0], torch.arange(8, device="cuda") * 1000)
    back = idx.read(1000, 1)
    assert torch.equal(back.cuda()[0, :dim], rows[1000])   # the fp32 rows as given are kept


def test_sample_cache_invalidated_by_reset(monkeypatch):
    """clm_index_reset / append drop the threshold sample: refilling the same row count with
    different rows must not reuse the old rows' sample (a stale theta could drop true top-k)."""
    n, dim, nq = 1_000_000, 256, 32   # nq * n > 2^24: the bounded (sampled) search serves
    idx = CosineIndex(dim, capacity=n)
    for seed in (1, 2):
        g = torch.Generator(device="cuda").manual_seed(seed)
        rows = torch.randn((n, dim), generator=g, device="cuda").half()
        q = rows[:nq].float() + 0.05 * torch.randn((nq, dim), generator=g, device="cuda")
        idx.reset()
        idx.append(rows)
        s1, i1 = idx.search(q, 5)
        monkeypatch.setenv("CLM_SEARCH_FULL", "1")
        s2, i2 = idx.search(q, 5)
        monkeypatch.delenv("CLM_SEARCH_FULL")
        assert torch.equal(i1, i2) and torch.equal(s1, s2)
        assert torch.equal(i1[:, 0], torch.arange(nq, device="cuda"))
    assert idx.stats()["filtered"] == 2 * nq


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
        assert np.allclose([r.score for r in res], g["vals"][q], atol=1e-6, rtol=0)
        assert res[0].text == ix.texts[res[0].index]
    res = ix.search_with_embedding(ix.embeddings[2].unsqueeze(0), top_k=3)
    assert abs(res[1].score - 0.828312) < 1e-6 and abs(res[2].score - 0.818218) < 1e-6
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
    assert np.max(np.abs(cs.numpy() - g["cos_q0"])) < 1e-6
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    for q in range(8):
        v, i = top_k_similar(torch.from_numpy(qs[q].astype(np.float32)), E, 10)
        assert S.same_topk_up_to_ties(i.numpy(), g["idx_k10"][q], exact[q], EPS_TIE)
        assert np.max(np.abs(v.numpy() - g["vals_k10"][q])) < 1e-6
    # fp32 clustered rows (not fp16-representable), any dim: exact scores and order
    g2 = golden("search_fp32.npz")
    _, _, cr, cq = syn.fp32_search_inputs()
    cs = cosine_similarity(torch.from_numpy(cq[0]), torch.from_numpy(cr))
    assert np.max(np.abs(cs.numpy() - g2["clus_cos_q0"])) < 1e-6
    ex = S.cosine_scores(cq.astype(np.float64), cr.astype(np.float64))
    for q in range(0, 64, 9):
        v, i = top_k_similar(torch.from_numpy(cq[q]), torch.from_numpy(cr), 50)
        assert S.same_topk_up_to_ties(i.numpy(), g2["clus_idx_k50"][q], ex[q], EPS_TIE)
        assert np.max(np.abs(v.numpy() - g2["clus_vals_k50"][q])) < 1e-6
    odd = cosine_similarity(torch.from_numpy(cq[0, :100]), torch.from_numpy(cr[:, :100]))   # dim 100
    ref = S.cosine_scores(cq[:1, :100].astype(np.float64), cr[:, :100].astype(np.float64))[0]
    assert np.max(np.abs(odd.numpy() - ref)) < 1e-6


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
    assert torch.all(torch.abs(s[:, 0] - 1) < 1e-6)
    assert torch.all(s[:, 1:] <= s[:, :-1])


@pytest.mark.parametrize("k", [1, 5, 16, 48])
def test_filtered_path_equals_exact_path(k, monkeypatch):
    """The sampled single-pass bounded search returns exactly what the fp16-scan-bounded search
    returns (same exact scores bit for bit, same indices), and reports which path served."""
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


def test_filtered_path_overflow_falls_back(monkeypatch):
    """300k identical rows make every one of them a candidate (> capacity): those queries
    are redone exactly and return the k smallest indices of the tie group."""
    monkeypatch.setenv("CLM_SEARCH_BOUNDED", "1")   # 2 queries x 1M rows: small enough for the full scan
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


def test_many_overflowing_queries_one_exact_rescan(monkeypatch):
    """A block where most queries overflow their candidate lists (near-duplicate rows, like a
    finder index built from one description template): they are redone together by one exact
    scan and agree bit for bit with the full exact scan of every query."""
    monkeypatch.setenv("CLM_SEARCH_BOUNDED", "1")
    n, dim, k = 400_000, 128, 8
    g = torch.Generator(device="cuda").manual_seed(5)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    dups = torch.randn((3, dim), generator=g, device="cuda")
    for j in range(3):   # three tie groups of 60k rows each
        rows[j * 100_000: j * 100_000 + 60_000] = dups[j] + 1e-3 * torch.randn((60_000, dim), generator=g,
                                                                                device="cuda")
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows.half())
    q = torch.cat([dups.repeat(20, 1), torch.randn((4, dim), generator=g, device="cuda")]).half()
    s, i = idx.search(q, k)
    assert idx.stats()["overflow"] >= 60
    monkeypatch.delenv("CLM_SEARCH_BOUNDED")
    monkeypatch.setenv("CLM_SEARCH_FULL", "1")
    s_ref, i_ref = idx.search(q, k)
    assert torch.equal(i, i_ref) and torch.equal(s, s_ref)
    idx.close()


@pytest.mark.parametrize("k", [1, 8, 1024])
def test_overflow_wide_and_exact_paths(monkeypatch, k):
    """Overflowed lists are rebuilt whole and re-scored chunk-wise when ceil(list / 4096) * k <=
    8192 (k = 1, 8: tie groups of 60k rows), else redone by the exact scan (k = 1024); both agree
    bit for bit with the full exact scan, including the random queries of the same block."""
    monkeypatch.setenv("CLM_SEARCH_BOUNDED", "1")
    n, dim = 300_000, 96
    g = torch.Generator(device="cuda").manual_seed(11)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    dups = torch.randn((2, dim), generator=g, device="cuda")
    rows[10_000:70_000] = dups[0] + 1e-3 * torch.randn((60_000, dim), generator=g, device="cuda")
    rows[200_000:205_000] = dups[1] + 1e-3 * torch.randn((5_000, dim), generator=g, device="cuda")
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows.half())
    q = torch.cat([dups.repeat(3, 1), torch.randn((5, dim), generator=g, device="cuda")]).half()
    s, i = idx.search(q, k)
    assert idx.stats()["overflow"] >= 3
    monkeypatch.delenv("CLM_SEARCH_BOUNDED")
    monkeypatch.setenv("CLM_SEARCH_FULL", "1")
    s_ref, i_ref = idx.search(q, k)
    assert torch.equal(i, i_ref) and torch.equal(s, s_ref)
    idx.close()


@pytest.mark.parametrize("case", ["negative_topk", "wide_norms", "zero_row"])
def test_filter_skip_test_edge_cases(monkeypatch, case):
    """The filter GEMM skips a wave when (max acc * rscale) * (max or min cscale) is below every
    row's threshold (GemmArgs::cbound). Cases that exercise each side of that bound agree bit for
    bit with the full exact scan: all top-k scores negative (thresholds < 0: the min-cscale side),
    fp16 rows with norms over 4 decades (cscale spread 1e4), and a zero row (inverse norm inf:
    the bound is off and every element is tested)."""
    monkeypatch.setenv("CLM_SEARCH_BOUNDED", "1")
    n, dim, k = 300_000, 128, 10
    g = torch.Generator(device="cuda").manual_seed(21)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    q = torch.randn((24, dim), generator=g, device="cuda")
    if case == "negative_topk":
        rows = rows.abs() + 0.05           # every row in the positive orthant
        q = -(q.abs() + 0.05)              # every query in the negative one: all cosines < 0
    elif case == "wide_norms":
        rows = rows * torch.exp(torch.empty((n, 1), device="cuda").uniform_(-4.6, 4.6, generator=g))
    else:
        rows[12345] = 0
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows.half())
    s, i = idx.search(q.half(), k)
    assert idx.stats()["filtered"] + idx.stats()["overflow"] >= 24
    if case == "negative_topk":
        assert torch.all(s < 0)
    monkeypatch.delenv("CLM_SEARCH_BOUNDED")
    monkeypatch.setenv("CLM_SEARCH_FULL", "1")
    s_ref, i_ref = idx.search(q.half(), k)
    assert torch.equal(i, i_ref) and torch.equal(s, s_ref)
    idx.close()


def test_bounded_search_many_query_blocks(monkeypatch):
    """5,121 queries through the sampled bounded search: three balanced query blocks (1728, 1728,
    1665 rows; the filter GEMM on G2 tiles of both shapes) return exactly what the full exact scan
    returns."""
    monkeypatch.setenv("CLM_SEARCH_BOUNDED", "1")
    n, dim, nq, k = 40_000, 128, 5121, 5   # n >= 4 x the 8192-row sample: the sampled path serves
    g = torch.Generator(device="cuda").manual_seed(31)
    rows = torch.randn((n, dim), generator=g, device="cuda").half()
    q = torch.randn((nq, dim), generator=g, device="cuda").half()
    q[:64] = rows[torch.arange(64, device="cuda") * 600]   # exact hits at rank 0
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows)
    s, i = idx.search(q, k)
    assert idx.stats()["filtered"] + idx.stats()["overflow"] >= nq
    assert torch.equal(i[:64, 0], torch.arange(64, device="cuda") * 600)
    monkeypatch.delenv("CLM_SEARCH_BOUNDED")
    monkeypatch.setenv("CLM_SEARCH_FULL", "1")
    s_ref, i_ref = idx.search(q, k)
    assert torch.equal(i, i_ref) and torch.equal(s, s_ref)
    idx.close()


@pytest.mark.parametrize("k", [1, 3, 5, 8])
@pytest.mark.parametrize("shape", [(300, 195_328, 195_328, 0), (64, 10_001, 10_240, 0), (32, 8191, 8192, 1)])
def test_topk_threshold_streaming_equals_radix(k, shape):
    """The sampled search's thresholds: the one-pass streaming k-th value (method 0) equals the
    radix top-k select + gather (method 1) bit for bit, and numpy's k-th largest minus the margin,
    on rows with heavy duplicates, +-inf, ragged C (scalar tail) and a misaligned row base."""
    from clip_lora_match_amd import _capi as C
    nq, c, lds, shift = shape
    g = torch.Generator(device="cuda").manual_seed(k * 7 + c)
    buf = torch.randn((nq * lds + shift,), generator=g, device="cuda")
    sc = buf[shift:].view(nq, lds)
    sc[: nq // 3] = torch.round(sc[: nq // 3] * 4) / 4          # few distinct values: tie groups
    sc[nq // 3, :16] = float("inf")
    sc[nq // 3 + 1] = -float("inf")
    sc[nq // 3 + 1, 5] = 2.0
    th = [torch.empty(nq, device="cuda") for _ in range(2)]
    margin = 0.003
    L = C.lib()
    for m in (0, 1):
        C.check(L.clm_topk_threshold(0, C.ptr(sc), lds, nq, c, k, margin, m, C.ptr(th[m]), None))
    torch.cuda.synchronize()
    assert torch.equal(th[0].view(torch.int32), th[1].view(torch.int32))
    ref = np.sort(sc[:, :c].cpu().numpy(), axis=1)[:, c - k] - np.float32(margin)
    assert np.array_equal(th[0].cpu().numpy(), ref.astype(np.float32))
    assert L.clm_topk_threshold(0, C.ptr(sc), lds, nq, c, 9, margin, 0, C.ptr(th[0]), None) != 0


# ---- query fusion (seeker_service.py:84-186) ------------------------------------------------
def _unit_rows(n, d, seed):
    x = np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)
    return x / np.linalg.norm(x, axis=-1, keepdims=True)


@pytest.mark.parametrize("n,d", [(1, 512), (300, 512), (7, 768), (5, 100)])
def test_fuse_queries_vs_oracle(n, d):
    from clip_lora_match_amd.seeker import fuse_query_embeddings
    t, i = _unit_rows(n, d, 11), _unit_rows(n, d, 12)
    for wt, wi in ((0.5, 0.5), (0.7, 0.3), (1.0, 0.0)):
        got = fuse_query_embeddings(torch.from_numpy(t).cuda(), torch.from_numpy(i).cuda(), wt, wi)
        assert got.device.type == "cuda" and got.shape == (n, d)
        np.testing.assert_allclose(got.cpu().numpy(), S.fuse_query(t, i, wt, wi), atol=1e-6, rtol=0)
    # single modality: renormalise that side (:149-152); either side
    np.testing.assert_allclose(fuse_query_embeddings(None, torch.from_numpy(3 * i).cuda()).cpu().numpy(),
                               S.fuse_query(None, 3 * i), atol=1e-6, rtol=0)
    np.testing.assert_allclose(fuse_query_embeddings(torch.from_numpy(2 * t).cuda(), None).cpu().numpy(),
                               S.fuse_query(2 * t, None), atol=1e-6, rtol=0)


def test_fuse_queries_host_tensors_shapes_and_errors():
    from clip_lora_match_amd.seeker import fuse_query_embeddings
    t, i = _unit_rows(3, 512, 13), _unit_rows(3, 512, 14)
    got = fuse_query_embeddings(torch.from_numpy(t[0]), torch.from_numpy(i[0]))   # host, (D,)
    assert got.device.type == "cpu" and got.shape == (512,)
    np.testing.assert_allclose(got.numpy(), S.fuse_query(t[0], i[0]), atol=1e-6, rtol=0)
    with pytest.raises(ValueError):
        fuse_query_embeddings(None, None)
    with pytest.raises(ValueError):
        fuse_query_embeddings(torch.from_numpy(t), torch.from_numpy(i[:2]))
    # mixed residency: the host side is moved to the device; the result follows the text side
    got = fuse_query_embeddings(torch.from_numpy(t).cuda(), torch.from_numpy(i))
    np.testing.assert_allclose(got.cpu().numpy(), S.fuse_query(t, i), atol=1e-6, rtol=0)


def test_fuse_queries_c_abi_host_pointers():
    """clm_fuse_queries on host buffers (staged through HBM inside the library), in place,
    and its argument checks."""
    import ctypes

    from clip_lora_match_amd import _capi as C
    t, i = _unit_rows(9, 512, 15), _unit_rows(9, 512, 16)
    out = np.empty_like(t)
    vp = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
    C.check(C.lib().clm_fuse_queries(0, vp(t), 0.6, vp(i), 0.4, 9, 512, vp(out), None))
    np.testing.assert_allclose(out, S.fuse_query(t, i, 0.6, 0.4), atol=1e-6, rtol=0)
    a = 5 * t.copy()
    C.check(C.lib().clm_fuse_queries(0, vp(a), 1.0, None, 0.0, 9, 512, vp(a), None))   # in place, one side
    np.testing.assert_allclose(a, S.fuse_query(5 * t, None), atol=1e-6, rtol=0)
    assert C.lib().clm_fuse_queries(0, vp(t), 1.0, None, 0.0, 9, 0, vp(out), None) == C.CLM_E_ARG
    assert C.lib().clm_fuse_queries(0, vp(t), 1.0, None, 0.0, 0, 512, vp(out), None) == C.CLM_OK
    dev = torch.from_numpy(t).cuda()
    with pytest.raises(ValueError):   # mixed device / host pointers are refused
        C.check(C.lib().clm_fuse_queries(0, C.ptr(dev), 1.0, None, 0.0, 9, 512, vp(out), None))


def test_build_query_embedding_and_search_items(tmp_path):
    from PIL import Image

    from conftest import synthetic as synth
    from clip_lora_match_amd.engine import ClipLoraModel
    from clip_lora_match_amd.processor import ClipProcessor
    from clip_lora_match_amd.seeker import build_query_embedding, search_items
    from oracle import clip_ref as R

    cfg, sd, lora = synth("tiny")
    m = ClipLoraModel(cfg, compute_dtype="float16", lora_mode="merged", max_batch=8)
    m.load_tensors(sd)
    m.load_tensors(lora)
    m.finalize()
    proc = ClipProcessor(cfg)
    img = syn.images_u8(1, cfg.image_size, 21)
    Image.fromarray(img[0]).save(tmp_path / "q.png")
    ids = syn.captions(1, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 22)
    row = [int(v) for v in ids[0]]
    ri = R.image_features(sd, cfg, R.preprocess_u8(img, cfg.mean, cfg.std), lora)[0]
    rt = R.text_features(sd, cfg, ids, lora)[0]
    dev = m.device
    both = build_query_embedding(row, tmp_path / "q.png", m, proc, dev)
    assert both.device.type == "cpu" and both.dtype == torch.float32
    ref = S.fuse_query(rt, ri)
    assert 1 - float(np.dot(both.numpy(), ref)) <= 1e-5
    only_img = build_query_embedding("   ", tmp_path / "q.png", m, proc, dev)   # blank text = absent (:98)
    assert 1 - float(np.dot(only_img.numpy(), ri / np.linalg.norm(ri))) <= 1e-5
    with pytest.raises(ValueError):
        build_query_embedding("", None, m, proc, dev)
    # resident index with the fused query planted at row 17: it must come back first
    E = _unit_rows(64, cfg.proj_dim, 23)
    E[17] = both.numpy()
    index = TextSearchIndex(embeddings=torch.from_numpy(E), image_paths=[f"p{j}" for j in range(64)],
                            texts=[f"t{j}" for j in range(64)])
    res = search_items(index, m, proc, dev, query_text=row, query_image_path="q.png", top_k=3, root_dir=tmp_path)
    assert res[0].index == 17 and res[0].image_path == "p17" and abs(res[0].score - 1.0) < 1e-3
    with pytest.raises(FileNotFoundError):
        search_items(index, m, proc, dev, query_text=row, query_image_path="missing.png", root_dir=tmp_path)


def test_full_size_config4_index():
    """configs[4] at its full size: 10 M x 512 fp16 rows in HBM, 512 queries (a planted copy of
    a row for the first 64). Planted rows come back at rank 0 with score 1; the sampled bounded
    search equals the full exact scan bit for bit on a query subset; and a host check of 4
    queries (fp32 scan of every row in 1 M-row chunks, then an fp64 re-score of each chunk's
    top 64) gives the same top-5 up to 2e-6 near-ties."""
    n, dim, nq, k = 10_000_000, 512, 512, 5
    idx = CosineIndex(dim, capacity=n)
    g = torch.Generator(device="cuda").manual_seed(77)
    chunk = 1 << 20
    host = []
    for r0 in range(0, n, chunk):
        x = torch.randn((min(chunk, n - r0), dim), generator=g, device="cuda")
        xh = (x / x.norm(dim=-1, keepdim=True)).half()
        idx.append(xh)
        host.append(xh.cpu())
        del x, xh
    rows = torch.cat(host)
    del host
    gc = torch.Generator().manual_seed(78)
    plant = torch.randint(0, n, (64,), generator=gc)
    q = torch.randn((nq, dim), generator=gc).half()
    q[:64] = rows[plant]
    s, i = idx.search(q.cuda(), k)
    assert idx.stats()["filtered"] == nq
    assert torch.equal(i[:64, 0].cpu(), plant) and torch.all(s[:64, 0] == 1.0)
    assert torch.all(s[:, 1:] <= s[:, :-1])
    import os
    os.environ["CLM_SEARCH_FULL"] = "1"
    try:
        s2, i2 = idx.search(q[64:96].cuda(), k)
    finally:
        del os.environ["CLM_SEARCH_FULL"]
    assert torch.equal(i2, i[64:96]) and torch.equal(s2, s[64:96])
    qs = q[100:104].float().numpy().astype(np.float64)
    qs /= np.linalg.norm(qs, axis=-1, keepdims=True)
    cand = []
    for r0 in range(0, n, chunk):
        blk = rows[r0:r0 + chunk].float()
        sc = (torch.from_numpy(qs).float() @ blk.T)
        cand.append(torch.topk(sc, 64, dim=1).indices + r0)
    cand = torch.cat(cand, 1).numpy()
    for j in range(4):
        c = np.unique(cand[j])
        rr = rows[c].double().numpy()
        ex = (rr @ qs[j]) / np.linalg.norm(rr, axis=-1)
        order = np.lexsort((c, -ex))[:k]
        exd = dict(zip(c.tolist(), ex.tolist()))
        got = i[100 + j].cpu().numpy()
        assert S.same_topk_up_to_ties(got, c[order], _sparse_scores(exd, n), 2e-6), (j, got, c[order])
        assert np.max(np.abs(s[100 + j].cpu().numpy() - ex[order])) < 1e-6


class _sparse_scores:
    """exact scores by global row index for the rows a check looked at (same_topk_up_to_ties
    indexes its `exact_scores` argument by row)"""

    def __init__(self, d, n):
        self.d = d

    def __getitem__(self, idx):
        return np.array([self.d.get(int(t), -9.0) for t in np.atleast_1d(idx)])


# ---- shard persistence (SURVEY §5 checkpoint row) ---------------------------------------------
def test_shard_roundtrip_bit_identical_to_pt_reload(tmp_path):
    """TextSearchIndex.save_shard / load_shard vs the reference .pt reload of the same index:
    same rows, metadata and search results bit for bit; appends keep working after a reload."""
    from clip_lora_match_amd.search import TextSearchIndex, read_shard_header
    rows = syn.clustered_rows(300, 40, 512, 0.05, seed=71)           # 12,000 fp32 rows, near-ties
    q = torch.from_numpy(syn.clustered_rows(300, 1, 512, 0.05, seed=71, noise_seed=72)[:64])
    pt = tmp_path / "idx.pt"
    torch.save({"embeddings": torch.from_numpy(rows), "image_paths": [f"p{i}.jpg" for i in range(len(rows))],
                "texts": [f"t{i}" for i in range(len(rows))]}, pt)
    a = TextSearchIndex(pt)
    shard = tmp_path / "idx.clmidx"
    a.save_shard(shard)
    hdr, secs = read_shard_header(shard)
    assert hdr["n"] == len(rows) and hdr["has_f32"] and all(o % 4096 == 0 for o, _ in secs.values())
    b = TextSearchIndex.load_shard(shard)
    assert b.num_items == a.num_items and b.dim == 512
    assert torch.equal(b.embeddings, a.embeddings)
    assert b.image_paths == a.image_paths and b.texts == a.texts
    for k in (1, 5, 50):
        sa, ia = a.search_batch(q, k)
        sb, ib = b.search_batch(q, k)
        assert torch.equal(ia, ib) and torch.equal(sa, sb)
    r = b.search_with_embedding(q[3], top_k=3)
    assert r[0].image_path == f"p{r[0].index}.jpg" and r[0].text == f"t{r[0].index}"
    extra = torch.from_numpy(syn.gaussian_rows(10, 512, 73, fp16=False))
    a.append(extra, [f"x{i}" for i in range(10)], [""] * 10)
    b.append(extra, [f"x{i}" for i in range(10)], [""] * 10)
    sa, ia = a.search_batch(extra[:4], 2)
    sb, ib = b.search_batch(extra[:4], 2)
    assert torch.equal(ia, ib) and torch.equal(sa, sb) and ia[:, 0].tolist() == list(range(12000, 12004))


def test_empty_index_shard_roundtrip(tmp_path):
    """An index saved while empty (a FinderIndex before its first report) reloads as an empty index
    that accepts appends and searches them (no data sections to map at n = 0)."""
    from clip_lora_match_amd.search import TextSearchIndex
    pt = tmp_path / "empty.pt"
    torch.save({"embeddings": torch.empty((0, 512)), "image_paths": [], "texts": []}, pt)
    a = TextSearchIndex(pt)
    shard = tmp_path / "empty.clmidx"
    a.save_shard(shard)
    b = TextSearchIndex.load_shard(shard)
    assert b.num_items == 0 and b.dim == 512 and b.embeddings.shape == (0, 512)
    rows = torch.from_numpy(syn.gaussian_rows(6, 512, 75, fp16=False))
    b.append(rows, [f"p{i}" for i in range(6)], [""] * 6)
    s, i = b.search_batch(rows[:3], 2)
    assert i[:, 0].tolist() == [0, 1, 2]
    idx = CosineIndex(64)
    idx.save_shard(tmp_path / "empty64.clmidx")
    re_, hdr = CosineIndex.load_shard(tmp_path / "empty64.clmidx")
    assert hdr["n"] == 0 and len(re_) == 0
    idx.close()
    re_.close()


def test_fp16_shard_roundtrip_and_bad_files(tmp_path):
    """An fp16 CosineIndex (no fp32 copy, the configs[4] layout) in small chunks; a file that is
    not a shard raises ValueError, a missing one FileNotFoundError."""
    rows = torch.from_numpy(syn.gaussian_rows(5000, 256, 74, fp16=True))
    idx = CosineIndex(256)
    idx.append(rows)
    p = tmp_path / "f16.clmidx"
    idx.save_shard(p, chunk_rows=777)
    re_, hdr = CosineIndex.load_shard(p, chunk_rows=1000)
    assert not hdr["has_f32"] and len(re_) == 5000
    q = rows[:32].float() + 0.01
    s1, i1 = idx.search(q, 7)
    s2, i2 = re_.search(q, 7)
    assert torch.equal(i1, i2) and torch.equal(s1, s2)
    bad = tmp_path / "bad.clmidx"
    bad.write_bytes(b"not a shard at all")
    with pytest.raises(ValueError):
        CosineIndex.load_shard(bad)
    with pytest.raises(FileNotFoundError):
        CosineIndex.load_shard(tmp_path / "missing.clmidx")
    idx.close()
    re_.close()


@pytest.mark.parametrize("name", ["gauss", "clus"])
def test_large_k_vs_reference_golden(name):
    """k > 1024 (the exact scan + topk_any: exact k-th key, collection, LDS runs + merge passes)
    against the reference's own top_k_similar at k = 1025, 2000, 4096 = N: indices up to 2e-6
    near-ties, scores within 1e-6; through CosineIndex, top_k_similar and TextSearchIndex (top_k
    past N returns all N rows, as min(top_k, N) in search.py:98)."""
    g = golden("search_large_k.npz")
    gr, gq, cr, cq = syn.fp32_search_inputs()
    rows, qs = (gr, gq[:4]) if name == "gauss" else (cr, cq[:4])
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    idx = CosineIndex(rows.shape[1], capacity=rows.shape[0])
    idx.append(torch.from_numpy(rows))
    for k in (1025, 2000, 4096):
        s, i = idx.search(torch.from_numpy(qs), k)
        s, i = s.cpu().numpy(), i.cpu().numpy()
        _agree(i, g[f"{name}_idx_k{k}"].astype(np.int64), exact)
        assert np.max(np.abs(s - g[f"{name}_vals_k{k}"])) < 1e-6
        _, oi = S.topk(exact, k)
        _agree(i, oi, exact)
        assert len(set(i[0].tolist())) == k
    v, ix = top_k_similar(torch.from_numpy(qs[1]), torch.from_numpy(rows), 2000)
    assert v.shape == (2000,) and ix.shape == (2000,)
    _agree(ix.cpu().numpy()[None], g[f"{name}_idx_k2000"][1:2].astype(np.int64), exact[1:2])
    tsi = TextSearchIndex(embeddings=torch.from_numpy(rows), image_paths=[f"img{j}" for j in range(rows.shape[0])],
                          texts=[f"t{j}" for j in range(rows.shape[0])])
    res = tsi.search_with_embedding(torch.from_numpy(qs[0]), top_k=10_000)
    assert len(res) == rows.shape[0]
    got = np.array([r.index for r in res])
    _agree(got[None], g[f"{name}_idx_k4096"][:1].astype(np.int64), exact[:1])
    assert res[0].image_path == f"img{got[0]}"


@pytest.mark.parametrize("k", [5, 50, 1500])
def test_wide_dim_vs_reference_golden(k):
    """dim 1536 > 1024 (the index takes any multiple-of-64 dim up to 65536 after padding; the
    candidate margin holds to 8192): the reference's top_k_similar goldens, through top_k_similar
    and a bounded (sampled) CosineIndex search."""
    g = golden("search_large_k.npz")
    rows = syn.gaussian_rows(2048, 1536, seed=int(g["wide_seeds"][0]), fp16=False)
    qs = syn.gaussian_rows(8, 1536, seed=int(g["wide_seeds"][1]), fp16=False)
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    want = g[f"wide_idx_k{k}"].astype(np.int64)
    for q in range(2):
        v, ix = top_k_similar(torch.from_numpy(qs[q]), torch.from_numpy(rows), k)
        _agree(ix.cpu().numpy()[None], want[q:q + 1], exact[q:q + 1])
        assert np.max(np.abs(v.cpu().numpy() - g[f"wide_vals_k{k}"][q])) < 1e-6
    idx = CosineIndex(1536, capacity=2048)
    idx.append(torch.from_numpy(rows).cuda())
    import os
    os.environ["CLM_SEARCH_BOUNDED"] = "1"
    try:
        s, i = idx.search(torch.from_numpy(qs).cuda(), k)
    finally:
        del os.environ["CLM_SEARCH_BOUNDED"]
    _agree(i.cpu().numpy(), want, exact)
    assert np.max(np.abs(s.cpu().numpy() - g[f"wide_vals_k{k}"])) < 1e-6


def test_merge_past_one_sort():
    """merge_topk_gpu / clm_topk_merge with more candidates than one LDS sort (parts * k_in >
    8192) and k > 1024: the (score desc, index asc) order of the union, empty (-1) slots last."""
    from clip_lora_match_amd.distributed import merge_topk_gpu
    g = np.random.default_rng(5)
    nq, parts, k_in, k = 3, 4, 2500, 3000
    sc = (g.integers(0, 200, (nq, parts * k_in)) / 200.0).astype(np.float32)   # many ties
    ix = np.stack([g.permutation(10 * parts * k_in)[:parts * k_in] for _ in range(nq)]).astype(np.int64)
    ix[:, ::97] = -1
    s, i = merge_topk_gpu(torch.from_numpy(sc).cuda(), torch.from_numpy(ix).cuda(), parts, k)
    s, i = s.cpu().numpy(), i.cpu().numpy()
    for q in range(nq):
        ok = ix[q] >= 0
        order = np.lexsort((ix[q][ok], -sc[q][ok]))[:k]
        assert np.array_equal(i[q], ix[q][ok][order]) and np.array_equal(s[q], sc[q][ok][order])


def test_filter_tile_per_block_near_duplicates(monkeypatch):
    """The filter pass's tile is chosen per query block from that block's sampled candidate counts
    (no state carried between searches): a near-duplicate block runs gemm_kernel 256 x 256, a random
    block G2 256 x 192. Two bounded searches of the near-duplicate queries, then random queries,
    then the near-duplicates again: each equals the full exact scan bit for bit, the second equals
    the first, and the stats show which tile served which block."""
    monkeypatch.setenv("CLM_SEARCH_BOUNDED", "1")
    n, dim, k = 400_000, 128, 5
    g = torch.Generator(device="cuda").manual_seed(8)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    dups = torch.randn((4, dim), generator=g, device="cuda")
    for j in range(4):
        rows[j * 90_000: j * 90_000 + 40_000] = dups[j] + 1e-3 * torch.randn((40_000, dim), generator=g,
                                                                               device="cuda")
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows.half())
    qd = dups.repeat(16, 1).half()
    qr = torch.randn((64, dim), generator=g, device="cuda").half()
    runs = [idx.search(qd, k), idx.search(qd, k)]
    st = idx.stats()
    assert st["filter_dense"] == 2 * qd.shape[0] and st["filter_g2"] == 0, st
    runs.append(idx.search(qr, k))
    st2 = idx.stats()
    assert st2["filter_g2"] == qr.shape[0] and st2["filter_dense"] == st["filter_dense"], st2
    runs.append(idx.search(qd, k))
    monkeypatch.delenv("CLM_SEARCH_BOUNDED")
    monkeypatch.setenv("CLM_SEARCH_FULL", "1")
    ref_d, ref_r = idx.search(qd, k), idx.search(qr, k)
    for (s, i), (rs, ri) in zip(runs, [ref_d, ref_d, ref_r, ref_d]):
        assert torch.equal(i, ri) and torch.equal(s, rs)
    idx.close()


@pytest.mark.parametrize("M,N", [(512, 256 * 300), (300, 256 * 257)])
def test_sample_group_maxima_many_tiles_per_workgroup(M, N):
    """The sampled search's group-maxima score form (GemmArgs::out16 == 2, config 1) with more tiles
    than workgroups, so every workgroup's LDS ring crosses tile ends after those epilogues (ADVICE
    r05: the counted wait at a tile end must not assume more stores than this form issues). Each
    row's stored values equal, as a multiset, f16_down of the maxima of its groups of 4 columns
    of the fp32 scores of the same tile config; and mode 1 equals f16_down of every score."""
    from test_host import _f16_down
    from clip_lora_match_amd import _capi as C
    g = torch.Generator(device="cuda").manual_seed(M + N)
    K = 512
    A = (torch.randn((M, K), generator=g, device="cuda") * 0.05).half()
    W = (torch.randn((N, K), generator=g, device="cuda") * 0.05).half()
    rs = torch.rand(M, generator=g, device="cuda") + 0.5
    cs = torch.rand(N, generator=g, device="cuda") + 0.5
    st = C.stream_of(A.device)
    f32 = torch.empty((M, N), device="cuda")
    C.check(C.lib().clm_gemm(0, C.CLM_F16, C.CLM_EPI_SCORE, 1, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(f32), N,
                             None, C.ptr(rs), C.ptr(cs), st), "clm_gemm")
    s16 = torch.empty((M, N), device="cuda", dtype=torch.int16)
    C.check(C.lib().clm_gemm_scores16(0, 1, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(rs), C.ptr(cs), C.ptr(s16), N, 1,
                                      st), "clm_gemm_scores16 mode 1")
    ldg = N // 4 + 64
    grp = torch.full((M, ldg), -1, device="cuda", dtype=torch.int16)
    C.check(C.lib().clm_gemm_scores16(0, 1, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(rs), C.ptr(cs), C.ptr(grp), ldg,
                                      2, st), "clm_gemm_scores16 mode 2")
    torch.cuda.synchronize()
    sc = f32.cpu().numpy()
    want16 = _f16_down(sc)
    assert np.array_equal(s16.cpu().numpy().view(np.float16), want16)
    want = np.sort(_f16_down(sc.reshape(M, N // 4, 4).max(2)).astype(np.float32), axis=1)
    got = grp.cpu().numpy()
    assert (got[:, N // 4:] == -1).all()   # nothing past the row's groups
    got = np.sort(got[:, : N // 4].view(np.float16).astype(np.float32), axis=1)
    assert np.array_equal(got, want)


def _set_env(monkeypatch, env):
    for name in ("CLM_SEARCH_SMALLQ", "CLM_SEARCH_FULL", "CLM_SEARCH_BOUNDED", "CLM_SEARCH_EXACT"):
        monkeypatch.delenv(name, raising=False)
    for kv in env.items():
        monkeypatch.setenv(*kv)


@pytest.mark.parametrize("nq", [1, 2, 7, 16])
@pytest.mark.parametrize("name", ["gauss", "clus", "gauss_f16"])
def test_small_batch_vs_reference_golden(name, nq, monkeypatch):
    """Small query batches -- the reference's own one-query-per-call pattern (search.py:93-99,
    seeker_service.py:183-186) -- through the one-pass streaming search (search_small, forced at
    this size by CLM_SEARCH_SMALLQ=1), against the reference's top_k_similar goldens: indices
    equal up to 2e-6 near-ties, scores within 1e-6. The clustered set keeps each query's 64
    near rows inside one 256-row chunk, so the chunk-maximum threshold is loose there and lists
    overflow into the whole-list pass: that path is checked too. k = 50 needs 50 chunks (the
    4,096-row index has 16) and falls back to the regular routing."""
    _set_env(monkeypatch, {"CLM_SEARCH_SMALLQ": "1"})
    if name == "gauss_f16":
        g = golden("search_gauss.npz")
        rows = syn.gaussian_rows(int(g["n"]), int(g["dim"]), int(g["row_seed"]))
        qs = syn.gaussian_rows(int(g["nq"]), int(g["dim"]), int(g["q_seed"]))
        key = ""
    else:
        g = golden("search_fp32.npz")
        gr, gq, cr, cq = syn.fp32_search_inputs()
        rows, qs = (gr, gq) if name == "gauss" else (cr, cq)
        key = name + "_"
    idx = CosineIndex(512, capacity=rows.shape[0])
    idx.append(torch.from_numpy(rows))
    exact = S.cosine_scores(qs.astype(np.float64), rows.astype(np.float64))
    for k in (1, 5, 10, 50):
        for q0 in range(0, qs.shape[0], nq):
            s, i = idx.search(torch.from_numpy(qs[q0:q0 + nq]), k)
            s, i = s.cpu().numpy(), i.cpu().numpy()
            _agree(i, g[f"{key}idx_k{k}"][q0:q0 + nq], exact[q0:q0 + nq])
            assert np.max(np.abs(s - g[f"{key}vals_k{k}"][q0:q0 + nq])) < 1e-6, (k, q0)
    st = idx.stats()   # k = 1, 5, 10: every query on the streaming search (or its overflow pass); k = 50: the full scan
    assert st["small_scan"] + st["overflow"] == 3 * qs.shape[0] and st["full_exact"] == qs.shape[0], st
    assert st["small_scan"] > 0, st


@pytest.mark.parametrize("dim,n,fp32_rows", [(512, 1_200_003, True), (768, 300_001, False), (64, 100_000, False)])
def test_small_batch_bit_identical_to_full_scan(dim, n, fp32_rows, monkeypatch):
    """search_small == the full exact scan, indices and scores bit for bit: nq 1 / 5 / 16, k up to
    100, near-duplicate queries, a ragged last block and chunk (n % 256 != 0), fp32 rows (re-score
    against the fp32 copy) and fp16-only indexes, row widths 64 / 512 / 768."""
    g = torch.Generator(device="cuda").manual_seed(dim + n)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    if not fp32_rows:
        rows = rows.half()
    q = torch.randn((16, dim), generator=g, device="cuda")
    q[:4] = rows[torch.arange(4, device="cuda") * 1000 + 7].float() + 0.01 * q[:4]
    q[4] = rows[n - 1].float()                      # the last (ragged) block's last row
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows)
    for nq in (1, 5, 16):
        for k in (1, 5, 12, 100):
            _set_env(monkeypatch, {"CLM_SEARCH_SMALLQ": "1"})
            s1, i1 = idx.search(q[:nq], k)
            _set_env(monkeypatch, {"CLM_SEARCH_FULL": "1", "CLM_SEARCH_SMALLQ": "0"})
            s2, i2 = idx.search(q[:nq], k)
            assert torch.equal(i1, i2) and torch.equal(s1, s2), (nq, k)
    _set_env(monkeypatch, {})
    assert torch.equal(i2[:4, 0], torch.arange(4, device="cuda") * 1000 + 7)
    assert int(i2[4, 0]) == n - 1
    st = idx.stats()
    assert st["small_scan"] + st["overflow"] == 4 * (1 + 5 + 16) and st["small_scan"] > 0, st


def test_small_batch_overflow_near_duplicates(monkeypatch):
    """A query whose candidate window holds thousands of rows (5,000 near copies of one row spread
    over many chunks, like a finder index of one description template): its list overflows
    CAND_CAP and is rebuilt whole; the result equals the full exact scan's."""
    n, dim = 400_000, 512
    g = torch.Generator(device="cuda").manual_seed(3)
    rows = torch.randn((n, dim), generator=g, device="cuda")
    center = rows[123].clone()
    dup = torch.arange(5000, device="cuda") * 80 + 11
    rows[dup] = center + 1e-3 * torch.randn((5000, dim), generator=g, device="cuda")
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows)
    q = torch.stack([center, torch.randn(dim, generator=g, device="cuda")])
    for k in (1, 5, 64):
        _set_env(monkeypatch, {"CLM_SEARCH_SMALLQ": "1"})
        s1, i1 = idx.search(q, k)
        _set_env(monkeypatch, {"CLM_SEARCH_FULL": "1", "CLM_SEARCH_SMALLQ": "0"})
        s2, i2 = idx.search(q, k)
        assert torch.equal(i1, i2) and torch.equal(s1, s2), k
    _set_env(monkeypatch, {})
    assert idx.stats()["overflow"] >= 3, idx.stats()


def test_small_batch_default_routing(monkeypatch):
    """Without any switch, nq <= 16 on an index of >= 65,536 rows takes the streaming search
    (stats), and equals the sampled bounded search bit for bit; one query per call too (the
    reference's pattern, which the full exact scan served before round 6)."""
    _set_env(monkeypatch, {})
    n, dim = 9_000_000, 64
    g = torch.Generator(device="cuda").manual_seed(4)
    rows = torch.randn((n, dim), generator=g, device="cuda").half()
    q = rows[torch.tensor([5, 8_999_999], device="cuda")].float() + 0.02 * torch.randn((2, dim), generator=g,
                                                                                        device="cuda")
    idx = CosineIndex(dim, capacity=n)
    idx.append(rows)
    s1, i1 = idx.search(q, 5)
    assert idx.stats()["small_scan"] == 2, idx.stats()
    _set_env(monkeypatch, {"CLM_SEARCH_SMALLQ": "0"})
    s2, i2 = idx.search(q, 5)
    assert idx.stats()["filtered"] == 2, idx.stats()
    assert torch.equal(i1, i2) and torch.equal(s1, s2)
    assert int(i1[0, 0]) == 5 and int(i1[1, 0]) == 8_999_999
    _set_env(monkeypatch, {})
    s3, i3 = idx.search(q[1], 5)
    assert idx.stats()["small_scan"] == 3, idx.stats()
    assert torch.equal(i3[0], i1[1]) and torch.equal(s3[0], s1[1])
