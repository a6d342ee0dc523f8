"""The CPU oracle against the goldens (transformers CLIPModel + the reference's own
similarity.py outputs), so the GPU parity tests rest on a pinned checker."""
import numpy as np
import pytest

from conftest import GOLDEN, golden, synthetic

import clip_lora_match_amd as clm
from clip_lora_match_amd import synthetic as syn
from oracle import clip_ref as R
from oracle import search_ref as S


def test_preprocess_is_clip_image_processor_exactly():
    transformers = pytest.importorskip("transformers")
    from transformers import CLIPImageProcessor
    cfg = clm.get_preset("ViT-B/32")
    imgs = syn.images_u8(2, cfg.image_size, 3)
    pv = CLIPImageProcessor()(images=list(imgs), return_tensors="np")["pixel_values"]
    assert np.array_equal(pv, R.preprocess_u8(imgs, cfg.mean, cfg.std))


@pytest.mark.parametrize("name,preset", [("enc_tiny_lora.npz", "tiny"), ("enc_b32_lora.npz", "ViT-B/32"),
                                         ("enc_l14_lora.npz", "ViT-L/14@336")])
def test_oracle_matches_transformers_golden(name, preset):
    g = golden(name)
    cfg, sd, lora = synthetic(preset, True)
    assert cfg.lora_r == int(g["r"]) and ",".join(cfg.lora_targets) == str(g["targets"])
    imgs = syn.images_u8(int(g["n_img"]), cfg.image_size, int(g["img_seed"]))
    ids = syn.captions(int(g["n_txt"]), int(g["L"]), cfg.bos_token_id, cfg.eos_token_id, int(g["cap_seed"]))
    assert np.array_equal(ids, g["ids"])
    fi = R.image_features(sd, cfg, R.preprocess_u8(imgs, cfg.mean, cfg.std), lora)
    ft = R.text_features(sd, cfg, ids, lora)
    assert np.max(np.abs(fi - g["emb_img"])) < 2e-6
    assert np.max(np.abs(ft - g["emb_txt"])) < 2e-6
    # LoRA is not a no-op in the fixtures (non-zero B)
    assert np.max(np.abs(g["emb_txt"] - g["emb_txt_base"])) > 1e-2
    assert np.max(np.abs(g["emb_img"] - g["emb_img_base"])) > 1e-3


def test_eos_rules_agree_for_clip_ids():
    cfg = clm.get_preset("ViT-B/32")
    ids = syn.captions(32, 77, cfg.bos_token_id, cfg.eos_token_id, 5)
    assert np.array_equal(R.eos_positions(ids, cfg.eos_token_id), R.eos_positions(ids, 2))


@pytest.mark.parametrize("k", [1, 5, 10, 50])
def test_search_oracle_vs_reference_golden(k):
    g = golden("search_gauss.npz")
    rows = syn.gaussian_rows(int(g["n"]), int(g["dim"]), int(g["row_seed"]))
    qs = syn.gaussian_rows(int(g["nq"]), int(g["dim"]), int(g["q_seed"]))
    exact = S.cosine_scores(qs, rows)
    vals, idx = S.topk(exact, k)
    for q in range(qs.shape[0]):
        assert S.same_topk_up_to_ties(idx[q], g[f"idx_k{k}"][q], exact[q], 2e-6)
    assert np.max(np.abs(vals - g[f"vals_k{k}"])) < 1e-6
    assert np.max(np.abs(exact[0] - g["cos_q0"])) < 1e-6


def test_custom_index_known_answers():
    import torch
    g = golden("custom_index_top3.npz")
    obj = torch.load(f"{GOLDEN}/custom_items_index.pt", map_location="cpu", weights_only=True)
    E = obj["embeddings"].float().numpy()
    assert E.shape == (6, 512) and len(obj["image_paths"]) == 6 and len(obj["texts"]) == 6
    vals, idx = S.search(E, E, 3)
    assert idx.tolist() == g["idx"].tolist() == [[0, 1, 2], [1, 2, 0], [2, 1, 5], [3, 4, 5], [4, 3, 5], [5, 2, 4]]
    assert abs(vals[2, 1] - 0.828312) < 1e-6 and abs(vals[2, 2] - 0.818218) < 1e-6


def test_topk_tie_rule_and_tie_comparator():
    s = np.array([[0.5, 0.9, 0.9, 0.1, 0.9]])
    v, i = S.topk(s, 3)
    assert i.tolist() == [[1, 2, 4]]
    assert S.same_topk_up_to_ties(np.array([1, 4, 2]), np.array([1, 2, 4]), s[0], 1e-9)
    assert not S.same_topk_up_to_ties(np.array([1, 0, 2]), np.array([1, 2, 4]), s[0], 1e-9)


def test_fuse_query_oracle_is_seeker_service_rule():
    """S.fuse_query restates seeker_service.py:148-157; check it against that expression
    evaluated with torch fp32 exactly as the service writes it (sum over (emb, w) pairs)."""
    import torch
    rng = np.random.default_rng(3)
    t = rng.standard_normal((6, 512)).astype(np.float32)
    i = rng.standard_normal((6, 512)).astype(np.float32)
    t /= np.linalg.norm(t, axis=-1, keepdims=True)
    i /= np.linalg.norm(i, axis=-1, keepdims=True)
    embs = [(torch.from_numpy(t), 0.5), (torch.from_numpy(i), 0.5)]
    weighted = sum(w * e for e, w in embs)
    weighted = weighted / weighted.norm(dim=-1, keepdim=True)
    np.testing.assert_allclose(S.fuse_query(t, i), weighted.numpy(), atol=2e-7, rtol=0)
    one = torch.from_numpy(3 * t)
    np.testing.assert_allclose(S.fuse_query(None, 3 * t), (one / one.norm(dim=-1, keepdim=True)).numpy(),
                               atol=2e-7, rtol=0)
    # the fused query of a pair lies between its parts: equal cosine to both at 0.5/0.5
    f = S.fuse_query(t, i)
    np.testing.assert_allclose(np.sum(f * t, -1), np.sum(f * i, -1), atol=1e-6)
    with pytest.raises(ValueError):
        S.fuse_query(None, None)


@pytest.mark.parametrize("name", ["gauss", "clus"])
@pytest.mark.parametrize("k", [1, 5, 10, 50])
def test_search_oracle_vs_reference_fp32_golden(name, k):
    """fp32 (not fp16-representable) rows/queries: the oracle's exact (fp64) ranking equals the
    reference's fp32 top_k_similar up to 2e-6 near-ties, and its scores match to fp32 rounding.
    The clustered set has top-k scores 1e-5..1e-4 apart (below fp16 operand rounding)."""
    g = golden("search_fp32.npz")
    gr, gq, cr, cq = syn.fp32_search_inputs()
    rows, qs = (gr, gq) if name == "gauss" else (cr, cq)
    exact = S.cosine_scores(qs, rows)
    vals, idx = S.topk(exact, k)
    for q in range(qs.shape[0]):
        assert S.same_topk_up_to_ties(idx[q], g[f"{name}_idx_k{k}"][q], exact[q], 2e-6)
    assert np.max(np.abs(vals - g[f"{name}_vals_k{k}"])) < 1e-6
    assert np.max(np.abs(exact[0] - g[f"{name}_cos_q0"])) < 1e-6
    if name == "clus" and k == 10:   # the fixture is non-trivial: neighbours closer than fp16 resolution
        gaps = -np.diff(vals, axis=1)
        assert np.median(gaps) < 1e-4


@pytest.mark.parametrize("name", ["gauss", "clus"])
@pytest.mark.parametrize("k", [1025, 2000, 4096])
def test_search_oracle_vs_reference_large_k(name, k):
    """k > 1024 up to k = N (search_large_k.npz, the reference's own top_k_similar on the fp32 sets):
    the oracle's exact ranking equals it up to 2e-6 near-ties, scores to fp32 rounding."""
    g = golden("search_large_k.npz")
    gr, gq, cr, cq = syn.fp32_search_inputs()
    rows, qs = (gr, gq[:4]) if name == "gauss" else (cr, cq[:4])
    exact = S.cosine_scores(qs, rows)
    vals, idx = S.topk(exact, k)
    for q in range(4):
        assert S.same_topk_up_to_ties(idx[q], g[f"{name}_idx_k{k}"][q].astype(np.int64), exact[q], 2e-6)
    assert np.max(np.abs(vals - g[f"{name}_vals_k{k}"])) < 1e-6


@pytest.mark.parametrize("k", [5, 50, 1500])
def test_search_oracle_vs_reference_wide_dim(k):
    """dim 1536 (> 1024) rows through the reference's top_k_similar: the oracle agrees."""
    g = golden("search_large_k.npz")
    rows = syn.gaussian_rows(2048, 1536, seed=int(g["wide_seeds"][0]), fp16=False)
    qs = syn.gaussian_rows(8, 1536, seed=int(g["wide_seeds"][1]), fp16=False)
    exact = S.cosine_scores(qs, rows)
    vals, idx = S.topk(exact, k)
    for q in range(8):
        assert S.same_topk_up_to_ties(idx[q], g[f"wide_idx_k{k}"][q].astype(np.int64), exact[q], 2e-6)
    assert np.max(np.abs(vals - g[f"wide_vals_k{k}"])) < 1e-6


def test_image_oracle_reproduces_clip_image_processor_golden():
    """oracle.image_ref (PIL's bicubic resample restated + transformers' size / crop rules) gives
    the pixel_values CLIPImageProcessor produced for the reference's 17 committed images and the
    odd-size synthetic set, bit for bit (sha256 of the float32 pixel_values)."""
    from golden_images import pil_images, sha
    from oracle import image_ref as IR
    g = golden("enc_b32_lora_images.npz")
    cfg = clm.get_preset("ViT-B/32")
    labels, pils = pil_images()
    for i, (lab, im) in enumerate(zip(labels, pils)):
        a = np.asarray(im, np.uint8)
        assert sha(a) == str(g["dec_sha"][i]), f"{lab}: decoded pixels differ from the golden's"
        crop = IR.resize_crop_u8(a, cfg.image_size)
        assert sha(R.preprocess_u8(crop[None], cfg.mean, cfg.std)[0]) == str(g["pv_sha"][i]), lab


@pytest.mark.parametrize("seed", range(4))
def test_image_oracle_equals_pil_resize(seed):
    """the numpy restatement of Resample.c vs Pillow itself, random sizes and both schedules"""
    from PIL import Image
    from oracle import image_ref as IR
    rng = np.random.default_rng(seed)
    for _ in range(12):
        h, w = (int(v) for v in rng.integers(1, 400, 2))
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        nh, nw = IR.shortest_edge_size(h, w, 224)
        pil = np.asarray(Image.fromarray(a).resize((nw, nh), Image.BICUBIC))
        assert np.array_equal(IR.resize_bicubic(a, nw, nh), pil), (h, w)
        assert np.array_equal(IR.resize_crop_u8_window(a, 224), IR.resize_crop_u8(a, 224)), (h, w)
