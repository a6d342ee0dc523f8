"""GPU parity of the batched index build (index_build.rebuild_index, the reference's
scripts/rebuild_index.py:28-115) against the reference's per-item loop on our encoder
and the CPU oracle; the .pt it writes loads in TextSearchIndex and finds every item."""
import numpy as np
import pytest
import torch

from conftest import synthetic

from clip_lora_match_amd import synthetic as syn
from clip_lora_match_amd.clip_model import encode_image, encode_text
from clip_lora_match_amd.engine import ClipLoraModel
from clip_lora_match_amd.index_build import encode_items, rebuild_index
from clip_lora_match_amd.processor import ClipProcessor
from clip_lora_match_amd.search import TextSearchIndex
from oracle import clip_ref as R

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiny():
    cfg, sd, lora = synthetic("tiny")
    m = ClipLoraModel(cfg, compute_dtype="float16", lora_mode="merged", max_batch=16)
    m.load_tensors(sd)
    m.load_tensors(lora)
    m.finalize()
    return m, ClipProcessor(cfg), cfg, sd, lora


def _id_rows(cfg, n, seed):
    ids = syn.captions(n, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, seed)
    rows = []
    for r in ids:   # each caption cut at its first EOS (what the tokenizer emits per item)
        e = int(np.argmax(r == cfg.eos_token_id))
        rows.append([int(v) for v in r[:e + 1]])
    return ids, rows


def test_rebuild_text_index_matches_per_item_loop(tiny, tmp_path):
    m, proc, cfg, sd, lora = tiny
    ids, rows = _id_rows(cfg, 37, 61)
    paths = [f"img/{j}.jpg" for j in range(37)]
    out = tmp_path / "index" / "items.pt"
    E = rebuild_index(m, proc, rows, paths, out, batch_size=8)            # ragged last batch (37 = 4*8 + 5)
    assert E.shape == (37, cfg.proj_dim) and E.dtype == torch.float32
    # the reference loop: encode_text per item, then a second normalise (rebuild_index.py:64-77)
    loop = torch.stack([encode_text(r, m, proc, m.device) for r in rows])
    loop = loop / loop.norm(dim=-1, keepdim=True)
    assert float((1 - (E * loop).sum(-1)).abs().max()) <= 1e-6
    ref = R.text_features(sd, cfg, ids, lora)
    ref = ref / np.linalg.norm(ref, axis=-1, keepdims=True)
    assert float(np.max(1 - np.sum(E.numpy() * ref, -1))) <= 1e-5
    # batch size does not change a row (batch-invariant encoder)
    assert torch.equal(rebuild_index(m, proc, rows, paths, tmp_path / "b3.pt", batch_size=3), E)
    # the file is the reference's format; every item finds itself first
    obj = torch.load(out, weights_only=True)
    assert set(obj) == {"embeddings", "image_paths", "texts"} and obj["image_paths"] == paths
    idx = TextSearchIndex(out)
    for j in (0, 17, 36):
        res = idx.search_with_embedding(E[j], top_k=2)
        assert res[0].index == j and res[0].image_path == paths[j]


def test_rebuild_image_index_and_edge_cases(tiny, tmp_path):
    from PIL import Image
    m, proc, cfg, sd, lora = tiny
    imgs = syn.images_u8(5, cfg.image_size, 62)
    paths = []
    for j in range(5):
        p = tmp_path / f"{j}.png"
        Image.fromarray(imgs[j]).save(p)
        paths.append(str(p))
    E = rebuild_index(m, proc, [""] * 5, paths, tmp_path / "img.pt", batch_size=2, from_images=True)
    loop = torch.stack([encode_image(p, m, proc, m.device) for p in paths])
    assert float((1 - (E * loop).sum(-1)).abs().max()) <= 1e-6
    ref = R.image_features(sd, cfg, R.preprocess_u8(imgs, cfg.mean, cfg.std), lora)
    ref = ref / np.linalg.norm(ref, axis=-1, keepdims=True)
    assert float(np.max(1 - np.sum(E.numpy() * ref, -1))) <= 1e-5
    # no items: nothing written (rebuild_index.py:54-56); mismatched lists and bad mode raise
    assert rebuild_index(m, proc, [], [], tmp_path / "none.pt").shape == (0, cfg.proj_dim)
    assert not (tmp_path / "none.pt").exists()
    with pytest.raises(ValueError):
        rebuild_index(m, proc, ["a"], [], tmp_path / "x.pt")
    with pytest.raises(ValueError):
        encode_items(m, proc)
    with pytest.raises(FileNotFoundError):
        encode_items(m, proc, images=[str(tmp_path / "missing.png")])
