"""The drop-in API end to end on the GPU:
load_clip_model from a YAML config + a PEFT adapter directory -> encode_image / encode_text /
embed_* / search_by_* / the finder's report flow, against the transformers-generated goldens.

Tolerances as tests/test_gpu_encode.py (fp16 parity mode: scores 1e-3, 1 - cos 1e-5).
"""
import os

import numpy as np
import pytest
import torch
import yaml

from conftest import GOLDEN, golden, synthetic

from clip_lora_match_amd import synthetic as syn
from clip_lora_match_amd import weights as W
from clip_lora_match_amd.clip_model import encode_image, encode_text, load_clip_model
from clip_lora_match_amd.embed_image import embed_image, embed_images_batch
from clip_lora_match_amd.embed_text import embed_text
from clip_lora_match_amd.lora_adapter import LoraConfig, attach_lora_to_clip, create_lora_config
from clip_lora_match_amd.search import TextSearchIndex

pytestmark = pytest.mark.gpu
TOL = {"float16": dict(score=1e-3, cos=1e-5), "bfloat16": dict(score=2.5e-3, cos=1e-4)}
TOK_DIR = os.path.join(GOLDEN, "clip_bpe")


def _check(a, b, dtype="float16"):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    cos = np.sum(a * b, -1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
    assert np.max(1 - cos) <= TOL[dtype]["cos"], f"1 - cos {np.max(1 - cos):.3e}"
    assert np.max(np.abs(a @ a.T - b @ b.T)) <= TOL[dtype]["score"]


def _yaml(tmp_path, dtype="float32", **model):
    cfg = {"model": {"name": "openai/clip-vit-base-patch32", "device": "cpu", "dtype": dtype, **model},
           "preprocess": {"image_size": 224}}
    p = tmp_path / "clip_config.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return p


def _images(tmp_path, n, seed, size=224):
    from PIL import Image
    imgs = syn.images_u8(n, size, seed)
    paths = []
    for i in range(n):
        p = tmp_path / f"img{i}.png"
        Image.fromarray(imgs[i]).save(p)
        paths.append(p)
    return imgs, paths


def _peft_dir(tmp_path, cfg, lora, key_style):
    tensors = lora
    if key_style == "default":     # PEFT keeps the adapter name in some versions' keys
        tensors = {k.replace(".lora_A.weight", ".lora_A.default.weight").replace(
            ".lora_B.weight", ".lora_B.default.weight"): v for k, v in lora.items()}
    elif key_style == "bare":      # no base_model.model. prefix
        tensors = {k[len("base_model.model."):]: v for k, v in lora.items()}
    d = tmp_path / f"adapter_{key_style}"
    W.save_peft_adapter(d, tensors, cfg.lora_r, cfg.lora_alpha, cfg.lora_targets)
    return d


@pytest.mark.parametrize("key_style", ["plain", "default", "bare"])
@pytest.mark.parametrize("dtype", ["float32", "bfloat16"])
def test_load_clip_model_peft_dir_vs_golden(tmp_path, key_style, dtype):
    """configs[1] through the drop-in: YAML + PEFT adapter dir -> encode_image (PNG files) /
    encode_text, vs the transformers+LoRA goldens (clip_model.py:37-150)."""
    g = golden("enc_b32_lora.npz")
    cfg, sd, lora = synthetic("ViT-B/32")
    adir = _peft_dir(tmp_path, cfg, lora, key_style)
    model, proc, dev = load_clip_model(_yaml(tmp_path, dtype), use_lora=True, lora_weights_path=adir,
                                       weights_dir="synthetic", max_batch=8)
    assert dev.type == "cuda" and model.cfg.lora_r == 8 and model.cfg.lora_scaling == 2.0
    _, paths = _images(tmp_path, int(g["n_img"]), int(g["img_seed"]))
    ei = np.stack([encode_image(p, model, proc, dev).numpy() for p in paths])
    et = np.stack([encode_text([int(v) for v in row], model, proc, dev).numpy() for row in g["ids"]])
    assert ei.dtype == np.float32 and ei.shape == (4, 512)
    np.testing.assert_allclose(np.linalg.norm(ei, axis=-1), 1.0, atol=1e-6)
    mode = "bfloat16" if dtype == "bfloat16" else "float16"
    _check(ei, g["emb_img"], mode)
    _check(et, g["emb_txt"], mode)
    model.close()


def test_configs0_no_lora_and_missing_lora_dir(tmp_path, capsys):
    """configs[0] (B/32, no LoRA) vs the base goldens; a missing adapter dir prints the
    reference's warning and runs the base model (clip_model.py:70-75); strict raises."""
    g = golden("enc_b32_lora.npz")
    _, paths = _images(tmp_path, int(g["n_img"]), int(g["img_seed"]))
    y = _yaml(tmp_path)
    for kw in ({"use_lora": False}, {"use_lora": True, "lora_weights_path": tmp_path / "nope"},
               {"use_lora": True}):
        model, proc, dev = load_clip_model(y, weights_dir="synthetic", max_batch=8, **kw)
        assert model.cfg.lora_r == 0
        ei = np.stack([encode_image(p, model, proc, dev).numpy() for p in paths])
        et = np.stack([encode_text(row, model, proc, dev).numpy() for row in torch.from_numpy(g["ids"])])
        _check(ei, g["emb_img_base"])
        _check(et, g["emb_txt_base"])
        model.close()
    out = capsys.readouterr().out
    assert "tidak ditemukan" in out and "tidak diset" in out
    with pytest.raises(FileNotFoundError):
        load_clip_model(y, use_lora=True, lora_weights_path=tmp_path / "nope", weights_dir="synthetic",
                        strict_lora=True)
    with pytest.raises(FileNotFoundError):
        encode_image(tmp_path / "missing.png", None, None, None)


def test_weights_are_never_silently_synthetic(tmp_path, monkeypatch):
    monkeypatch.delenv("CLM_WEIGHTS_DIR", raising=False)
    with pytest.raises(OSError):
        load_clip_model(_yaml(tmp_path))
    with pytest.raises(FileNotFoundError):
        load_clip_model(_yaml(tmp_path, weights_dir=str(tmp_path / "no_ckpt")))
    with pytest.raises(FileNotFoundError):
        load_clip_model(tmp_path / "missing.yaml")


def test_local_checkpoint_dir(tmp_path):
    """A transformers-layout checkpoint dir (model.safetensors) named in the YAML is loaded."""
    from safetensors.numpy import save_file
    cfg, sd, _ = synthetic("ViT-B/32", lora_on=False)
    ck = tmp_path / "ckpt"
    ck.mkdir()
    save_file({k: np.ascontiguousarray(v) for k, v in sd.items()}, str(ck / "model.safetensors"))
    g = golden("enc_b32_lora.npz")
    model, proc, dev = load_clip_model(_yaml(tmp_path, weights_dir=str(ck)), max_batch=8)
    et = embed_text(model, proc, g["ids"].tolist(), dev)
    _check(et.numpy(), g["emb_txt_base"])
    model.close()


def test_attach_lora_keeps_the_models_weights(tmp_path):
    """attach_lora_to_clip wraps THE GIVEN model (lora_adapter.py:46-56): a PEFT-initialised
    adapter (B = 0) leaves its embeddings unchanged; the synthetic adapter reproduces the
    LoRA golden. The base here is a local checkpoint, not the synthetic default."""
    from safetensors.numpy import save_file
    g = golden("enc_b32_lora.npz")
    cfg, sd, _ = synthetic("ViT-B/32", lora_on=False)
    ck = tmp_path / "ckpt"
    ck.mkdir()
    save_file({k: np.ascontiguousarray(v) for k, v in sd.items()}, str(ck / "model.safetensors"))
    model, proc, dev = load_clip_model(_yaml(tmp_path), weights_dir=ck, max_batch=8)
    ids = torch.from_numpy(g["ids"]).cuda()
    base = model.encode_ids(ids).cpu().numpy()
    lc = tmp_path / "lora_config.yaml"
    lc.write_text(yaml.safe_dump({"lora": {"r": 8, "alpha": 16, "dropout": 0.1},
                                  "model": {"target_modules": ["q_proj", "k_proj", "v_proj", "out_proj"]}}))
    lcfg = create_lora_config(lc)
    same = attach_lora_to_clip(model, lcfg)
    assert same is model and model.cfg.lora_r == 8
    after = model.encode_ids(ids).cpu().numpy()
    assert np.max(np.abs(after - base)) < 1e-6
    _check(base, g["emb_txt_base"])
    attach_lora_to_clip(model, lcfg, init="synthetic", seed=1)
    _check(model.encode_ids(ids).cpu().numpy(), g["emb_txt"])
    model.close()


def test_embed_image_and_batch(tmp_path):
    from PIL import Image
    g = golden("enc_b32_lora.npz")
    model, proc, dev = load_clip_model(_yaml(tmp_path), use_lora=True, lora_weights_path="synthetic",
                                       weights_dir="synthetic", max_batch=3)
    imgs, paths = _images(tmp_path, int(g["n_img"]), int(g["img_seed"]))
    e0 = embed_image(model, proc, paths[0], dev)
    assert e0.shape == (512,) and e0.device.type == "cpu"
    _check(e0[None].numpy(), g["emb_img"][:1])
    mixed = [paths[0], Image.fromarray(imgs[1]), imgs[2], str(paths[3])]
    eb = embed_images_batch(model, proc, mixed, dev, batch_size=2)   # chunks > max_batch are split
    assert eb.shape == (4, 512)
    _check(eb.numpy(), g["emb_img"])
    raw = embed_images_batch(model, proc, paths, dev, normalize=False)
    np.testing.assert_allclose((raw / raw.norm(dim=-1, keepdim=True)).numpy(), eb.numpy(), atol=1e-6)
    empty = embed_images_batch(model, proc, [], dev)
    assert empty.shape == (0,)
    # non-224 inputs go through the GPU resize / centre-crop path (tests/test_gpu_image.py checks its bits)
    big = Image.fromarray(syn.images_u8(1, 300, 5)[0]).resize((300, 260))
    assert embed_image(model, proc, big, dev).shape == (512,)
    with pytest.raises(FileNotFoundError):
        embed_image(model, proc, tmp_path / "nope.png", dev)
    model.close()


def test_embed_text_strings_through_the_bpe_tokenizer(tmp_path):
    """embed_text with str / list[str] (processor.tokenizer over a local vocab, padding to the
    longest row, embed_text.py:35-41) == the same captions' token ids encoded directly."""
    from clip_lora_match_amd.tokenizer import ClipBPETokenizer
    model, proc, dev = load_clip_model(_yaml(tmp_path, tokenizer_dir=TOK_DIR), use_lora=True,
                                       lora_weights_path="synthetic", weights_dir="synthetic", max_batch=8)
    tok = ClipBPETokenizer.from_dir(TOK_DIR)
    caps = ["a red backpack found near the library", "Dompet hitam, ditemukan di kantin",
            "it's a blue umbrella!! (don't lose it)"]
    one = embed_text(model, proc, caps[0], dev)
    many = embed_text(model, proc, caps, dev)
    assert one.shape == (512,) and many.shape == (3, 512)
    ids = tok(caps, padding=True, truncation=True, max_length=77)["input_ids"]
    direct = model.encode_ids(torch.tensor(ids, dtype=torch.int32).cuda()).cpu()
    assert torch.equal(many, direct)
    _check(one[None].numpy(), many[:1].numpy())     # longest-row padding: same pooled EOS row
    e = encode_text(caps[1], model, proc, dev)
    _check(e[None].numpy(), many[1:2].numpy())
    model.close()


def test_search_by_text_and_image(tmp_path):
    model, proc, dev = load_clip_model(_yaml(tmp_path, tokenizer_dir=TOK_DIR), use_lora=True,
                                       lora_weights_path="synthetic", weights_dir="synthetic", max_batch=8)
    _, paths = _images(tmp_path, 2, 77)
    q_img = encode_image(paths[0], model, proc, dev)
    q_txt = encode_text("black wallet with student card", model, proc, dev)
    E = torch.from_numpy(syn.gaussian_rows(500, 512, 3, fp16=False))
    E[123] = q_img
    E[321] = q_txt
    idx_path = tmp_path / "idx.pt"
    torch.save({"embeddings": E, "image_paths": [f"p{i}" for i in range(500)],
                "texts": [f"t{i}" for i in range(500)]}, idx_path)
    ix = TextSearchIndex(idx_path)
    r = ix.search_by_image(paths[0], model, proc, dev, top_k=3)
    assert r[0].index == 123 and r[0].image_path == "p123" and abs(r[0].score - 1.0) < 1e-6
    r = ix.search_by_text("black wallet with student card", model, proc, dev, top_k=3)
    assert r[0].index == 321 and r[0].text == "t321" and abs(r[0].score - 1.0) < 1e-6
    with pytest.raises(FileNotFoundError):
        ix.search_by_image(tmp_path / "nope.png", model, proc, dev)
    model.close()


def test_finder_report_flow_and_o1_append(tmp_path):
    """finder_service.py:107-216 on a resident index: report -> searchable at once -> the saved
    .pt reloads with identical results; 1000 single appends cost amortised O(1) (the host
    mirror reallocates O(log n) times, never per report)."""
    from clip_lora_match_amd.finder import FinderIndex
    model, proc, dev = load_clip_model(_yaml(tmp_path, tokenizer_dir=TOK_DIR), use_lora=True,
                                       lora_weights_path="synthetic", weights_dir="synthetic", max_batch=8)
    _, paths = _images(tmp_path, 3, 91)
    up = tmp_path / "data" / "reported"
    fi = FinderIndex(model, proc, dev, tmp_path / "data" / "index.pt", root_dir=tmp_path, upload_dir=up,
                     save_every=2)
    rec = fi.report_item(paths[0], "dompet hitam", location="kantin")
    assert rec["id"] == 0 and rec["description"] == "dompet hitam, ditemukan di kantin"
    assert rec["image_path"] == "data/reported/img0.png" and (up / "img0.png").exists()
    assert not (tmp_path / "data" / "index.pt").exists()          # save_every=2: not yet
    fi.report_item(paths[1], "red backpack")
    assert (tmp_path / "data" / "index.pt").exists()
    q = encode_text("dompet hitam, ditemukan di kantin", model, proc, dev)
    assert fi.search(q, 1)[0].index == 0
    # 3000 sequential single-row appends: amortised O(1) host + HBM append (the host buffer
    # doubles: 1024 -> 2048 -> 4096 rows, three allocations in all)
    ix = fi.index
    ptrs = set()
    rows = syn.gaussian_rows(3000, 512, 8, fp16=False)
    for i in range(3000):
        ix.append(torch.from_numpy(rows[i]), [f"x{i}"], [f"y{i}"])
        ptrs.add(ix._host.data_ptr())
    assert ix.num_items == 3002 and len(ptrs) <= 3
    fi.flush()
    ix2 = TextSearchIndex(tmp_path / "data" / "index.pt")
    qs = torch.from_numpy(rows[::97])
    s1, i1 = ix.search_batch(qs, 10)
    s2, i2 = ix2.search_batch(qs, 10)     # the reload re-normalises the saved rows (search.py:68)
    assert torch.equal(i1, i2) and torch.allclose(s1, s2, atol=1e-6, rtol=0)
    assert ix2.texts[1] == "red backpack" and ix2.image_paths[-1] == "x2999"
    with pytest.raises(FileNotFoundError):
        fi.report_item(tmp_path / "nope.png", "x")
    # token-id descriptions: no location to append, and never mixed with strings in one batch;
    # both rejected before any image is copied
    ids = [49406, 320, 1125, 49407]
    n0 = fi.index.num_items
    with pytest.raises(ValueError):
        fi.report_item(paths[2], ids, location="kantin")
    with pytest.raises(ValueError):
        fi.report_items([paths[2], paths[2]], ["tas", ids])
    assert fi.index.num_items == n0 and not (up / "img2.png").exists()
    assert fi.report_item(paths[2], ids)["description"] == ""
    model.close()
