"""Images of any size through the product path (SURVEY §8(a) A8 + A4/A6): host decode ->
clm_resize_crop (PIL-exact bicubic shortest-edge resize + centre crop on the GPU) -> uint8 encode.

Inputs: the reference's 17 committed images (data/custom/*, data/reported/images; 36x46 to
1599x899, one palette PNG) and the seeded odd-size synthetic set. Checked against
  * the CPU oracle (oracle/image_ref.py, pinned to PIL and CLIPImageProcessor): crops bit for bit;
  * CLIPImageProcessor's pixel_values (sha256 in the golden): bit for bit after normalisation;
  * transformers CLIPModel + LoRA embeddings of those pixel_values (B/32, synthetic weights):
    fp16 operands, scores <= 1e-3 and 1 - cos <= 1e-5 (north_star's bar).
"""
import ctypes

import numpy as np
import pytest
import torch
import yaml

from conftest import golden
from golden_images import pil_images, sha, write_ref_files

import clip_lora_match_amd as clm
from clip_lora_match_amd import _capi
from clip_lora_match_amd.clip_model import encode_image, load_clip_model
from clip_lora_match_amd.embed_image import embed_image, embed_images_batch
from clip_lora_match_amd.processor import ClipProcessor
from oracle import clip_ref as R
from oracle import image_ref as IR

pytestmark = pytest.mark.gpu
SCORE_TOL, COS_TOL = 1e-3, 1e-5


def _check(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    cos = np.sum(a * b, -1) / (np.linalg.norm(a, axis=-1) * np.linalg.norm(b, axis=-1))
    assert np.max(1 - cos) <= COS_TOL, f"1 - cos {np.max(1 - cos):.3e}"
    err = np.max(np.abs(a @ a.T - b @ b.T))
    assert err <= SCORE_TOL, f"score err {err:.3e}"
    return float(np.max(1 - cos)), float(err)


def _proc():
    return ClipProcessor(clm.get_preset("ViT-B/32"))


def test_resize_crop_is_clip_image_processor_bit_exact():
    g = golden("enc_b32_lora_images.npz")
    cfg = clm.get_preset("ViT-B/32")
    labels, pils = pil_images()
    proc = _proc()
    crops = proc.images_u8(pils, "cuda").cpu().numpy()
    pv = proc.pixel_values(pils).numpy()
    assert crops.shape == (len(pils), 224, 224, 3) and pv.shape == (len(pils), 3, 224, 224)
    for i, (lab, im) in enumerate(zip(labels, pils)):
        a = np.asarray(im, np.uint8)
        assert np.array_equal(crops[i], IR.resize_crop_u8(a, cfg.image_size)), lab
        assert sha(R.preprocess_u8(crops[i][None], cfg.mean, cfg.std)[0]) == str(g["pv_sha"][i]), lab
        assert sha(pv[i]) == str(g["pv_sha"][i]), lab


@pytest.mark.parametrize("seed", range(3))
def test_resize_crop_random_sizes_vs_oracle(seed):
    """mixed sizes in one launch (tiny, strips, up- and down-scales), one call vs the oracle"""
    rng = np.random.default_rng(100 + seed)
    imgs = []
    for _ in range(9):
        h, w = (int(v) for v in rng.integers(1, 900, 2))
        if rng.random() < 0.3:
            h = int(rng.integers(1, 20))
        imgs.append(rng.integers(0, 256, (h, w, 3), dtype=np.uint8))
    imgs.append(rng.integers(0, 256, (224, 224, 3), dtype=np.uint8))   # identity size in a mixed batch
    out = _proc().images_u8(imgs, "cuda").cpu().numpy()
    for i, a in enumerate(imgs):
        assert np.array_equal(out[i], IR.resize_crop_u8(a, 224)), a.shape


def test_resize_crop_c_abi_host_buffers_and_errors():
    """clm_resize_crop on host pointers (staged through the device) == device pointers; bad sizes
    raise ValueError (CLM_E_ARG)."""
    L = _capi.lib()
    rng = np.random.default_rng(7)
    imgs = [rng.integers(0, 256, (h, w, 3), dtype=np.uint8) for h, w in ((300, 200), (31, 517), (5, 5))]
    flat = np.concatenate([a.reshape(-1) for a in imgs])
    offs = np.array([0, imgs[0].size, imgs[0].size + imgs[1].size], np.int64)
    hw = np.array([a.shape[:2] for a in imgs], np.int32).reshape(-1)
    out = np.zeros((3, 224, 224, 3), np.uint8)
    P64, P32 = ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32)
    _capi.check(L.clm_resize_crop(0, flat.ctypes.data, offs.ctypes.data_as(P64), hw.ctypes.data_as(P32), 3, 224,
                                  out.ctypes.data, None))
    for i, a in enumerate(imgs):
        assert np.array_equal(out[i], IR.resize_crop_u8(a, 224))
    dev = _proc().images_u8(imgs, "cuda").cpu().numpy()
    assert np.array_equal(dev, out)
    bad = np.array([0, 5, 5, 5, 5, 5], np.int32)
    with pytest.raises(ValueError):
        _capi.check(L.clm_resize_crop(0, flat.ctypes.data, offs.ctypes.data_as(P64), bad.ctypes.data_as(P32), 3,
                                      224, out.ctypes.data, None))
    # a 1 x 10^7 strip: its long side would resize to 2.24e9 pixels (past int) -- refused before any
    # byte is read, as PIL refuses it
    strip = np.array([1, 10_000_000], np.int32)
    with pytest.raises(ValueError):
        _capi.check(L.clm_resize_crop(0, flat.ctypes.data, offs.ctypes.data_as(P64), strip.ctypes.data_as(P32), 1,
                                      224, out.ctypes.data, None))


def _load(tmp_path, max_batch=8):
    cfg = {"model": {"name": "openai/clip-vit-base-patch32", "device": "cpu", "dtype": "float32"},
           "preprocess": {"image_size": 224}}
    p = tmp_path / "clip_config.yaml"
    p.write_text(yaml.safe_dump(cfg))
    return load_clip_model(p, use_lora=True, lora_weights_path="synthetic", weights_dir="synthetic",
                           max_batch=max_batch)


def test_encode_image_reference_files_vs_golden(tmp_path):
    """encode_image(path) -- the reference's per-call API -- on the reference's own image files,
    and embed_images_batch over the whole set, against CLIPModel + LoRA on CLIPImageProcessor's
    pixel_values."""
    g = golden("enc_b32_lora_images.npz")
    n_ref = int(g["n_ref"])
    model, proc, dev = _load(tmp_path)
    paths = write_ref_files(tmp_path)
    assert len(paths) == n_ref
    per_call = np.stack([encode_image(p, model, proc, dev).numpy() for p in paths])
    cos_e, score_e = _check(per_call, g["emb_img"][:n_ref])
    print(f"\nreference images, encode_image fp16: max 1-cos {cos_e:.2e}, max score err {score_e:.2e}")
    _, pils = pil_images()
    batch = embed_images_batch(model, proc, list(paths) + pils[n_ref:], dev, batch_size=8)
    assert batch.shape == (len(pils), 512)
    cos_b, score_b = _check(batch.numpy(), g["emb_img"])
    print(f"all {len(pils)} images, embed_images_batch fp16: max 1-cos {cos_b:.2e}, max score err {score_b:.2e}")
    # the single-image API on a PIL input of odd size
    e = embed_image(model, proc, pils[n_ref + 1], dev)
    _check(e[None].numpy(), g["emb_img"][n_ref + 1:n_ref + 2])
    model.close()
