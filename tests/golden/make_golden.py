"""Generate the golden fixtures in tests/golden/ (run in the build container, where
transformers 5.15.0 and the read-only reference at /root/reference exist):

  python tests/golden/make_golden.py

Encoder goldens: transformers.CLIPModel fp32 on CPU (the arithmetic the
reference's models/clip_model.py delegates to, clip_model.py:59,115,144) with
the deterministic synthetic weights of weights.synthetic_state_dict, PEFT LoRA
restated as forward hooks y += (alpha/r) (x A^T) B^T on every targeted Linear
(PEFT matches target_modules by suffix: both towers), `.pooler_output` (the
transformers>=5 spelling of what get_*_features returned in 4.x)
and the L2 normalisation of clip_model.py:116,148. Pixel values come from
transformers' CLIPImageProcessor on the synthetic uint8 images.

Search goldens: the reference's own src/embedding/similarity.py top_k_similar
(imported from /root/reference; it needs only torch) on synthetic normalised
Gaussian fp16-rounded rows/queries, and on the reference's committed
data/index/custom_items_index.pt (copied here as a data fixture).

Image-preprocessing goldens (`images`): the reference's 17 committed images
(data/custom/{images,crops,query_crops}, data/reported/images; 14 distinct files, 36x46 to
1599x899, one palette PNG) and the seeded odd-size synthetic set (synthetic.odd_images, plus
"L" and "RGBA" variants), decoded as the reference decodes (PIL open + convert("RGB"),
models/clip_model.py:105) and preprocessed by transformers' CLIPImageProcessor (its PIL backend,
the reference's resize + centre-crop), then encoded by CLIPModel + LoRA hooks (B/32, the
synthetic weights). Stored: sha256 of the decoded pixels and of the float32 pixel_values, and
the fp32 embeddings. The inputs must reach the GPU box, which has no /root/reference: the 14
files' encoded bytes (930 KB, the smallest lossless form of their pixels) are the input half of
this vector set, in ref_images.npz.

Only inputs' seeds and outputs are stored; the weights are regenerated from
their seeds by the tests.
"""
from __future__ import annotations

import importlib.util
import os
import shutil
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
REF = "/root/reference"

import clip_lora_match_amd as clm  # noqa: E402
from clip_lora_match_amd import synthetic as syn  # noqa: E402
from clip_lora_match_amd import weights as W  # noqa: E402
from oracle import hf_ref as H  # noqa: E402

torch.set_num_threads(8)


def encode(cfg, sd, lora, images, ids):
    m = H.hf_model(cfg, sd, lora)
    return H.encode(m, cfg, H.pixel_values(cfg, images), ids)


def encoder_golden(name, preset, n_img, n_txt, L, lora_on, img_seed=1234, cap_seed=99):
    cfg = clm.get_preset(preset)
    if not lora_on:
        cfg = cfg.with_lora(0, 0.0, ())
    sd = W.synthetic_state_dict(cfg, 0)
    lora = W.synthetic_lora(cfg, 1) if lora_on else None
    images = syn.images_u8(n_img, cfg.image_size, img_seed)
    ids = syn.captions(n_txt, L, cfg.bos_token_id, cfg.eos_token_id, cap_seed)
    fi, ft = encode(cfg, sd, lora, images, ids)
    out = dict(preset=np.array(preset), lora=np.array(int(lora_on)), r=np.array(cfg.lora_r),
               alpha=np.array(cfg.lora_alpha), targets=np.array(",".join(cfg.lora_targets)),
               weight_seed=np.array(0), lora_seed=np.array(1), img_seed=np.array(img_seed),
               cap_seed=np.array(cap_seed), n_img=np.array(n_img), n_txt=np.array(n_txt), L=np.array(L),
               ids=ids, emb_img=fi, emb_txt=ft)
    if lora_on:  # also the base model, so tests can prove LoRA changes the result
        fi0, ft0 = encode(cfg, sd, None, images, ids)
        out.update(emb_img_base=fi0, emb_txt_base=ft0)
    np.savez_compressed(os.path.join(HERE, name), **out)
    print(f"{name}: img {fi.shape} txt {ft.shape}")


REF_IMAGE_DIRS = ("data/custom/images", "data/custom/crops", "data/custom/query_crops", "data/reported/images")


def _sha(a: np.ndarray) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def image_golden():
    """ref_images.npz (inputs) + enc_b32_lora_images.npz (expected outputs); see module doc."""
    import hashlib
    import io
    import glob
    from PIL import Image
    from oracle import clip_ref as R
    from oracle import image_ref as IR
    names, blobs, files = [], {}, []
    for d in REF_IMAGE_DIRS:
        for f in sorted(glob.glob(os.path.join(REF, d, "*"))):
            if f.lower().endswith((".jpg", ".jpeg", ".png")):
                raw = open(f, "rb").read()
                key = hashlib.sha256(raw).hexdigest()[:16]
                blobs.setdefault(key, np.frombuffer(raw, np.uint8))
                names.append(os.path.relpath(f, REF))
                files.append(key)
    np.savez_compressed(os.path.join(HERE, "ref_images.npz"), names=np.array(names), keys=np.array(files),
                        **{"blob_" + k: v for k, v in blobs.items()})
    cfg = clm.get_preset("ViT-B/32")
    sd, lora = W.synthetic_state_dict(cfg, 0), W.synthetic_lora(cfg, 1)
    pils = [Image.open(io.BytesIO(blobs[k].tobytes())).convert("RGB") for k in files]
    odd = syn.odd_images()
    pils += [Image.fromarray(a) for a in odd]
    pils += [Image.fromarray(odd[4]).convert("L").convert("RGB"),
             Image.fromarray(np.dstack([odd[9], odd[9][..., :1]])).convert("RGB")]
    labels = names + [f"odd{i}" for i in range(len(odd))] + ["odd4_L", "odd9_RGBA"]
    from transformers import CLIPImageProcessor
    proc = CLIPImageProcessor(size={"shortest_edge": cfg.image_size},
                              crop_size={"height": cfg.image_size, "width": cfg.image_size})
    pv = np.concatenate([proc(images=[p], return_tensors="np")["pixel_values"] for p in pils]).astype(np.float32)
    dec = [np.asarray(p, np.uint8) for p in pils]
    for i, a in enumerate(dec):   # the oracle restatement must reproduce the processor bit for bit
        mine = R.preprocess_u8(IR.resize_crop_u8(a, cfg.image_size)[None], cfg.mean, cfg.std)[0]
        assert mine.tobytes() == pv[i].tobytes(), labels[i]
    m = H.hf_model(cfg, sd, lora)
    embs = []
    with torch.no_grad():
        for i in range(0, len(pv), 8):
            f = m.get_image_features(pixel_values=torch.from_numpy(pv[i:i + 8])).pooler_output
            embs.append((f / f.norm(dim=-1, keepdim=True)).numpy())
    np.savez_compressed(os.path.join(HERE, "enc_b32_lora_images.npz"), labels=np.array(labels),
                        n_ref=np.array(len(names)), hw=np.array([a.shape[:2] for a in dec], np.int64),
                        dec_sha=np.array([_sha(a) for a in dec]), pv_sha=np.array([_sha(p) for p in pv]),
                        emb_img=np.concatenate(embs).astype(np.float32), odd_seed=np.array(4242))
    print(f"ref_images.npz: {len(blobs)} files for {len(names)} names; enc_b32_lora_images.npz: {len(labels)} images")


def _load_ref_similarity():
    spec = importlib.util.spec_from_file_location("ref_similarity", os.path.join(REF, "src/embedding/similarity.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def search_golden():
    sim = _load_ref_similarity()
    n, nq, dim = 4096, 64, 512
    rows = syn.gaussian_rows(n, dim, seed=7, fp16=True)
    qs = syn.gaussian_rows(nq, dim, seed=8, fp16=True)
    E = torch.from_numpy(rows.astype(np.float32))
    out = dict(n=np.array(n), nq=np.array(nq), dim=np.array(dim), row_seed=np.array(7), q_seed=np.array(8))
    for k in (1, 5, 10, 50):
        vals = np.zeros((nq, k), np.float32)
        idx = np.zeros((nq, k), np.int64)
        for i in range(nq):
            v, ix = sim.top_k_similar(torch.from_numpy(qs[i].astype(np.float32)), E, k)
            vals[i], idx[i] = v.numpy(), ix.numpy()
        out[f"vals_k{k}"] = vals
        out[f"idx_k{k}"] = idx
    cs = sim.cosine_similarity(torch.from_numpy(qs[0].astype(np.float32)), E).numpy()
    out["cos_q0"] = cs.astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "search_gauss.npz"), **out)
    print("search_gauss.npz")

    # the reference's committed 6x512 index (data fixture) + self-query top-3
    src = os.path.join(REF, "data/index/custom_items_index.pt")
    dst = os.path.join(HERE, "custom_items_index.pt")
    shutil.copyfile(src, dst)
    obj = torch.load(dst, map_location="cpu", weights_only=True)
    Ec = obj["embeddings"].float()
    vals = np.zeros((Ec.shape[0], 3), np.float32)
    idx = np.zeros((Ec.shape[0], 3), np.int64)
    for i in range(Ec.shape[0]):
        v, ix = sim.top_k_similar(Ec[i], Ec, 3)
        vals[i], idx[i] = v.numpy(), ix.numpy()
    np.savez_compressed(os.path.join(HERE, "custom_index_top3.npz"), vals=vals, idx=idx)
    print("custom_index_top3.npz", idx.tolist())


def search_fp32_golden():
    """fp32 (not fp16-representable) rows and queries through the reference's own
    similarity.top_k_similar / cosine_similarity: Gaussian and tightly clustered sets."""
    sim = _load_ref_similarity()
    dim = 512
    gauss_rows, gauss_q, clus, clus_q = syn.fp32_search_inputs()
    out = dict(dim=np.array(dim))   # inputs are regenerated from their seeds (fp32_search_inputs)
    for name, rows, qs in (("gauss", gauss_rows, gauss_q), ("clus", clus, clus_q)):
        E = torch.from_numpy(rows)
        for k in (1, 5, 10, 50):
            vals = np.zeros((qs.shape[0], k), np.float32)
            idx = np.zeros((qs.shape[0], k), np.int64)
            for i in range(qs.shape[0]):
                v, ix = sim.top_k_similar(torch.from_numpy(qs[i]), E, k)
                vals[i], idx[i] = v.numpy(), ix.numpy()
            out[f"{name}_vals_k{k}"] = vals
            out[f"{name}_idx_k{k}"] = idx
        out[f"{name}_cos_q0"] = sim.cosine_similarity(torch.from_numpy(qs[0]), E).numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, "search_fp32.npz"), **out)
    print("search_fp32.npz")


def search_large_golden():
    """k > 1024 (up to k = N and past it: torch.topk takes min(k, N)) and dim > 1024 through the
    reference's own similarity.top_k_similar: the first 4 queries of the fp32 Gaussian and clustered
    sets at k = 1025, 2000, 4096 = N (indices fit int16), and 8 queries on 2048 Gaussian fp32 rows of
    dim 1536 at k = 5, 50, 1500."""
    sim = _load_ref_similarity()
    gauss_rows, gauss_q, clus, clus_q = syn.fp32_search_inputs()
    out = {}
    for name, rows, qs in (("gauss", gauss_rows, gauss_q), ("clus", clus, clus_q)):
        E = torch.from_numpy(rows)
        for k in (1025, 2000, 4096):
            vals = np.zeros((4, k), np.float32)
            idx = np.zeros((4, k), np.int16)
            for i in range(4):
                v, ix = sim.top_k_similar(torch.from_numpy(qs[i]), E, k)
                vals[i], idx[i] = v.numpy(), ix.numpy().astype(np.int16)
            out[f"{name}_vals_k{k}"] = vals
            out[f"{name}_idx_k{k}"] = idx
    wide_rows = syn.gaussian_rows(2048, 1536, seed=31, fp16=False)
    wide_q = syn.gaussian_rows(8, 1536, seed=32, fp16=False)
    E = torch.from_numpy(wide_rows)
    for k in (5, 50, 1500):
        vals = np.zeros((8, k), np.float32)
        idx = np.zeros((8, k), np.int16)
        for i in range(8):
            v, ix = sim.top_k_similar(torch.from_numpy(wide_q[i]), E, k)
            vals[i], idx[i] = v.numpy(), ix.numpy().astype(np.int16)
        out[f"wide_vals_k{k}"] = vals
        out[f"wide_idx_k{k}"] = idx
    out["wide_seeds"] = np.array([31, 32])
    np.savez_compressed(os.path.join(HERE, "search_large_k.npz"), **out)
    print("search_large_k.npz")


if __name__ == "__main__":
    which = sys.argv[1:] or ["tiny", "b32", "b32_64", "l14", "search", "search_fp32", "search_large", "images"]
    if "tiny" in which:
        encoder_golden("enc_tiny_lora.npz", "tiny", 4, 4, 16, True)
    if "b32" in which:
        encoder_golden("enc_b32_lora.npz", "ViT-B/32", 4, 4, 77, True)
    if "b32_64" in which:   # the parity set bench.py scores its timed dtype against
        encoder_golden("enc_b32_lora_64.npz", "ViT-B/32", 64, 64, 77, True, img_seed=5000, cap_seed=5001)
    if "l14" in which:
        encoder_golden("enc_l14_lora.npz", "ViT-L/14@336", 2, 2, 77, True)
    if "search" in which:
        search_golden()
    if "search_fp32" in which:
        search_fp32_golden()
    if "search_large" in which:
        search_large_golden()
    if "images" in which:
        image_golden()
