"""Where does the bf16 score error come from? The 64 + 64 parity set
(tests/golden/enc_b32_lora_64.npz, transformers fp32 goldens) encoded with each tower in fp16 or
bf16 operands, combined per block of the 128 x 128 score matrix: img.img, img.txt, txt.txt max
|error| for every (vision dtype, text dtype) pair, plus the 1 - cos per tower.
usage: python tools/bf16_bisect.py -> one JSON line per combination"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import clip_lora_match_amd as clm  # noqa: E402
from clip_lora_match_amd import synthetic as syn  # noqa: E402
from clip_lora_match_amd import weights as W  # noqa: E402
from clip_lora_match_amd.engine import ClipLoraModel  # noqa: E402

cfg = clm.get_preset("ViT-B/32")
dev = torch.device("cuda", 0)
g = np.load(os.path.join(REPO, "tests", "golden", "enc_b32_lora_64.npz"), allow_pickle=False)
imgs = torch.from_numpy(syn.images_u8(int(g["n_img"]), cfg.image_size, int(g["img_seed"]))).to(dev)
ids = torch.from_numpy(g["ids"]).to(dev)
ri, rt = g["emb_img"].astype(np.float64), g["emb_txt"].astype(np.float64)
emb = {}
for dt in ("float16", "bfloat16"):
    m = ClipLoraModel(cfg, device=dev, compute_dtype=dt, max_batch=64)
    m.load_tensors(W.synthetic_state_dict(cfg, 0))
    m.load_tensors(W.synthetic_lora(cfg, 1))
    m.finalize()
    emb[dt] = (m.encode_pixels(imgs).double().cpu().numpy(), m.encode_ids(ids).double().cpu().numpy())
    m.close()


def one_minus_cos(a, b):
    return float(np.max(1 - np.sum(a * b, 1) / (np.linalg.norm(a, axis=1) * np.linalg.norm(b, axis=1))))


for vd in ("float16", "bfloat16"):
    for td in ("float16", "bfloat16"):
        a, b = emb[vd][0], emb[td][1]
        print(json.dumps({"vision": vd, "text": td,
                          "img_img": float(np.abs(a @ a.T - ri @ ri.T).max()),
                          "img_txt": float(np.abs(a @ b.T - ri @ rt.T).max()),
                          "txt_txt": float(np.abs(b @ b.T - rt @ rt.T).max()),
                          "vision_1mcos": one_minus_cos(a, ri), "text_1mcos": one_minus_cos(b, rt)}), flush=True)
