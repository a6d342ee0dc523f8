"""How much the two towers overlap in encode_pair: per-step wall time of the image tower alone,
the text tower alone (both eager on one stream), their sum, and encode_pair (two streams, graph
replay and eager), interleaved in one process. B/32 + LoRA merged, bf16, batch 256.
usage: python tools/tower_overlap.py -> one JSON line"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import clip_lora_match_amd as clm  # noqa: E402
from clip_lora_match_amd import synthetic as syn, weights as W  # noqa: E402
from clip_lora_match_amd.engine import ClipLoraModel  # noqa: E402

cfg = clm.get_preset("ViT-B/32")
dev = torch.device("cuda", 0)
B = 256
m = ClipLoraModel(cfg, device=dev, compute_dtype="bfloat16", lora_mode="merged", max_batch=B)
m.load_tensors(W.synthetic_state_dict(cfg, 0))
m.load_tensors(W.synthetic_lora(cfg, 1))
m.finalize()
imgs = torch.from_numpy(syn.images_u8(B, cfg.image_size, 1234)).to(dev)
ids = torch.from_numpy(syn.captions(B, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 99)).to(dev)
oi = torch.empty((B, cfg.proj_dim), device=dev)
ot = torch.empty((B, cfg.proj_dim), device=dev)
fns = {"image": lambda: m.encode_pixels(imgs, out=oi), "text": lambda: m.encode_ids(ids, out=ot),
       "pair_graph": lambda: m.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=True),
       "pair_eager": lambda: m.encode_pair(imgs, ids, out_img=oi, out_txt=ot, graph=False)}
res = {k: [] for k in fns}
for rnd in range(6):
    for k, f in fns.items():
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            f()
        torch.cuda.synchronize()
        if rnd:
            res[k].append((time.perf_counter() - t0) / 10 * 1e3)
med = {k: round(sorted(v)[len(v) // 2], 3) for k, v in res.items()}
med["sum_alone"] = round(med["image"] + med["text"], 3)
print(json.dumps({"ms_per_step": med}), flush=True)
