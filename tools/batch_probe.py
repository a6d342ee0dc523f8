"""Diagnostic: does an image's embedding depend on the batch it is encoded in?
Encodes the synthetic images 32..36 as one batch of 5 and 35..36 as a batch of 2 (fp16 B/32 +
merged LoRA, as tests/dist_gpu_worker.py) and prints the bit difference of the shared rows.
Run once per environment given on the command line (NAME:VAR=val,...), each in a child."""
import json
import os
import subprocess
import sys

CODE = r'''
import os, sys, json, numpy as np, torch
sys.path.insert(0, os.getcwd())
import clip_lora_match_amd as clm
from clip_lora_match_amd import synthetic as syn, weights as W
from clip_lora_match_amd.engine import ClipLoraModel
cfg = clm.get_preset("ViT-B/32")
dt = os.environ.get("DT", "float16")
m = ClipLoraModel(cfg, compute_dtype=dt, max_batch=8)
m.load_tensors(W.synthetic_state_dict(cfg, 0)); m.load_tensors(W.synthetic_lora(cfg, 1)); m.finalize()
imgs = np.stack(list(syn.images_u8(37, cfg.image_size, 300)))
enc = lambda a, b: m.encode_pixels(torch.from_numpy(imgs[a:b]).cuda()).cpu()
e5 = enc(32, 37); e2 = enc(35, 37); e1 = enc(36, 37); e5b = enc(32, 37); e8 = enc(29, 37)
d = lambda x, y: float((x.float() - y.float()).abs().max())
print(json.dumps({"b5_vs_b2": d(e5[3:], e2), "b5_vs_b1": d(e5[4:], e1), "b2_vs_b1": d(e2[1:], e1),
                  "b5_repeat": d(e5, e5b), "b8_vs_b5": d(e8[3:], e5)}))
'''
for spec in sys.argv[1:] or ["default:"]:
    name, _, kv = spec.partition(":")
    env = dict(os.environ)
    for item in filter(None, kv.split(",")):
        k, _, v = item.partition("=")
        env[k] = v
    out = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=300)
    print(name, out.stdout.strip().splitlines()[-1] if out.returncode == 0 else out.stderr[-1500:], flush=True)
