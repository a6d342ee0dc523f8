"""Diagnostic: tiny-tower batch invariance with the GEMM tile config forced (CLM_GEMM_CFG,
read once per process, so one subprocess per config)."""
import os
import subprocess
import sys

CHILD = r'''
import sys, torch
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from conftest import synthetic
from clip_lora_match_amd.engine import ClipLoraModel
from clip_lora_match_amd import synthetic as syn
cfg, sd, lora = synthetic("tiny", True)
m = ClipLoraModel(cfg, compute_dtype="float16", lora_mode="merged", max_batch=16)
m.load_tensors(sd); m.load_tensors(lora); m.finalize()
imgs = torch.from_numpy(syn.images_u8(7, cfg.image_size, 51)).cuda()
ids = torch.from_numpy(syn.captions(7, cfg.max_pos, cfg.bos_token_id, cfg.eos_token_id, 52)).cuda()
fi, ft = m.encode_pixels(imgs), m.encode_ids(ids)
res = []
for a, b in ((0, 3), (3, 7), (2, 3), (6, 7)):
    si = m.encode_pixels(imgs[a:b]); st = m.encode_ids(ids[a:b])
    res.append(f"img[{a}:{b}] {'ok' if torch.equal(si, fi[a:b]) else 'DIFF %.2e' % (si - fi[a:b]).abs().max().item()}")
    res.append(f"txt[{a}:{b}] {'ok' if torch.equal(st, ft[a:b]) else 'DIFF %.2e' % (st - ft[a:b]).abs().max().item()}")
print(" ".join(res))
'''

for cfg in ["", "0", "1", "2", "3", "4", "5", "6", "7", "8", "9", "10"]:
    env = dict(os.environ)
    if cfg:
        env["CLM_GEMM_CFG"] = cfg
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=300)
    print(f"cfg={cfg or 'auto'}:", r.stdout.strip() or r.stderr.strip()[-400:], flush=True)
