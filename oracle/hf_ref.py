"""ORACLE -- test infrastructure only. Never imported by the product path.

The reference's own encoder arithmetic: transformers CLIPModel (fp32, CPU),
which models/clip_model.py:59 builds, with PEFT LoRA restated as forward hooks
y += (alpha/r) (x A^T) B^T on every targeted Linear (PEFT matches
target_modules by name suffix, so both towers get adapters; dropout is the
identity at eval; wired at models/clip_model.py:78). Used to generate the
goldens (tests/golden/make_golden.py) and as bench.py's cpu_baseline leg.
"""
from __future__ import annotations

import numpy as np
import torch


def hf_model(cfg, sd, lora):
    from transformers import CLIPConfig, CLIPModel
    hc = CLIPConfig(
        text_config=dict(hidden_size=cfg.text.hidden, num_hidden_layers=cfg.text.layers,
                         num_attention_heads=cfg.text.heads, intermediate_size=cfg.text.mlp,
                         vocab_size=cfg.vocab, max_position_embeddings=cfg.max_pos,
                         eos_token_id=cfg.eos_token_id, bos_token_id=cfg.bos_token_id),
        vision_config=dict(hidden_size=cfg.vision.hidden, num_hidden_layers=cfg.vision.layers,
                           num_attention_heads=cfg.vision.heads, intermediate_size=cfg.vision.mlp,
                           patch_size=cfg.patch, image_size=cfg.image_size),
        projection_dim=cfg.proj_dim)
    m = CLIPModel(hc).eval()
    missing, unexpected = m.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=False)
    assert missing == ["logit_scale"] and not unexpected, (missing, unexpected)
    if lora:
        mods = dict(m.named_modules())
        for k in lora:
            if ".lora_A." not in k:
                continue
            path = k[len("base_model.model."):-len(".lora_A.weight")]
            A = torch.from_numpy(lora[k])
            B = torch.from_numpy(lora[k.replace(".lora_A.", ".lora_B.")])
            s = cfg.lora_scaling

            def hook(mod, inp, out, A=A, B=B, s=s):
                return out + s * ((inp[0] @ A.T) @ B.T)
            mods[path].register_forward_hook(hook)
    return m


def pixel_values(cfg, images_u8):
    from transformers import CLIPImageProcessor
    proc = CLIPImageProcessor(size={"shortest_edge": cfg.image_size},
                              crop_size={"height": cfg.image_size, "width": cfg.image_size})
    return proc(images=list(images_u8), return_tensors="pt")["pixel_values"]


def attention_mask(cfg, ids):
    return torch.from_numpy((np.cumsum(ids == cfg.eos_token_id, 1) <= 1).astype(np.int64))


def encode(model, cfg, pv, ids):
    """reference encode_image/encode_text semantics (clip_model.py:115-116,144-148), batched"""
    with torch.no_grad():
        fi = model.get_image_features(pixel_values=pv).pooler_output
        fi = fi / fi.norm(dim=-1, keepdim=True)
        ft = model.get_text_features(input_ids=torch.from_numpy(ids).long(),
                                     attention_mask=attention_mask(cfg, ids)).pooler_output
        ft = ft / ft.norm(dim=-1, keepdim=True)
    return fi.numpy().astype(np.float32), ft.numpy().astype(np.float32)


def encode_images(model, pv):
    """encode_image semantics only (clip_model.py:115-116), batched: unit rows"""
    with torch.no_grad():
        fi = model.get_image_features(pixel_values=pv).pooler_output
        return fi / fi.norm(dim=-1, keepdim=True)


def encode_texts(model, cfg, ids):
    """encode_text semantics only (clip_model.py:144-148), batched: unit rows"""
    with torch.no_grad():
        ft = model.get_text_features(input_ids=torch.from_numpy(ids).long(),
                                     attention_mask=attention_mask(cfg, ids)).pooler_output
        return ft / ft.norm(dim=-1, keepdim=True)
