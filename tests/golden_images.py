"""Inputs of the image-preprocessing vector set (tests/golden/make_golden.py image_golden):
the reference's committed images (their encoded bytes, ref_images.npz) and the seeded odd-size
synthetic images, in the golden's order."""
import io
import os

import numpy as np

from conftest import GOLDEN, golden

from clip_lora_match_amd import synthetic as syn


def ref_blobs():
    z = np.load(os.path.join(GOLDEN, "ref_images.npz"), allow_pickle=False)
    return [str(n) for n in z["names"]], [z["blob_" + str(k)].tobytes() for k in z["keys"]]


def write_ref_files(tmp_path):
    """the reference's images as files (original names) -> list of paths, golden order"""
    names, blobs = ref_blobs()
    paths = []
    for i, (n, b) in enumerate(zip(names, blobs)):
        p = tmp_path / f"{i:02d}_{os.path.basename(n)}"
        p.write_bytes(b)
        paths.append(p)
    return paths


def pil_images():
    """(labels, PIL RGB images) of the whole set, decoded as the reference decodes
    (Image.open(...).convert("RGB"), models/clip_model.py:105)."""
    from PIL import Image
    g = golden("enc_b32_lora_images.npz")
    _, blobs = ref_blobs()
    pils = [Image.open(io.BytesIO(b)).convert("RGB") for b in blobs]
    odd = syn.odd_images(int(g["odd_seed"]))
    pils += [Image.fromarray(a) for a in odd]
    pils += [Image.fromarray(odd[4]).convert("L").convert("RGB"),
             Image.fromarray(np.dstack([odd[9], odd[9][..., :1]])).convert("RGB")]
    labels = [str(x) for x in g["labels"]]
    assert len(pils) == len(labels)
    return labels, pils


def sha(a) -> str:
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()
