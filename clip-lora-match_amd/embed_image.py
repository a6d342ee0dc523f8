"""Drop-in for src/embedding/embed_image.py (embed_image :22-54,
embed_images_batch :57-98): batched image embeddings on the GPU encoder.
Batches go through whole (up to the context's max_batch per launch); the
reference's batch_size argument only bounds host-side decode memory."""
from __future__ import annotations

from pathlib import Path
from typing import Union

import torch

from .clip_model import _encode_images


def embed_image(model, processor, image, device: Union[str, torch.device] = "cpu",
                normalize: bool = True) -> torch.Tensor:
    """Returns (d,) float32 on the CPU."""
    if not hasattr(image, "size") and not isinstance(image, (str, Path)) and not hasattr(image, "shape"):
        raise TypeError("image must be a path, PIL image or uint8 array")
    feats = _encode_images([image], model, processor, normalize=normalize)
    return feats.squeeze(0).detach().cpu()


def embed_images_batch(model, processor, images: list, device: Union[str, torch.device] = "cpu",
                       normalize: bool = True, batch_size: int = 16) -> torch.Tensor:
    """Returns (N, d) float32 on the CPU; torch.empty(0) for an empty list."""
    if not images:
        return torch.empty(0)
    chunk = max(int(batch_size), getattr(model, "max_batch", batch_size))
    outs = []
    for i in range(0, len(images), chunk):
        outs.append(_encode_images(images[i:i + chunk], model, processor, normalize=normalize).cpu())
    return torch.cat(outs, dim=0)
