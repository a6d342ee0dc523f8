"""Drop-in for src/embedding/embed_text.py (embed_text :11-60): str -> (d,),
list -> (N, d), CPU float32. Captions are token ids padded with EOS to the
longest row (padding=True, truncation=True, max_length=model_max_length);
strings need a local CLIP BPE vocabulary (processor.ClipProcessor)."""
from __future__ import annotations

from typing import List, Union

import torch


def embed_text(model, processor, text: Union[str, List[str], List[int], List[List[int]], torch.Tensor],
               device: Union[str, torch.device] = "cpu", normalize: bool = True) -> torch.Tensor:
    single = isinstance(text, str) or (isinstance(text, (list, tuple)) and len(text) > 0
                                       and isinstance(text[0], int))
    if isinstance(text, torch.Tensor):
        single = text.dim() == 1
    ids = processor.token_ids([text] if isinstance(text, str) else text)
    feats = model.encode_ids(ids.to(model.device), normalize=normalize).cpu()
    return feats.squeeze(0) if single else feats
