"""CLIP byte-level BPE tokenizer (the text half of the CLIPProcessor that
models/clip_model.py:133-138 and src/embedding/embed_text.py:35-41 call), host-side.

Restates the published CLIP tokenizer as transformers 5.15 builds it on the `tokenizers`
library (TF/models/clip/tokenization_clip.py:56-122; OpenAI's simple_tokenizer.py):

  normalise    NFC, every whitespace run -> " ", lowercase
  pre-split    regex  <|startoftext|> | <|endoftext|> | 's|'t|'re|'ve|'m|'ll|'d
               | \\p{L}+ | \\p{N} (ONE digit) | [^\\s\\p{L}\\p{N}]+   (whitespace dropped)
  bytes        each piece's UTF-8 bytes -> GPT-2 byte-to-unicode characters
  BPE          symbols = characters, the last one suffixed "</w>"; repeatedly merge the
               adjacent pair with the lowest merges.txt rank; unknown symbols -> <|endoftext|>
  wrap         <|startoftext|> ids <|endoftext|>; truncation keeps the first max_length-2
               content ids; padding=True pads to the batch's longest row with <|endoftext|>

Files: vocab.json (token -> id) and merges.txt ("a b" per line, an optional "#version"
header), the layout `CLIPTokenizer.from_pretrained` reads. Parity is checked against
transformers' CLIPTokenizer built from the same files (tests/test_tokenizer.py).
"""
from __future__ import annotations

import json
import unicodedata
from functools import lru_cache
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Tuple, Union

import regex

_SPLIT = regex.compile(
    r"""<\|startoftext\|>|<\|endoftext\|>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]|[^\s\p{L}\p{N}]+""")
_WS = regex.compile(r"\s+")
BOS, EOS = "<|startoftext|>", "<|endoftext|>"


@lru_cache(maxsize=1)
def bytes_to_unicode() -> Dict[int, str]:
    """GPT-2's reversible byte -> printable-unicode map used by ByteLevel pre-tokenisation."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


def load_merges(path: Union[str, Path]) -> List[Tuple[str, str]]:
    out = []
    with open(path, "r", encoding="utf-8") as f:
        for i, line in enumerate(f):
            line = line.rstrip("\n")
            if (i == 0 and line.startswith("#version")) or not line.strip():
                continue
            a, b = line.split(" ")
            out.append((a, b))
    return out


class ClipBPETokenizer:
    def __init__(self, vocab: Union[str, Path, Dict[str, int]], merges: Union[str, Path, Sequence[Tuple[str, str]]],
                 model_max_length: int = 77):
        if not isinstance(vocab, dict):
            with open(vocab, "r", encoding="utf-8") as f:
                vocab = json.load(f)
        if not isinstance(merges, (list, tuple)):
            merges = load_merges(merges)
        self.encoder: Dict[str, int] = dict(vocab)
        self.decoder = {v: k for k, v in self.encoder.items()}
        self.ranks = {tuple(m): i for i, m in enumerate(merges)}
        self.byte_map = bytes_to_unicode()
        self.byte_unmap = {v: k for k, v in self.byte_map.items()}
        for tok in (BOS, EOS):
            if tok not in self.encoder:
                raise ValueError(f"vocabulary has no {tok}")
        self.bos_token_id = self.encoder[BOS]
        self.eos_token_id = self.encoder[EOS]
        self.pad_token_id = self.eos_token_id
        self.unk_token_id = self.eos_token_id
        self.model_max_length = model_max_length
        self._cache: Dict[str, List[int]] = {}

    @classmethod
    def from_dir(cls, path: Union[str, Path], model_max_length: int = 77) -> "ClipBPETokenizer":
        p = Path(path)
        return cls(p / "vocab.json", p / "merges.txt", model_max_length)

    # ------------------------------------------------------------------ BPE --
    def _bpe(self, piece: str) -> List[int]:
        hit = self._cache.get(piece)
        if hit is not None:
            return hit
        word = [self.byte_map[b] for b in piece.encode("utf-8")]
        word[-1] = word[-1] + "</w>"
        while len(word) > 1:
            best, best_rank = -1, None
            for i in range(len(word) - 1):
                r = self.ranks.get((word[i], word[i + 1]))
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = i, r
            if best < 0:
                break
            a, b = word[best], word[best + 1]
            merged, i = [], 0
            while i < len(word):   # merge every occurrence of (a, b), left to right
                if i < len(word) - 1 and word[i] == a and word[i + 1] == b:
                    merged.append(a + b)
                    i += 2
                else:
                    merged.append(word[i])
                    i += 1
            word = merged
        ids = [self.encoder.get(s, self.unk_token_id) for s in word]
        if len(self._cache) < 100_000:
            self._cache[piece] = ids
        return ids

    @staticmethod
    def normalize(text: str) -> str:
        return _WS.sub(" ", unicodedata.normalize("NFC", text)).lower()

    def encode(self, text: str, add_special_tokens: bool = True, max_length: Optional[int] = None,
               truncation: bool = False) -> List[int]:
        ids: List[int] = []
        for piece in _SPLIT.findall(self.normalize(text)):
            if piece in (BOS, EOS):
                ids.append(self.encoder[piece])
            else:
                ids.extend(self._bpe(piece))
        if truncation and max_length is not None:
            ids = ids[: max(0, max_length - (2 if add_special_tokens else 0))]
        return [self.bos_token_id] + ids + [self.eos_token_id] if add_special_tokens else ids

    def decode(self, ids: Sequence[int], skip_special_tokens: bool = True) -> str:
        toks = [self.decoder.get(int(i), "") for i in ids]
        if skip_special_tokens:
            toks = [t for t in toks if t not in (BOS, EOS)]
        out = bytearray()
        for c in "".join(toks).replace("</w>", " "):   # word ends become spaces (tokenization_clip.py:136)
            out += b" " if c == " " else bytes([self.byte_unmap[c]]) if c in self.byte_unmap else c.encode()
        return out.decode("utf-8", "replace").strip()

    def __call__(self, text: Union[str, Sequence[str]], padding: Union[bool, str] = False, truncation: bool = False,
                 max_length: Optional[int] = None, return_tensors: Optional[str] = None, **kw):
        """{"input_ids", "attention_mask"} like CLIPTokenizer.__call__; padding=True or "longest"
        pads to the batch's longest row, "max_length" to max_length."""
        batch = [text] if isinstance(text, str) else list(text)
        if truncation and max_length is None:
            max_length = self.model_max_length
        rows = [self.encode(t, True, max_length, truncation) for t in batch]
        if padding in (True, "longest"):
            width = max((len(r) for r in rows), default=0)
        elif padding == "max_length":
            width = max_length or self.model_max_length
        else:
            width = None
        masks = [[1] * len(r) for r in rows]
        if width is not None:
            masks = [m + [0] * (width - len(m)) for m in masks]
            rows = [r + [self.pad_token_id] * (width - len(r)) for r in rows]
        if return_tensors == "pt":
            import torch
            return {"input_ids": torch.tensor(rows, dtype=torch.long), "attention_mask": torch.tensor(masks)}
        if return_tensors == "np":
            import numpy as np
            return {"input_ids": np.asarray(rows, np.int64), "attention_mask": np.asarray(masks, np.int64)}
        if isinstance(text, str):
            return {"input_ids": rows[0], "attention_mask": masks[0]}
        return {"input_ids": rows, "attention_mask": masks}


__all__ = ["ClipBPETokenizer", "bytes_to_unicode", "load_merges"]
