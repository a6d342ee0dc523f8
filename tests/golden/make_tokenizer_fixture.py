"""Generate the small synthetic CLIP BPE vocabulary in tests/golden/clip_bpe/ (the real
49408-token CLIP vocabulary is not available offline):

  python tests/golden/make_tokenizer_fixture.py

A byte-level BPE is trained on a fixed corpus of lost-and-found item descriptions with the
CLIP pre-tokenisation (lowercase, letters / single digits / punctuation runs, "</w>" word
ends): 256 byte symbols, their 256 "</w>" forms, then one token per merge in merge order;
<|startoftext|> / <|endoftext|> sit at CLIP's ids 49406 / 49407 so the ids drive the
B/32 text tower unchanged. tests/test_tokenizer.py checks clip_lora_match_amd.tokenizer
against transformers' CLIPTokenizer built from these same files.
"""
from __future__ import annotations

import json
import os
import sys
from collections import Counter

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from clip_lora_match_amd.tokenizer import _SPLIT, ClipBPETokenizer, bytes_to_unicode  # noqa: E402

COLORS = ["red", "black", "blue", "white", "brown", "green", "grey", "pink", "merah", "hitam", "biru", "putih"]
ITEMS = ["backpack", "wallet", "phone", "umbrella", "jacket", "laptop bag", "water bottle", "keys", "tas ransel",
         "dompet", "kunci motor", "payung", "jaket", "botol minum", "earphones", "student card", "kartu mahasiswa"]
PLACES = ["library", "canteen", "parking lot", "gedung A", "lab komputer", "masjid", "lecture hall 3",
          "perpustakaan", "kantin", "lobby"]


def corpus():
    lines = []
    for i, c in enumerate(COLORS):
        for j, it in enumerate(ITEMS):
            p = PLACES[(i * 7 + j) % len(PLACES)]
            lines.append(f"{c} {it}, ditemukan di {p}")
            lines.append(f"A {c} {it} found near the {p} at {8 + (i + j) % 12}:{(i * j) % 60:02d}")
            lines.append(f"{it} warna {c} dengan stiker #{i}{j} -- isi: KTP & SIM (it's mine, don't lose it!)")
    lines += ["café crème — naïve résumé", "ümlaut Straße", "日本語のテキスト", "emoji 🎒🔑", "tab\tand\nnewline"]
    return lines


def train(n_merges: int = 600):
    bmap = bytes_to_unicode()
    words = Counter()
    for line in corpus():
        for piece in _SPLIT.findall(ClipBPETokenizer.normalize(line)):
            sym = [bmap[b] for b in piece.encode("utf-8")]
            sym[-1] += "</w>"
            words[tuple(sym)] += 1
    merges = []
    for _ in range(n_merges):
        pairs = Counter()
        for w, c in words.items():
            for a, b in zip(w, w[1:]):
                pairs[(a, b)] += c
        if not pairs:
            break
        best = min(pairs.items(), key=lambda kv: (-kv[1], kv[0]))[0]
        merges.append(best)
        nw = Counter()
        for w, c in words.items():
            out, i = [], 0
            while i < len(w):
                if i < len(w) - 1 and (w[i], w[i + 1]) == best:
                    out.append(w[i] + w[i + 1])
                    i += 2
                else:
                    out.append(w[i])
                    i += 1
            nw[tuple(out)] += c
        words = nw
    vocab = {}
    for ch in bmap.values():
        vocab[ch] = len(vocab)
    for ch in bmap.values():
        vocab[ch + "</w>"] = len(vocab)
    for a, b in merges:
        if a + b not in vocab:
            vocab[a + b] = len(vocab)
    vocab["<|startoftext|>"] = 49406
    vocab["<|endoftext|>"] = 49407
    return vocab, merges


if __name__ == "__main__":
    vocab, merges = train()
    out = os.path.join(HERE, "clip_bpe")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "vocab.json"), "w", encoding="utf-8") as f:
        json.dump(vocab, f, ensure_ascii=False)
    with open(os.path.join(out, "merges.txt"), "w", encoding="utf-8") as f:
        f.write("#version: 0.2\n")
        for a, b in merges:
            f.write(f"{a} {b}\n")
    print(f"clip_bpe: {len(vocab)} tokens, {len(merges)} merges")
