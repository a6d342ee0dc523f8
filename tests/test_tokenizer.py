"""The host CLIP BPE tokenizer (clip_lora_match_amd/tokenizer.py) against transformers'
CLIPTokenizer built from the same vocab.json / merges.txt (tests/golden/clip_bpe, made by
tests/golden/make_tokenizer_fixture.py). transformers 5.15 is the reference's tokenizer
implementation (clip_model.py:133-138 via CLIPProcessor; embed_text.py:35-41)."""
import json
import os

import pytest

from conftest import GOLDEN

from clip_lora_match_amd.tokenizer import ClipBPETokenizer, load_merges

TOK_DIR = os.path.join(GOLDEN, "clip_bpe")

CASES = [
    "a red backpack found near the library", "Dompet HITAM, ditemukan di kantin!!", "it's mine, don't lose it",
    "café  crème\t— naïve", "12:05 #42 ümlaut Straße", "日本語のテキスト 🎒🔑", "", "   ", "xyzzy qwerty zzz",
    "<|startoftext|>hello<|endoftext|>", "a " * 100, "RED\n\nbackpack", "students' card (KTP & SIM)",
    "I'LL be there, we'VE seen it", "3.14159 and 2,718", "tab\there", "ÅÉÎÕÜ ǅ ﬁ", "ño",
]


@pytest.fixture(scope="module")
def pair():
    transformers = pytest.importorskip("transformers")
    vocab = json.load(open(os.path.join(TOK_DIR, "vocab.json"), encoding="utf-8"))
    merges = load_merges(os.path.join(TOK_DIR, "merges.txt"))
    hf = transformers.CLIPTokenizer(vocab=vocab, merges=merges)
    return ClipBPETokenizer.from_dir(TOK_DIR), hf


@pytest.mark.parametrize("text", CASES)
def test_ids_equal_transformers(pair, text):
    ours, hf = pair
    for kw in ({}, {"truncation": True, "max_length": 77}, {"truncation": True, "max_length": 8}):
        assert ours(text, **kw)["input_ids"] == hf(text, **kw)["input_ids"], kw


def test_batch_padding_and_masks(pair):
    ours, hf = pair
    a = ours(CASES, padding=True, truncation=True, max_length=77)
    b = hf(CASES, padding=True, truncation=True, max_length=77)
    assert a["input_ids"] == b["input_ids"] and a["attention_mask"] == b["attention_mask"]
    a = ours(CASES[:3], padding="max_length", truncation=True, max_length=20)
    b = hf(CASES[:3], padding="max_length", truncation=True, max_length=20)
    assert a["input_ids"] == b["input_ids"]


def test_random_strings_equal_transformers(pair):
    from hypothesis import given, settings, strategies as st
    ours, hf = pair

    # assigned code points only (Python 3.10's Unicode 13 tables): an unassigned one, e.g.
    # U+323B0, is a letter to one Unicode database and not to another (the regex module vs the
    # tokenizers crate), which moves the pre-tokenizer split -- a version skew, not BPE
    @settings(max_examples=300, deadline=None, derandomize=True)
    @given(st.text(alphabet=st.characters(codec="utf-8", exclude_categories=("Cs", "Cn", "Co")), max_size=60))
    def check(t):
        assert ours(t, truncation=True, max_length=77)["input_ids"] == hf(t, truncation=True, max_length=77)["input_ids"]
    check()


def test_decode_roundtrip_and_specials(pair):
    ours, hf = pair
    t = "a red backpack found near the library"
    assert ours.decode(ours.encode(t)) == hf.decode(hf(t)["input_ids"], skip_special_tokens=True) == t
    assert ours.bos_token_id == 49406 and ours.eos_token_id == 49407


def test_processor_uses_it():
    import torch

    import clip_lora_match_amd as clm
    from clip_lora_match_amd.processor import ClipProcessor
    p = ClipProcessor(clm.get_preset("ViT-B/32"), tokenizer_dir=TOK_DIR)
    ids = p.token_ids(["red bag", "a much longer description of a lost item"])
    assert ids.dtype == torch.int32 and ids.shape[0] == 2
    assert int(ids[0, 0]) == 49406 and (ids[0] == 49407).any()
    enc = p(text="red bag")
    assert enc["input_ids"].dtype == torch.long and enc["attention_mask"].sum() == enc["input_ids"].shape[1]
