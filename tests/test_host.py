"""Host-side logic that needs no GPU: configs, weight generator, PEFT adapter
format, processor tokens, reference-format YAML handling, C-ABI exports."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import REPO

import clip_lora_match_amd as clm
from clip_lora_match_amd import synthetic as syn
from clip_lora_match_amd import weights as W


def test_preset_shapes_and_param_counts():
    cfg = clm.get_preset("openai/clip-vit-base-patch32")
    shapes = W.state_dict_shapes(cfg)
    assert sum(int(np.prod(s)) for s in shapes.values()) == 151_277_312   # CLIPModel minus logit_scale
    assert W.lora_param_count(cfg) == 983_040                               # 96 Linears
    assert len(W.lora_shapes(cfg)) == 2 * 96
    assert cfg.lora_scaling == 2.0 and cfg.vision_seq == 50
    l14 = clm.get_preset("ViT-L/14@336")
    assert l14.vision_seq == 577 and l14.lora_r == 16 and "fc2" in l14.lora_targets
    with pytest.raises(ValueError):
        clm.get_preset("no-such-model")


def test_synthetic_weights_deterministic_and_distinct():
    cfg = clm.get_preset("tiny")
    a, b = W.synthetic_state_dict(cfg, 0), W.synthetic_state_dict(cfg, 0)
    assert all(np.array_equal(a[k], b[k]) for k in a)
    c = W.synthetic_state_dict(cfg, 1)
    assert not np.array_equal(a["visual_projection.weight"], c["visual_projection.weight"])
    la = W.synthetic_lora(cfg, 1)
    assert all(np.abs(v).max() > 0 for k, v in la.items() if ".lora_B." in k)   # non-zero B


def test_peft_adapter_roundtrip(tmp_path):
    cfg = clm.get_preset("tiny")
    lora = W.synthetic_lora(cfg, 1)
    W.save_peft_adapter(tmp_path / "ad", lora, cfg.lora_r, cfg.lora_alpha, cfg.lora_targets)
    back, acfg = W.load_peft_adapter(tmp_path / "ad")
    assert acfg["r"] == cfg.lora_r and acfg["lora_alpha"] == cfg.lora_alpha
    assert set(back) == set(lora) and all(np.array_equal(back[k], lora[k]) for k in lora)
    with pytest.raises(FileNotFoundError):
        W.load_peft_adapter(tmp_path / "nope")


def test_peft_default_adapter_key_names(tmp_path):
    """PEFT writes '...lora_A.weight' (adapter name stripped); older dumps may keep
    '.default' -- both load."""
    from safetensors.numpy import save_file
    cfg = clm.get_preset("tiny")
    lora = W.synthetic_lora(cfg, 1)
    d = tmp_path / "ad2"
    d.mkdir()
    save_file({k.replace("base_model.model.", "").replace(".lora_A.weight", ".lora_A.default.weight")
               .replace(".lora_B.weight", ".lora_B.default.weight"): v for k, v in lora.items()},
              str(d / "adapter_model.safetensors"))
    (d / "adapter_config.json").write_text('{"r": 8, "lora_alpha": 16, "target_modules": ["q_proj"]}')
    back, _ = W.load_peft_adapter(d)
    assert set(back) == set(lora)


def test_synthetic_captions_structure():
    ids = syn.captions(50, 77, 49406, 49407, 3)
    assert ids.shape == (50, 77) and (ids[:, 0] == 49406).all()
    first_eos = (ids == 49407).argmax(1)
    assert (first_eos >= 7).all()
    for r, e in zip(ids, first_eos):
        assert (r[e:] == 49407).all() and (r[1:e] < 49406).all()


def test_processor_token_ids_padding():
    from clip_lora_match_amd.processor import ClipProcessor, TokenizerUnavailable
    cfg = clm.get_preset("ViT-B/32")
    p = ClipProcessor(cfg)
    t = p.token_ids([[49406, 5, 6, 49407], [49406, 7, 49407]])
    assert t.tolist() == [[49406, 5, 6, 49407], [49406, 7, 49407, 49407]]
    long = [49406] + [3] * 100 + [49407]
    assert p.token_ids(long).shape == (1, 77) and int(p.token_ids(long)[0, -1]) == 49407
    if p.tokenizer is None:
        with pytest.raises(TokenizerUnavailable):
            p.token_ids("a photo of a cat")


def test_reference_format_yaml(tmp_path):
    from clip_lora_match_amd.clip_model import _load_clip_config
    from clip_lora_match_amd.lora_adapter import create_lora_config
    y = tmp_path / "lora_config.yaml"
    y.write_text("model:\n  target_modules: [q_proj, k_proj, v_proj, out_proj]\nlora:\n  r: 8\n  alpha: 16\n"
                 "  dropout: 0.1\n  bias: none\n  task_type: FEATURE_EXTRACTION\n")
    c = create_lora_config(y)
    assert c.r == 8 and c.lora_alpha == 16 and c.target_modules == ["q_proj", "k_proj", "v_proj", "out_proj"]
    y2 = tmp_path / "l2.yaml"
    y2.write_text("lora: {r: 4}\n")
    assert create_lora_config(y2).target_modules == ["q_proj", "v_proj"]   # lora_adapter.py:33 default
    with pytest.raises(FileNotFoundError):
        create_lora_config(tmp_path / "none.yaml")
    with pytest.raises(FileNotFoundError):
        _load_clip_config(tmp_path / "none.yaml")


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "clm.h")).read()
    return sorted(set(re.findall(r"\b(clm_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    from clip_lora_match_amd import _capi
    lib = _capi.lib()
    syms = _header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(lib, s), s
    assert set(syms) == set(_capi.EXPORTED)
    assert lib.clm_model_desc_size() == ctypes.sizeof(_capi.ModelDesc)
    assert lib.clm_version().startswith(b"clm")


def test_library_has_gfx950_code_object():
    so = os.path.join(REPO, "clip-lora-match_amd", "libclm.so")
    assert b"amdgcn-amd-amdhsa--gfx950" in open(so, "rb").read()


def test_no_device_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is visible")
    from clip_lora_match_amd.engine import ClipLoraModel
    with pytest.raises(RuntimeError):
        ClipLoraModel(clm.get_preset("tiny"))


def _host_check():
    """(re)build the host-sanitizer harness (csrc/Makefile `sanitize`: ASan + UBSan on the host
    half of the C-ABI) and return its path"""
    import subprocess
    subprocess.run(["make", "-C", os.path.join(REPO, "clip-lora-match_amd", "csrc"), "sanitize"], check=True,
                   capture_output=True, timeout=1200)
    return os.path.join(REPO, "clip-lora-match_amd", "host_check")


def test_c_abi_under_host_sanitizers():
    """Every entry point's argument validation runs clean under ASan / UBSan (no device here: the
    device half of the harness runs in tests/test_gpu_kernels.py)."""
    import subprocess
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is visible: the GPU test runs the full harness")
    p = subprocess.run([_host_check()], capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "argument checks (no HIP device), 0 failure(s)" in p.stdout


def test_gemm_config_table_matches_the_test_matrix():
    """every tile config is reachable by the picker (k_gemm.hip pick_config); the GPU test matrix
    (test_gpu_kernels.py) covers exactly these ids"""
    from clip_lora_match_amd import _capi as C
    assert C.lib().clm_gemm_num_configs() == 15


def _f16_down(v):
    """numpy restatement of clm_common.hpp f16_down: the largest fp16 value <= v"""
    import numpy as np
    h = v.astype(np.float16)
    b = h.view(np.uint16).astype(np.int32)
    up = h.astype(np.float32) > v
    b = np.where(up & (b == 0), 0x8001, np.where(up & (b >= 0x8000), b + 1, np.where(up, b - 1, b)))
    return b.astype(np.uint16).view(np.float16)


def test_sampled_threshold_stays_a_lower_bound():
    """The bounded search's sampled θ (capi.cpp search_bounded) is the k-th largest of the stored
    sample scores minus the margin; round 5 stores them as fp16 rounded toward -inf and as maxima
    of groups of 4 sample rows. Both only lower the k-th largest: f16_down(v) <= v for every v
    (ties, subnormals, signs, infinities), and the k-th largest of group maxima (a subset of the
    values) is <= the k-th largest of all values -- so θ never rises above the fp32 one."""
    import numpy as np
    g = np.random.default_rng(5)
    v = np.concatenate([g.normal(0, 0.05, 200000), g.uniform(-1, 1, 20000),
                        np.float32(2.0) ** g.integers(-30, 5, 2000) * g.choice([-1, 1], 2000),
                        [0.0, -0.0, 1.0, -1.0, 65504.0, 1e6, -1e6, np.inf, -np.inf, 6e-8, -6e-8]]).astype(np.float32)
    with np.errstate(over="ignore"):
        h = _f16_down(v)
        rne = v.astype(np.float16)
    assert (h.astype(np.float32) <= v).all()
    fin = np.abs(v) <= 65504   # in range: RNE or the fp16 value one step below it
    down_one = h.astype(np.float32) == np.nextafter(rne, np.float16(-np.inf)).astype(np.float32)
    assert ((h == rne) | down_one)[fin].all()
    for k in (1, 5, 8):
        for _ in range(5):
            s = g.normal(0.0, 0.044, 195328).astype(np.float32)     # one query's sample scores
            kth32 = np.sort(s)[-k]
            grp = _f16_down(s.reshape(-1, 4).max(1)).astype(np.float32)
            kth_grp = np.sort(grp)[-k]
            assert kth_grp <= kth32
            assert kth32 - kth_grp < 0.05   # and it stays close (more candidates, not a collapse)
