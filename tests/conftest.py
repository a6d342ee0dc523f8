import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) HIP device")
    config.addinivalue_line("markers", "slow: long-running")


def pytest_runtest_setup(item):
    if "gpu" in item.keywords:
        import torch
        if not torch.cuda.is_available():
            pytest.fail("gpu test selected but no HIP device is visible (the product has no CPU fallback)")


_cache = {}


def synthetic(preset, lora_on=True):
    """(cfg, state_dict, lora) for a preset, cached per session."""
    key = (preset, lora_on)
    if key not in _cache:
        import clip_lora_match_amd as clm
        from clip_lora_match_amd import weights as W
        cfg = clm.get_preset(preset)
        if not lora_on:
            cfg = cfg.with_lora(0, 0.0, ())
        sd = W.synthetic_state_dict(cfg, 0)
        lora = W.synthetic_lora(cfg, 1) if lora_on else None
        _cache[key] = (cfg, sd, lora)
    return _cache[key]


def golden(name):
    return dict(np.load(os.path.join(GOLDEN, name), allow_pickle=False))


@pytest.fixture
def golden_loader():
    return golden
