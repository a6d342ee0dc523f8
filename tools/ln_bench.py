"""Time the encoder LayerNorm kernel (clm_layernorm) at the B/32 batch-256 shapes and the
L/14 shape; HIP events on the launch stream; algorithmic bytes = 4 d (fp32 row in) + 2 d
(16-bit row out) per row. Beside it: torch's fp32 -> 16-bit conversion copy, the same bytes
(the practical ceiling of a pass that reads and writes them). JSON lines.
(profiles/r03_v10_ln_persist_probe.jsonl was taken with a persistent-walk variant of the kernel,
selected by CLM_LN_PERSIST in that build; it was not kept.)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

SHAPES = {"vision_b32": (256 * 50, 768), "text_b32": (256 * 77, 512), "vision_l14": (128 * 577, 1024),
          "odd_rows": (12799, 768)}


def timed(fn, st):
    fn()
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            fn()
        e1.record(st)
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) / 20 * 1e3)
    return sorted(ts)[2]


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream()
    for name, (M, d) in SHAPES.items():
        x = torch.randn((M, d), device=dev)
        g, b = torch.randn(d, device=dev), torch.randn(d, device=dev)
        y = torch.empty((M, d), dtype=torch.bfloat16, device=dev)

        def run():
            C.check(C.lib().clm_layernorm(0, C.CLM_BF16, C.ptr(x), d, M, d, C.ptr(g), C.ptr(b), 1e-5, C.ptr(y), d,
                                          C.stream_of(dev)), "clm_layernorm")
        cu = timed(lambda: y.copy_(x), st)
        us = timed(run, st)
        print(json.dumps({"shape": name, "M": M, "d": d, "us": round(us, 2),
                          "GBps": round(M * d * 6 / (us * 1e-6) / 1e9, 1), "convert_copy_us": round(cu, 2)}),
              flush=True)

if __name__ == "__main__":
    main()
