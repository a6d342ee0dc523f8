"""Run the configs[3] leg alone (ViT-L/14@336 + LoRA r=16, batch 128) for traces and PMC passes
of its kernels (attn_long_kernel, the L/14 GEMMs):  python tools/l14_run.py [steps] [dtype]
Prints bench.l14_leg's JSON sub-object."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    dtype = sys.argv[2] if len(sys.argv) > 2 else "mixed"
    print(json.dumps(bench.l14_leg(torch.device("cuda:0"), steps=steps, warmup=1, dtype=dtype)), flush=True)
