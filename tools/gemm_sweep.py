"""Time every GEMM tile config on the encoder's GEMM shapes (B/32, batch 256), HIP-event
timed on the launch stream, interleaved rounds in one process. Prints JSON lines."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from clip_lora_match_amd import _capi as C  # noqa: E402

B = int(os.environ.get("SWEEP_B", "256"))
SHAPES = {  # name: (M, N, K, epi)
    "v_qkv": (B * 50, 2304, 768, C.CLM_EPI_STORE), "v_out": (B * 50, 768, 768, C.CLM_EPI_RESID),
    "v_fc1": (B * 50, 3072, 768, C.CLM_EPI_GELU), "v_fc2": (B * 50, 768, 3072, C.CLM_EPI_RESID),
    "t_qkv": (B * 77, 1536, 512, C.CLM_EPI_STORE), "t_out": (B * 77, 512, 512, C.CLM_EPI_RESID),
    "t_fc1": (B * 77, 2048, 512, C.CLM_EPI_GELU), "t_fc2": (B * 77, 512, 2048, C.CLM_EPI_RESID),
    "patch": (B * 49, 768, 3072, C.CLM_EPI_RESID), "sq4096": (4096, 4096, 4096, C.CLM_EPI_STORE),
}


def main():
    dev = torch.device("cuda", 0)
    L = C.lib()
    ncfg = L.clm_gemm_num_configs()
    st = torch.cuda.current_stream()
    res = {}
    bufs = {}
    for name, (M, N, K, epi) in SHAPES.items():
        A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
        W = ((torch.rand((N, K), device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        out = torch.zeros((M, N), device=dev, dtype=torch.float32 if epi == C.CLM_EPI_RESID else torch.bfloat16)
        bias = torch.zeros(N, device=dev)
        bufs[name] = (A, W, out, bias)
    only = os.environ.get("SWEEP_CFGS")
    cfgs = ([int(c) if c.lstrip("-").isdigit() else c for c in only.split(",")] if only
            else list(range(ncfg)) + [-1, "hipblaslt"])   # hipblaslt: torch.matmul, bf16 out, no epilogue
    obf = {n: torch.empty((b[0].shape[0], b[1].shape[0]), device=dev, dtype=torch.bfloat16) for n, b in bufs.items()}
    for rnd in range(3):
        for name, (M, N, K, epi) in SHAPES.items():
            A, W, out, bias = bufs[name]
            for cfg in cfgs:
                def run():
                    if cfg == "hipblaslt":
                        torch.matmul(A, W.t(), out=obf[name])
                        return
                    C.check(L.clm_gemm(0, C.CLM_BF16, epi, cfg, C.ptr(A), K, C.ptr(W), K, M, N, K, C.ptr(out),
                                       N, C.ptr(bias), None, None, C.stream_of(dev)))
                run()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                reps = 20
                e0.record(st)
                for _ in range(reps):
                    run()
                e1.record(st)
                e1.synchronize()
                us = e0.elapsed_time(e1) / reps * 1e3
                tf = 2.0 * M * N * K / (us * 1e-6) / 1e12
                res.setdefault((name, cfg), []).append((us, tf))
    for (name, cfg), v in sorted(res.items(), key=lambda kv: (kv[0][0], str(kv[0][1]))):
        best = min(v)
        print(json.dumps({"shape": name, "cfg": cfg, "us": round(best[0], 2), "tflops": round(best[1], 1)}))


if __name__ == "__main__":
    main()
