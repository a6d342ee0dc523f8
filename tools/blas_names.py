"""hipBLASLt's kernel choice for the encoder shapes (run under rocprofv3 --kernel-trace --stats: the
kernel names carry the macro tile, MFMA shape and schedule)."""
import torch
dev = torch.device("cuda", 0)
for M, N, K in ((8192, 8192, 8192), (73856, 4096, 1024), (12800, 3072, 768), (12800, 768, 3072),
                (12800, 768, 768), (19712, 512, 2048), (19712, 512, 512), (19712, 2048, 512)):
    A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
    W = (torch.rand((N, K), device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(5):
        C = torch.mm(A, W.t())
    torch.cuda.synchronize()
    print(M, N, K, flush=True)
print("ok")
