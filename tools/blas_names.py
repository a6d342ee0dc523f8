"""Run torch.mm (hipBLASLt) once per encoder GEMM shape, for rocprofv3 kernel names."""
import torch
B = 256
dev = torch.device("cuda", 0)
for M, N, K in [(B * 50, 2304, 768), (B * 50, 768, 768), (B * 50, 3072, 768), (B * 50, 768, 3072), (4096, 4096, 4096),
                (B * 77, 1536, 512), (B * 77, 2048, 512)]:
    A = torch.randn((M, K), device=dev).to(torch.bfloat16)
    W = torch.randn((N, K), device=dev).to(torch.bfloat16)
    for _ in range(3):
        torch.mm(A, W.t())
torch.cuda.synchronize()
print("ok")
