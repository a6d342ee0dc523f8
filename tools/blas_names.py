import torch
dev = torch.device("cuda", 0)
for M, N, K in ((8192, 8192, 8192), (73856, 4096, 1024), (12800, 3072, 768)):
    A = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
    W = (torch.rand((N, K), device=dev) * 2 - 1).to(torch.bfloat16)
    for _ in range(5):
        C = torch.mm(A, W.t())
    torch.cuda.synchronize()
print("ok")
