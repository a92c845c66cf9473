import torch
torch.cuda.set_device(0)
for M, N, K in ((4096, 4096, 4096), (12800, 768, 3072), (12800, 3072, 768), (1600, 768, 3072), (1600, 768, 768), (1600, 2304, 768)):
    A = torch.rand(M, K, device="cuda"); W = torch.rand(N, K, device="cuda")
    for _ in range(3):
        y = A @ W.t()
    torch.cuda.synchronize()
