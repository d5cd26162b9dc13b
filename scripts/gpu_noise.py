import torch, time
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
x = torch.randn(256 * 1024 * 1024 // 4, device="cuda")
t0 = time.time()
while time.time() - t0 < 40:
    for _ in range(20):
        c = a @ b
        y = x * 1.0001 + 0.5
    torch.cuda.synchronize()
print("noise done")
