"""Known-byte calibration for FETCH_SIZE / WRITE_SIZE: a 512 MiB fp32 device copy (reads and writes
exactly 512 MiB each, larger than the 256 MiB Infinity Cache)."""
import torch

n = 128 * 1024 * 1024
a = torch.ones(n, device="cuda:0")
b = torch.empty_like(a)
for _ in range(3):
    b.copy_(a)
torch.cuda.synchronize()
print("bytes per copy", 4 * n)
