"""HBM ceilings on this box for the bandwidth discussion: write-only (fill), copy, read-only (sum)."""
import torch
n = 1 << 29   # 512M floats = 2 GiB
x = torch.empty(n, device="cuda:0")
y = torch.empty(n, device="cuda:0")
def t(fn, reps=10):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / reps / 1e3
b = n * 4
w = t(lambda: x.fill_(1.0)); print(f"write-only fill: {b / w / 1e9:7.0f} GB/s", flush=True)
c = t(lambda: y.copy_(x)); print(f"copy (read+write): {2 * b / c / 1e9:7.0f} GB/s", flush=True)
r = t(lambda: x.sum()); print(f"read-only sum: {b / r / 1e9:7.0f} GB/s", flush=True)
