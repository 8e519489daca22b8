"""Does HBM read bandwidth of a freshly allocated large buffer depend on the
allocation history of the process?  Reads 8 x 1.92 GB buffers (the config
D-total pool) with torch.sum (an HBM-bound read) before and after the
config-C-like churn (100 x 160 MB allocated, used, freed, empty_cache)."""
import sys
import time

import torch


def bw(bufs, reps=20):
    torch.cuda.synchronize()
    for b in bufs:
        b.sum()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for i in range(reps):
        bufs[i % len(bufs)].sum()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    return bufs[0].numel() * 8 / ms / 1e6


def pool(n, nbytes):
    return [torch.rand(nbytes // 8, dtype=torch.float64, device="cuda") for _ in range(n)]


mode = sys.argv[1] if len(sys.argv) > 1 else "fresh"
if mode == "churn":
    c = pool(100, 160_000_000)
    for b in c:
        b.sum()
    del c
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
d = pool(8, 1_920_000_000)
print(mode, "GB/s", round(bw(d), 1), flush=True)
del d
torch.cuda.empty_cache()
d = pool(8, 1_920_000_000)
print(mode, "again GB/s", round(bw(d), 1), flush=True)
