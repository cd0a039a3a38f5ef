"""Host->device copy rates on this box (the ceiling of bench.py's end_to_end leg): one 152 MB
buffer (the C2 batch's host columns) pinned and pageable, H2D, 10 repetitions each."""
import json
import time

import torch


def rate(src, dst, reps=10):
    for _ in range(2):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    return src.numel() * reps / (time.perf_counter() - t) / 1e9


n = 152_640_000
dev = torch.empty(n, dtype=torch.uint8, device="cuda:0")
pinned = torch.empty(n, dtype=torch.uint8).pin_memory()
pageable = torch.empty(n, dtype=torch.uint8)
pinned.fill_(1)
pageable.fill_(1)
out = {"bytes": n, "h2d_pinned_GBps": round(rate(pinned, dev), 2), "h2d_pageable_GBps": round(rate(pageable, dev), 2),
       "d2h_pinned_GBps": round(rate(dev, pinned), 2)}
print(json.dumps(out))
