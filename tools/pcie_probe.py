#!/usr/bin/env python3
"""H2D / D2H bandwidth from pinned host memory on the current GPU, one
direction and both at once (two streams), with torch: the ceiling of the
host-fed runner's figure 2."""
import time

import torch


def bw(n_mb=512, reps=5):
    n = n_mb << 20
    h1 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    h2 = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    d1 = torch.empty(n, dtype=torch.uint8, device="cuda")
    d2 = torch.empty(n, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}
    for name, fn in (("h2d", lambda: d1.copy_(h1, non_blocking=True)),
                     ("d2h", lambda: h2.copy_(d2, non_blocking=True))):
        fn(); torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        out[name] = reps * n / (time.perf_counter() - t) / 1e9
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        with torch.cuda.stream(s1):
            d1.copy_(h1, non_blocking=True)
        with torch.cuda.stream(s2):
            h2.copy_(d2, non_blocking=True)
    torch.cuda.synchronize()
    out["both"] = 2 * reps * n / (time.perf_counter() - t) / 1e9
    return out


if __name__ == "__main__":
    print({k: round(v, 1) for k, v in bw().items()}, "GB/s")
