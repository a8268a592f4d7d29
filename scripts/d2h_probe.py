"""Diagnostic: device-to-host copy rate into pinned memory by transfer size and streams."""
import time

import torch

dev = torch.device("cuda:0")
for mb in (8, 32, 128, 32):
    n = mb * (1 << 20) // 8
    src = [torch.randn(n, device=dev, dtype=torch.float64) for _ in range(4)]
    dst = [torch.empty(n, dtype=torch.float64, pin_memory=True) for _ in range(4)]
    for k in range(4):
        dst[k].copy_(src[k])                           # touch the pinned pages once
    for nstreams in (1, 2):
        streams = [torch.cuda.Stream() for _ in range(nstreams)]
        reps = 16
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for r in range(reps):
            with torch.cuda.stream(streams[r % nstreams]):
                dst[r % 4].copy_(src[r % 4], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(f"{mb} MB x {reps}, {nstreams} streams: {reps * mb / 1024 / dt:.1f} GB/s", flush=True)
