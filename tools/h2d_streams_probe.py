"""PCIe H2D rate of one 12 GB pinned buffer: one copy on one stream vs the rows split over 2 / 4
streams (independent DMA queues), each measured twice with events."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

dev = torch.device("cuda", 0)
m, n = 1_000_000, 3000
h = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
h.fill_(1.0)
d = torch.empty((m, n), dtype=torch.float32, device=dev)
gb = m * n * 4 / 1e9
for ns in (1, 2, 4, 1):
    streams = [torch.cuda.Stream(dev, priority=-1) for _ in range(ns)]
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        step = (m + ns - 1) // ns
        for i, s in enumerate(streams):
            with torch.cuda.stream(s):
                d[i * step: (i + 1) * step].copy_(h[i * step: (i + 1) * step], non_blocking=True)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print("streams %d rep %d: %.4f s %.1f GB/s" % (ns, rep, dt, gb / dt), flush=True)
