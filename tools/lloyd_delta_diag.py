"""Per-iteration view of the small-k Lloyd loop's label book on uniform rows: the step kernel's
time and the moved rows of every iteration (delta steps forced after the first when --force, full
steps only with --full, no book with --nobook, else the loop's own 1/4 rule)."""
import argparse
import json
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from spark_rapids_ml_nai_amd import ops  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--cols", type=int, default=64)
ap.add_argument("--k", type=int, default=20)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--force", action="store_true")
ap.add_argument("--full", action="store_true", help="every step a full step (mode 0)")
ap.add_argument("--nobook", action="store_true", help="no label book (the loop's step before delta steps)")
a = ap.parse_args()
dev = torch.device("cuda:0")
g = torch.Generator(device=dev).manual_seed(0)
X = torch.rand(a.rows, a.cols, device=dev, generator=g)
m, n, k = a.rows, a.cols, a.k
kn = k * n
C64 = X[torch.randint(0, m, (k,), device=dev, generator=g)].double()
mu = C64.mean(0)
C64 = (C64 - mu).contiguous()
C32 = C64.float().contiguous()
cn = (C32 * C32).sum(1).contiguous()
mu32 = mu.float().contiguous()
flags = torch.zeros(3, dtype=torch.int32, device=dev)
book = (torch.empty(m, dtype=torch.int32, device=dev), flags[2:3])
G = torch.empty(kn + k, dtype=torch.float64, device=dev)
buf = torch.zeros(kn + k + 2, dtype=torch.float64, device=dev)
stat = torch.zeros(2, dtype=torch.float64, device=dev)
ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
for it in range(a.iters):
    mode = int(flags[2].item())
    buf.zero_()
    ev[0].record()
    bk = None if a.nobook else book
    ops.kmeans_lloyd_small(X, C32, cn, out=buf, done=flags, rows_out=False, mu=mu32, book=bk)
    ev[1].record()
    ev[2].record()
    ops.kmeans_small_update(buf, k, n, C64, C32, cn, 0.0, flags, stat, G=None if bk is None else G)
    ev[3].record()
    torch.cuda.synchronize()
    rec = dict(it=it, mode=mode, moved=int(buf[kn + k + 1].item()), step_ms=round(ev[0].elapsed_time(ev[1]), 3),
               sums_ms=round(ev[1].elapsed_time(ev[2]), 3), update_ms=round(ev[2].elapsed_time(ev[3]), 3))
    print(json.dumps(rec), flush=True)
    if a.force:
        flags[2] = 1
    if a.full:
        flags[2] = 0
