"""Distributed DBSCAN (reference: ``DBSCANModel._transform`` + cuML ``DBSCANMG.fit_predict``,
``clustering.py:940-1091``).

The reference collects the whole dataset on the driver and broadcasts it (C21). Here every rank
all-gathers the rows over RCCL (each MI355X holds the full matrix in its 288 GB), takes a
contiguous share of the lower-triangle 128x128 tile pairs and runs two fused MFMA sweeps:
  1. eps-degrees -> all-reduce SUM -> core flags (degree >= min_samples, self included);
  2. core-core edges -> per-rank union-find forest (+ nearest core neighbour of border points);
the forests are all-gathered and merged on device (every rank ends with identical roots = the
smallest core index of each component), border keys all-reduced with MIN. Labels are numbered
by ascending root, i.e. in order of each cluster's first core point (sklearn's numbering);
noise is -1.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext


def _share(total: int, rank: int, world: int) -> Tuple[int, int]:
    b = np.linspace(0, total, world + 1).astype(np.int64)
    return int(b[rank]), int(b[rank + 1])


def dbscan_fit_predict(X_local: torch.Tensor, ctx: WorkerContext, eps: float, min_samples: int,
                       metric: str = "euclidean") -> Tuple[np.ndarray, np.ndarray]:
    """(labels of this rank's rows, core-sample flags of this rank's rows)."""
    parts = ctx.comm.allgatherv(X_local.float().contiguous())
    sizes = [p.shape[0] for p in parts]
    start = sum(sizes[: ctx.rank])
    X = torch.cat([p.to(X_local.device) for p in parts], 0).contiguous()
    N = X.shape[0]
    if metric == "cosine":
        X = X / X.norm(dim=1, keepdim=True).clamp_min(1e-30)
        eps2 = 2.0 * float(eps)  # ||a - b||^2 = 2 (1 - cos) for unit rows
    elif metric in ("euclidean", "l2"):
        eps2 = float(eps) ** 2
    else:
        raise ValueError("Unsupported metric %r for DBSCAN" % metric)
    xn = ops.row_sqnorm(X)
    t0, t1 = _share(ops.dbscan_num_tiles(N), ctx.rank, ctx.world_size)
    counts = ops.dbscan_degree(X, xn, eps2, t0, t1)
    ctx.comm.allreduce(counts)
    core = (counts >= int(min_samples)).to(torch.uint8)
    parent = torch.arange(N, dtype=torch.int32, device=X.device)
    best = torch.full((N,), -1, dtype=torch.int64, device=X.device)
    ops.dbscan_link(X, xn, eps2, t0, t1, core, parent, best)
    if ctx.world_size > 1:
        ctx.comm.allreduce(best, op="min")
        forests = ctx.comm.allgather(parent.view(1, -1))
        for r in range(ctx.world_size):
            if r != ctx.rank:
                ops.uf_unite_pairs(parent, forests[r].to(X.device))
    ops.uf_compress(parent)
    # clusters numbered by ascending root (root-flag prefix scan on the device)
    labels = ops.dbscan_labels(parent, core, best)
    sl = slice(start, start + X_local.shape[0])
    return labels[sl].cpu().numpy(), core[sl].bool().cpu().numpy()
