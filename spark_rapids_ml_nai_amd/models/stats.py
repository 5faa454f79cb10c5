"""Shared first pass over a row shard: column moments, scatter matrix, X^T y — optionally
consuming the shard chunk-by-chunk while its H2D is still in flight (``ops.ingest.StreamedRows``).

Numerics: the Gram is accumulated about a shift mu0 = mean of the first chunk (an estimate of
the column means, so the fp32 products see centred values, like the fused-centring SYRK of the
non-streaming path), then corrected exactly in fp64:

    C_r = sum (x - mu0)(x - mu0)^T - m_r d d^T,          d = mean_r - mu0   (local scatter)
    C   = sum_r [ C_r + m_r (mean_r - mu)(mean_r - mu)^T ]                 (global, one all-reduce)
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Optional

import torch

from .. import ops
from ..parallel.context import WorkerContext


@dataclass
class ScatterStats:
    m_total: int
    mean: torch.Tensor  # global column means (fp64)
    sumsq: Optional[torch.Tensor]  # global column sums of squares (fp64)
    scatter: torch.Tensor  # global centred scatter (n x n fp64)
    xty: Optional[torch.Tensor]  # global raw X^T y (fp64)
    y_sum: float = 0.0
    y_sumsq: float = 0.0


def scatter_stats(X: torch.Tensor, ctx: WorkerContext, m_total: int, stream: Any = None,
                  y: Optional[torch.Tensor] = None, need_sq: bool = True) -> ScatterStats:
    n = X.shape[1]
    dev = X.device
    chunks = stream.chunks() if stream is not None else [(0, X.shape[0], X)]
    s = ops.zeros(n, dtype=torch.float64, device=dev)
    q = ops.zeros(n, dtype=torch.float64, device=dev) if need_sq else None
    G = ops.zeros((n, n), dtype=torch.float64, device=dev)
    xty = ops.zeros((n, 1), dtype=torch.float64, device=dev) if y is not None else None
    mu0 = None
    m_r = 0
    for r0, r1, Xc in chunks:
        ops.col_moments(Xc, need_sq=need_sq, out=(s, q))  # accumulated in place: no per-chunk fill / add
        if mu0 is None:
            mu0 = s / max(r1 - r0, 1)  # the first chunk's means
            mu0f = mu0.float() if Xc.dtype == torch.float32 else mu0  # the Gram's shift, converted once
        ops.gram(Xc, mu0f, out=G, finalize=False)
        if y is not None:
            ops.xtv(Xc, y[r0:r1].view(-1, 1), out=xty)
        m_r += r1 - r0
    ops.gram_mirror(G)
    if mu0 is None:
        mu0 = ops.zeros(n, dtype=torch.float64, device=dev)
    mean_r = s / max(m_r, 1)
    d = mean_r - mu0
    G -= float(m_r) * torch.outer(d, d)  # local scatter about the local mean
    ys = ops.zeros(2, dtype=torch.float64, device=dev)
    if y is not None:
        yd = y.double()
        ys = torch.stack([yd.sum(), (yd * yd).sum()])
    small = torch.cat([s] + ([q] if need_sq else []) + [ys])
    ctx.comm.allreduce(small)
    s_g = small[:n]
    q_g = small[n: 2 * n] if need_sq else None
    ys = small[-2:]
    mean = s_g / float(m_total)
    e = mean_r - mean
    G += float(m_r) * torch.outer(e, e)
    big = torch.cat([G.view(-1)] + ([xty.view(-1)] if y is not None else []))
    ctx.comm.allreduce(big)
    scatter = big[: n * n].view(n, n)
    xty_g = big[n * n:] if y is not None else None
    ysh = ys.cpu().tolist()
    return ScatterStats(m_total, mean, q_g, scatter, xty_g, ysh[0], ysh[1])
