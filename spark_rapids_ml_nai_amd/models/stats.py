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
    # the two all-reduce buffers are allocated whole and the accumulators are views of them: small =
    # [column sums | sums of squares | y sum, y sum of squares], big = [scatter | X^T y]
    ns = n + (n if need_sq else 0)
    small = ops.zeros(ns + 2, dtype=torch.float64, device=dev)
    big = ops.zeros(n * n + (n if y is not None else 0), dtype=torch.float64, device=dev)
    s = small[:n]
    q = small[n: 2 * n] if need_sq else None
    G = big[: n * n].view(n, n)
    xty = big[n * n:].view(n, 1) if y is not None else None
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
    mean_r = s / max(m_r, 1)  # (before the all-reduce sums s over the ranks)
    if y is not None:
        if dev.type == "cuda" and y.dtype in (torch.float32, torch.float64) and y.is_contiguous():
            ws = torch.empty(int(ops.native.lib().srml_sum_sq_ws()), dtype=torch.float64, device=dev)
            ops.native.call("srml_sum_sq", y.data_ptr(), int(y.dtype == torch.float64), y.shape[0], ws.data_ptr(),
                            small[ns:].data_ptr(), ops.native.stream(dev))
        else:
            yd = y.double()
            small[ns:] = torch.stack([yd.sum(), (yd * yd).sum()])
    ctx.comm.allreduce(small)
    s_g = small[:n]
    q_g = small[n: 2 * n] if need_sq else None
    mean = s_g / float(m_total)
    # local scatter about mu0 -> about the local mean -> about the global mean, in one pass
    if dev.type == "cuda":
        ops.native.call("srml_scatter_shift", G.data_ptr(), n, mean_r.data_ptr(), mu0.data_ptr(), mean.data_ptr(),
                        float(m_r), ops.native.stream(dev))
    else:
        d = mean_r - mu0
        e = mean_r - mean
        G += float(m_r) * (torch.outer(e, e) - torch.outer(d, d))
    ctx.comm.allreduce(big)
    scatter = G
    xty_g = xty.view(-1) if y is not None else None
    ysh = small[ns:].cpu().tolist()
    return ScatterStats(m_total, mean, q_g, scatter, xty_g, ysh[0], ysh[1])
