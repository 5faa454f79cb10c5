"""Distributed exact and IVF-Flat approximate k-nearest-neighbour search.

Reference: exact — cuML ``NearestNeighborsMG.kneighbors`` with UCX query fan-out and a partial
top-k merge (``knn.py:638-749``; every item row id additionally travelled through the Spark
driver); approximate — one cuML IVF-Flat index per item partition, queries broadcast, top-k
merged by a Spark SQL ``groupBy(query_id)`` (``knn.py:1154-1380``).

MI355X design (per rank = per item partition):
* queries are all-gathered over RCCL (device collective, no driver hop);
* exact: the fused MFMA distance + LDS top-k kernel (``srml_knn_f32``) over the local items;
* IVF-Flat: coarse quantiser trained with the device KMeans kernels, items bucketed into
  contiguous inverted lists (device sort), probes chosen with the same top-k kernel against the
  centroids, lists scanned by ``srml_ivf_search_f32``;
* partial (distance, global id) lists all-gathered and merged with one device top-k; each rank
  keeps the rows of its own queries.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext


def _gather_queries(Q: torch.Tensor, ctx: WorkerContext) -> Tuple[torch.Tensor, int, int]:
    parts = ctx.comm.allgatherv(Q.contiguous())
    sizes = [p.shape[0] for p in parts]
    start = sum(sizes[: ctx.rank])
    return torch.cat([p.to(Q.device) for p in parts], 0), start, Q.shape[0]


def _merge_partials(d: torch.Tensor, i: torch.Tensor, k: int, ctx: WorkerContext, start: int, nloc: int,
                    largest: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    if ctx.world_size > 1:
        dd = ctx.comm.allgather(d.contiguous().unsqueeze(0))  # (w, q, k)
        ii = ctx.comm.allgather(i.contiguous().unsqueeze(0))
        d = dd.permute(1, 0, 2).reshape(d.shape[0], -1)
        i = ii.permute(1, 0, 2).reshape(i.shape[0], -1)
        d = d[start: start + nloc]
        i = i[start: start + nloc]
        kk = min(k, d.shape[1])
        v, j = torch.topk(d, kk, dim=1, largest=largest)
        return v, i.gather(1, j)
    return d[start: start + nloc], i[start: start + nloc]


def _finish(d: torch.Tensor, metric: str) -> torch.Tensor:
    if metric in ("euclidean", "l2"):
        return torch.sqrt(d.clamp_min(0))
    if metric == "inner_product":
        return -0.5 * d
    return d


def _refine(Q: torch.Tensor, items: torch.Tensor, pos: torch.Tensor, metric: str) -> torch.Tensor:
    """Recompute the selected candidates' distances directly (q - i, not ||q||^2 + ||i||^2 - 2 q.i),
    so near-duplicates do not lose all their digits to fp32 cancellation. O(q k n), chunked."""
    nq, k = pos.shape
    n = Q.shape[1]
    out = torch.empty((nq, k), dtype=torch.float32, device=Q.device)
    step = max(1, (1 << 26) // max(1, k * n))
    valid = pos >= 0
    p = pos.clamp_min(0)
    for s in range(0, nq, step):
        rows = items.index_select(0, p[s: s + step].reshape(-1)).view(-1, k, n).float()
        q = Q[s: s + step].float().unsqueeze(1)
        if metric == "inner_product":
            out[s: s + step] = -2.0 * (rows * q).sum(-1)
        else:
            out[s: s + step] = ((rows - q) ** 2).sum(-1)
    return torch.where(valid, out, torch.full_like(out, float("inf")))


def _resort(d: torch.Tensor, i: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    v, j = torch.sort(d, dim=1)
    return v, i.gather(1, j)


def exact_knn(items: torch.Tensor, item_ids: torch.Tensor, queries: torch.Tensor, k: int, ctx: WorkerContext,
              metric: str = "euclidean") -> Tuple[np.ndarray, np.ndarray]:
    Qall, start, nloc = _gather_queries(queries, ctx)
    if items.shape[0] == 0:
        d = torch.full((Qall.shape[0], k), float("inf"), device=Qall.device)
        gi = torch.full((Qall.shape[0], k), -1, dtype=torch.int64, device=Qall.device)
    else:
        if metric == "inner_product":
            z_i = torch.zeros(items.shape[0], device=items.device)
            z_q = torch.zeros(Qall.shape[0], device=items.device)
            d, li = ops.knn(Qall, items, k, inorm=z_i, qnorm=z_q)  # d = -2 q.i
        else:
            d, li = ops.knn(Qall, items, k)
        d, li = _resort(_refine(Qall, items, li, metric), li)
        gi = torch.where(li >= 0, item_ids[li.clamp_min(0)], torch.full_like(li, -1))
        if d.shape[1] < k:  # fewer local items than k
            pad = k - d.shape[1]
            d = torch.cat([d, torch.full((d.shape[0], pad), float("inf"), device=d.device)], 1)
            gi = torch.cat([gi, torch.full((gi.shape[0], pad), -1, dtype=torch.int64, device=gi.device)], 1)
    d, gi = _merge_partials(d, gi, k, ctx, start, nloc)
    return _finish(d, metric).cpu().numpy(), gi.cpu().numpy()


@dataclass
class IVFIndex:
    centroids: torch.Tensor
    cnorm: torch.Tensor
    list_off: torch.Tensor
    items: torch.Tensor
    inorm: torch.Tensor
    ids: torch.Tensor


def build_ivf(X: torch.Tensor, ids: torch.Tensor, nlist: int, seed: int = 1, iters: int = 20,
              train_rows_per_list: int = 256) -> IVFIndex:
    """Coarse quantiser (Lloyd on a row subsample, as IVF trainers do) + contiguous inverted lists."""
    m = X.shape[0]
    nlist = max(1, min(int(nlist), m))
    gen = torch.Generator().manual_seed(int(seed))
    ntrain = min(m, max(nlist * train_rows_per_list, 4 * nlist))
    T = X if ntrain == m else X.index_select(0, torch.randperm(m, generator=gen)[:ntrain].to(X.device))
    C = T.index_select(0, torch.randperm(T.shape[0], generator=gen)[:nlist].to(X.device)).float().clone()
    tn = ops.row_sqnorm(T)
    for _ in range(max(1, iters)):
        lab, _d = ops.nearest_centroid(T, C, tn)
        sums, counts = ops.cluster_sums(T, lab, nlist)
        C = torch.where(counts.view(-1, 1) > 0, (sums / counts.clamp_min(1).double().view(-1, 1)).float(), C)
    lab, _ = ops.nearest_centroid(X, C)
    lab = lab.long()
    order = torch.argsort(lab, stable=True)
    counts = torch.bincount(lab, minlength=nlist)
    off = torch.zeros(nlist + 1, dtype=torch.int64, device=X.device)
    off[1:] = torch.cumsum(counts, 0)
    items = X.index_select(0, order).contiguous()
    return IVFIndex(C.contiguous(), ops.row_sqnorm(C), off, items, ops.row_sqnorm(items), ids.index_select(0, order))


def ivf_knn(index: Optional[IVFIndex], queries: torch.Tensor, k: int, nprobe: int, ctx: WorkerContext,
            metric: str = "euclidean") -> Tuple[np.ndarray, np.ndarray]:
    Qall, start, nloc = _gather_queries(queries, ctx)
    if index is None:
        d = torch.full((Qall.shape[0], k), float("inf"), device=Qall.device)
        gi = torch.full((Qall.shape[0], k), -1, dtype=torch.int64, device=Qall.device)
    else:
        nprobe = max(1, min(int(nprobe), index.centroids.shape[0], ops.KNN_KMAX))
        qn = ops.row_sqnorm(Qall)
        _, probes = ops.knn(Qall, index.centroids, nprobe, inorm=index.cnorm, qnorm=qn)
        pos_ids = torch.arange(index.items.shape[0], dtype=torch.int64, device=Qall.device)
        if metric == "inner_product":
            z = torch.zeros_like(index.inorm)
            d, pos = ops.ivf_search(Qall, probes.int(), index.list_off, index.items, z, pos_ids, k,
                                    qnorm=torch.zeros_like(qn))
        else:
            d, pos = ops.ivf_search(Qall, probes.int(), index.list_off, index.items, index.inorm, pos_ids, k, qnorm=qn)
        d, pos = _resort(_refine(Qall, index.items, pos, metric), pos)
        gi = torch.where(pos >= 0, index.ids[pos.clamp_min(0)], torch.full_like(pos, -1))
    d, gi = _merge_partials(d, gi, k, ctx, start, nloc)
    return _finish(d, metric).cpu().numpy(), gi.cpu().numpy()
