"""Distributed exact and IVF-Flat approximate k-nearest-neighbour search.

Reference: exact — cuML ``NearestNeighborsMG.kneighbors`` with UCX query fan-out and a partial
top-k merge (``knn.py:638-749``; every item row id additionally travelled through the Spark
driver); approximate — one cuML IVF-Flat index per item partition, queries broadcast, top-k
merged by a Spark SQL ``groupBy(query_id)`` (``knn.py:1154-1380``).

MI355X design (per rank = per item partition):
* query fan-out is a point-to-point RING (the role of the reference's UCX send/recv): every
  rank's query block travels once around the ranks together with its running top-k; at each hop
  the holder scores it against its local items and merges (device radix-select top-k with ids),
  and the NEXT block's transfer (isend/irecv over RCCL/xGMI) overlaps that compute. After W hops
  the finished block is back at its owner. Per-rank memory is two query blocks + their top-k
  lists, instead of every rank's queries (the all-gather's O(Q·n) per rank);
* exact: the fused MFMA distance + LDS top-k kernel (``srml_knn_f32``, k <= 64) or the distance
  chunk + radix-select path (k <= 1024) over the local items, candidates refined exactly;
* IVF-Flat: coarse quantiser trained with the device KMeans kernels, items bucketed into
  contiguous inverted lists (device sort), probes chosen with the same top-k kernel against the
  centroids, lists scanned by ``srml_ivf_search_f32``; queries ride the same ring.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext


def _merge_lists(d1: torch.Tensor, i1: torch.Tensor, d2: torch.Tensor, i2: torch.Tensor, k: int
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """k smallest of two (distance, id) lists per row (ties keep the earlier list)."""
    D = torch.cat([d1, d2], 1)
    I = torch.cat([i1, i2], 1)
    return ops.topk_rows(D, k, ids=I)  # radix select on the device (k <= ops.TOPK_KMAX)


def _ring_search(queries: torch.Tensor, k: int, ctx: WorkerContext, local: Callable[[torch.Tensor], Tuple[
        torch.Tensor, torch.Tensor]]) -> Tuple[torch.Tensor, torch.Tensor]:
    """Run ``local(Q) -> (d [q, k], global ids [q, k])`` for every rank's query block on every
    rank's items by passing (block, running top-k) around the ring; returns this rank's merged
    lists.

    Per hop: the NEXT query block's isend/irecv starts first and the held block is scored while it
    travels; the held block's running lists (sent by the previous rank after ITS merge) are only
    waited for after that scoring, merged, and forwarded at once — so each list exchange overlaps
    the next hop's scoring instead of sitting between hops on the critical path."""
    W, r = ctx.world_size, ctx.rank
    dev = queries.device
    nq = queries.shape[0]
    if W == 1:
        return local(queries)
    sizes = [int(v) for v in ctx.comm.allgather(torch.tensor([nq], dtype=torch.int64, device=ctx.device)).tolist()]
    n = queries.shape[1]
    nxt, prv = (r + 1) % W, (r - 1) % W
    Qc = queries.contiguous()
    dc = torch.full((nq, k), float("inf"), dtype=torch.float32, device=dev)
    ic = torch.full((nq, k), -1, dtype=torch.int64, device=dev)
    h_lists = None  # in-flight exchange of the running lists of the block held at this hop
    for s in range(W):
        h_q = None
        if s < W - 1:  # the next block is already on its way while this one is scored
            rows = sizes[(r - s - 1) % W]
            Qn = torch.empty((rows, n), dtype=Qc.dtype, device=dev)
            h_q = ctx.comm.isendrecv(Qc, nxt, Qn, prv)
        ld = li = None
        if Qc.shape[0]:
            ld, li = local(Qc)
        if h_lists is not None:  # this block's lists, merged by the previous rank at the last hop
            for h in h_lists:
                ctx.comm.wait_sendrecv(h)
            h_lists = None
        if ld is not None:
            dc, ic = _merge_lists(dc, ic, ld.float(), li, k)
        if s < W - 1:
            ctx.comm.wait_sendrecv(h_q)
            dn = torch.empty((rows, k), dtype=torch.float32, device=dev)
            inn = torch.empty((rows, k), dtype=torch.int64, device=dev)
            # forward the merged lists with the block they belong to (already sent); overlaps the
            # next hop's scoring
            h_lists = (ctx.comm.isendrecv(dc.contiguous(), nxt, dn, prv),
                       ctx.comm.isendrecv(ic.contiguous(), nxt, inn, prv))
            Qc, dc, ic = Qn, dn, inn
    # the block now held belongs to the next rank: hand it home, receive ours
    d_own = torch.empty((nq, k), dtype=torch.float32, device=dev)
    i_own = torch.empty((nq, k), dtype=torch.int64, device=dev)
    h1 = ctx.comm.isendrecv(dc.contiguous(), nxt, d_own, prv)
    h2 = ctx.comm.isendrecv(ic.contiguous(), nxt, i_own, prv)
    ctx.comm.wait_sendrecv(h1)
    ctx.comm.wait_sendrecv(h2)
    return d_own, i_own


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


def _refine_sorted(Q: torch.Tensor, items: torch.Tensor, pos: torch.Tensor, metric: str
                   ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact re-scored candidates sorted per query: the fused device kernel
    (``ops.knn_refine_sort``) when it applies, else the chunked torch re-score + sort."""
    r = ops.knn_refine_sort(Q, items, pos, inner_product=metric == "inner_product")
    if r is not None:
        return r
    return _resort(_refine(Q, items, pos, metric), pos)


def _pad_k(d: torch.Tensor, gi: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    if d.shape[1] < k:  # fewer local items than k
        pad = k - d.shape[1]
        d = torch.cat([d, torch.full((d.shape[0], pad), float("inf"), device=d.device)], 1)
        gi = torch.cat([gi, torch.full((gi.shape[0], pad), -1, dtype=torch.int64, device=gi.device)], 1)
    return d, gi


def exact_knn(items: torch.Tensor, item_ids: torch.Tensor, queries: torch.Tensor, k: int, ctx: WorkerContext,
              metric: str = "euclidean") -> Tuple[np.ndarray, np.ndarray]:
    def local(Q: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        if items.shape[0] == 0:
            return (torch.full((Q.shape[0], k), float("inf"), device=Q.device),
                    torch.full((Q.shape[0], k), -1, dtype=torch.int64, device=Q.device))
        if metric == "inner_product":
            z_i = ops.zeros(items.shape[0], device=items.device)
            z_q = ops.zeros(Q.shape[0], device=items.device)
            d, li = ops.knn(Q, items, k, inorm=z_i, qnorm=z_q)  # d = -2 q.i
        else:
            d, li = ops.knn(Q, items, k)
        d, li = _refine_sorted(Q, items, li, metric)
        gi = torch.where(li >= 0, item_ids[li.clamp_min(0)], torch.full_like(li, -1))
        return _pad_k(d, gi, k)

    d, gi = _ring_search(queries, k, ctx, local)
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
    FT = ops.quantizer_planes(T) if nlist > 256 else None  # bucketing only: the fp16 filter's arg-min
    tn = ops.row_sqnorm(T) if FT is None else None
    for _ in range(max(1, iters)):
        lab = ops.nearest_list(T, C, FT, tn)
        sums, counts = ops.cluster_sums(T, lab, nlist)
        C = torch.where(counts.view(-1, 1) > 0, (sums / counts.clamp_min(1).double().view(-1, 1)).float(), C)
    lab = ops.nearest_list(X, C, ops.quantizer_planes(X) if nlist > 256 else None)
    order, off, _ = ops.label_sort(lab, nlist)  # stable: rows keep their order inside a list
    order = order.long()
    items = X.index_select(0, order).contiguous()
    return IVFIndex(C.contiguous(), ops.row_sqnorm(C), off, items, ops.row_sqnorm(items), ids.index_select(0, order))


def ivf_knn(index: Optional[IVFIndex], queries: torch.Tensor, k: int, nprobe: int, ctx: WorkerContext,
            metric: str = "euclidean") -> Tuple[np.ndarray, np.ndarray]:
    def local(Q: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        if index is None:
            return (torch.full((Q.shape[0], k), float("inf"), device=Q.device),
                    torch.full((Q.shape[0], k), -1, dtype=torch.int64, device=Q.device))
        npb = max(1, min(int(nprobe), index.centroids.shape[0], ops.KNN_KMAX))
        qn = ops.row_sqnorm(Q)
        _, probes = ops.knn(Q, index.centroids, npb, inorm=index.cnorm, qnorm=qn)
        pos_ids = torch.arange(index.items.shape[0], dtype=torch.int64, device=Q.device)
        if metric == "inner_product":
            z = torch.zeros_like(index.inorm)
            d, pos = ops.ivf_search(Q, probes.int(), index.list_off, index.items, z, pos_ids, k,
                                    qnorm=torch.zeros_like(qn))
        else:
            d, pos = ops.ivf_search(Q, probes.int(), index.list_off, index.items, index.inorm, pos_ids, k, qnorm=qn)
        d, pos = _refine_sorted(Q, index.items, pos, metric)
        gi = torch.where(pos >= 0, index.ids[pos.clamp_min(0)], torch.full_like(pos, -1))
        return _pad_k(d, gi, k)

    d, gi = _ring_search(queries, k, ctx, local)
    return _finish(d, metric).cpu().numpy(), gi.cpu().numpy()
