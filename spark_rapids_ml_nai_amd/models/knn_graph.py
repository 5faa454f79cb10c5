"""All-points kNN graphs for UMAP (single device or distributed over RCCL).

* ``knn_graph_brute`` — exact: fused MFMA distance + LDS top-k (``ops.knn``); distributed, each
  rank queries its row block against the replicated X and the blocks are all-gathered.
* ``knn_graph_ivf`` — approximate (the north-star 20M x 128 graph, BASELINE.json config 5):
  k-means lists, every 128-row query tile of a list matched against the ``nprobe`` lists
  nearest to its list's centroid by the MFMA tile kernel ``ops.knn_lists``, candidates
  re-scored exactly. Distributed, every phase shards: the quantiser's Lloyd iterations run on
  1/W of the training sample per rank (cluster sums all-reduced), each rank buckets its 1/W of
  the rows (labels all-gathered) and takes a contiguous, work-balanced range of query tiles.

The reference fits UMAP on one GPU with cuML's own kNN (``umap.py:840-850,924-958``).
"""
from __future__ import annotations

import math
import os

from typing import Any, Optional, Tuple

import numpy as np
import torch

from .. import ops

BRUTE_MAX_ROWS = 100_000  # build_algo="auto": exact graph up to this many rows, IVF lists beyond
IVF_LIST_ROWS = 1024      # target rows per inverted list
IVF_NPROBE = 16           # lists probed per query list
# quantiser training: Lloyd iterations and sample rows per list (SRML_IVF_TRAIN_ITERS / _ROWS)
IVF_TRAIN_ITERS = int(os.environ.get("SRML_IVF_TRAIN_ITERS", "10"))
IVF_TRAIN_ROWS = int(os.environ.get("SRML_IVF_TRAIN_ROWS", "64"))


def row_split(n: int, ctx: Any) -> Tuple[int, int]:
    if ctx is None or ctx.world_size <= 1:
        return 0, n
    b = np.linspace(0, n, ctx.world_size + 1).astype(np.int64)
    return int(b[ctx.rank]), int(b[ctx.rank + 1])


def gather_rows(t: torch.Tensor, ctx: Any) -> torch.Tensor:
    if ctx is None or ctx.world_size <= 1:
        return t
    return torch.cat([p.to(t.device) for p in ctx.comm.allgatherv(t.contiguous())], 0)


def refine_sorted(Q: torch.Tensor, I: torch.Tensor, idx: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact squared distances q - i of the selected candidates (no ||q||^2 + ||i||^2 - 2 q.i
    cancellation), sorted ascending; missing candidates (-1) sort last at +inf."""
    r = ops.knn_refine_sort(Q, I, idx)  # fused device kernel (k <= 64, fp32)
    if r is not None:
        return r
    k = idx.shape[1]
    step = max(1, (1 << 26) // max(1, k * Q.shape[1]))
    out = torch.empty(idx.shape, dtype=torch.float32, device=Q.device)
    for s in range(0, Q.shape[0], step):
        rows = I.index_select(0, idx[s: s + step].clamp_min(0).reshape(-1)).view(-1, k, Q.shape[1])
        out[s: s + step] = ((rows - Q[s: s + step].unsqueeze(1)) ** 2).sum(-1)
    out = torch.where(idx >= 0, out, torch.full_like(out, float("inf")))
    d2, j = torch.sort(out, dim=1)
    return d2, idx.gather(1, j)


def knn_graph(Q: torch.Tensor, I: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact (euclidean distances [mq, k] fp32, indices [mq, k] int64) of Q's rows in I."""
    _, idx = ops.knn(Q, I, k, inorm=ops.row_sqnorm(I))
    d2, idx = refine_sorted(Q, I, idx)
    return torch.sqrt(d2.clamp_min(0)), idx


def knn_graph_brute(X: torch.Tensor, k: int, ctx: Any = None) -> Tuple[torch.Tensor, torch.Tensor]:
    lo, hi = row_split(X.shape[0], ctx)
    dist, idx = knn_graph(X[lo:hi], X, k)
    return gather_rows(dist, ctx), gather_rows(idx, ctx)


def record_phase(phases: Optional[dict], name: str, rows: int, t0: float, dev: torch.device) -> float:
    """Per-rank phase log of a distributed graph / layout build: rows this rank processed and the
    phase's wall time (the phase's device work drained first). Returns the new phase start."""
    if phases is None:
        return t0
    import time

    if dev.type == "cuda":
        torch.cuda.current_stream(dev).synchronize()
    t1 = time.perf_counter()
    phases[name] = {"rows": int(rows), "s": round(t1 - t0, 4)}
    return t1


def train_quantizer(X: torch.Tensor, nlist: int, seed: int, iters: Optional[int] = None,
                    train_rows_per_list: Optional[int] = None, ctx: Any = None) -> torch.Tensor:
    """IVF coarse quantiser: Lloyd iterations (fused MFMA nearest-centroid + cluster sums) on a
    row subsample, as IVF trainers do. Distributed (``ctx``, X replicated): every rank draws the
    same sample and seeds, labels its own 1/W of the sample and the cluster sums are all-reduced
    (ONE k x (n + 1) fp64 buffer per iteration): every rank ends with the same centres."""
    m = X.shape[0]
    iters = IVF_TRAIN_ITERS if iters is None else iters
    train_rows_per_list = IVF_TRAIN_ROWS if train_rows_per_list is None else train_rows_per_list
    gen = torch.Generator(device=X.device).manual_seed(int(seed))  # device permutations: no host RNG
    ntrain = min(m, max(nlist * train_rows_per_list, 4 * nlist))
    T = X if ntrain == m else X.index_select(0, torch.randperm(m, generator=gen, device=X.device)[:ntrain])
    C = T.index_select(0, torch.randperm(T.shape[0], generator=gen, device=X.device)[:nlist]).float().clone()
    lo, hi = row_split(T.shape[0], ctx)
    Tl = T[lo:hi].contiguous() if (lo, hi) != (0, T.shape[0]) else T
    dist = ctx is not None and ctx.world_size > 1
    FT = ops.quantizer_planes(Tl) if nlist > 256 and Tl.shape[0] else None  # bucketing only: the filter's arg-min
    tn = ops.row_sqnorm(Tl) if FT is None and Tl.shape[0] else None
    n = X.shape[1]
    for _ in range(max(1, iters)):
        if Tl.shape[0]:
            lab = ops.nearest_list(Tl, C, FT, tn)
            sums, counts = ops.cluster_sums(Tl, lab, nlist)
        else:
            sums = torch.zeros((nlist, n), dtype=torch.float64, device=X.device)
            counts = torch.zeros(nlist, dtype=torch.int64, device=X.device)
        if dist:
            buf = torch.cat([sums.reshape(-1), counts.double()])
            ctx.comm.allreduce(buf)
            sums, counts = buf[: nlist * n].view(nlist, n), buf[nlist * n:]
        C = torch.where(counts.view(-1, 1) > 0, (sums / counts.clamp_min(1).double().view(-1, 1)).float(), C)
    return C.contiguous()


def ivf_tiles(counts: torch.Tensor, off: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(tile_q0, tile_list): <= 128-row query tiles of every list, in row order."""
    nlist = counts.shape[0]
    ntile = (counts + 127) // 128
    tile_list = torch.repeat_interleave(torch.arange(nlist, device=counts.device), ntile)
    first = torch.cumsum(ntile, 0) - ntile
    tile_q0 = off[tile_list] + 128 * (torch.arange(tile_list.shape[0], device=counts.device) - first[tile_list])
    return tile_q0, tile_list


def balanced_tile_range(tile_q0: torch.Tensor, tile_list: torch.Tensor, off: torch.Tensor, counts: torch.Tensor,
                        probes: torch.Tensor, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous tile range of ``rank`` with ~1/world of the work (tile rows x candidate rows)."""
    T = int(tile_list.shape[0])
    if world <= 1 or T == 0:
        return 0, T
    cand = torch.where(probes >= 0, counts[probes.clamp_min(0)], torch.zeros_like(probes)).sum(1)
    rows = torch.minimum(off[tile_list + 1] - tile_q0, torch.full_like(tile_q0, 128))
    cw = torch.cumsum((rows * cand[tile_list]).double(), 0)
    tot = float(cw[-1])
    targets = torch.tensor([tot * r / world for r in range(world + 1)], dtype=torch.float64, device=cw.device)
    cuts = torch.searchsorted(cw, targets).cpu().tolist()
    cuts[0], cuts[-1] = 0, T
    lo = int(min(cuts[rank], T))
    return lo, int(max(lo, min(cuts[rank + 1], T)))


def knn_graph_ivf(X: torch.Tensor, k: int, nlist: Optional[int] = None, nprobe: Optional[int] = None,
                  seed: int = 0, ctx: Any = None, list_order: bool = False, phases: Optional[dict] = None) -> Any:
    """Approximate all-points graph: (euclidean distances [N, k], indices [N, k] int64).

    ``list_order=True`` returns ``(dist, idx, order)`` with the graph left in inverted-list order:
    row i of the graph is original row ``order[i]`` and the indices are list-order positions.
    Rows of one list are neighbours in space, so consumers that gather neighbour rows (the
    spectral SpMM, the layout epochs) read mostly-local memory instead of random rows."""
    import time

    N = X.shape[0]
    nlist = int(nlist) if nlist else max(1, int(round(N / IVF_LIST_ROWS)))
    nlist = max(1, min(nlist, N))
    nprobe = max(1, min(int(nprobe) if nprobe else IVF_NPROBE, nlist, ops.KNN_KMAX))
    t0 = time.perf_counter()
    C = train_quantizer(X, nlist, seed, ctx=ctx)
    ntrain = min(N, max(nlist * IVF_TRAIN_ROWS, 4 * nlist))
    t0 = record_phase(phases, "quantizer", row_split(ntrain, ctx)[1] - row_split(ntrain, ctx)[0], t0, X.device)
    if nlist >= 64:
        # spatial list order: lists grouped by a coarse k-means of their centroids, so the lists a
        # list probes (and a row's neighbours) get nearby ids; everything indexed by list-order
        # position downstream (UMAP's SpMM / epochs) then gathers from a compact window
        kc = max(2, int(round(math.sqrt(nlist))))
        cl = ops.nearest_list(C, train_quantizer(C, kc, seed + 1))
        C = C.index_select(0, torch.argsort(cl.long() * nlist + torch.arange(nlist, device=C.device))).contiguous()
    world = ctx.world_size if ctx is not None else 1
    # bucketing: every rank labels its own row block, the labels are all-gathered (N x 4 B)
    blo, bhi = row_split(N, ctx)
    Xb = X[blo:bhi]
    lab = ops.nearest_list(Xb, C, ops.quantizer_planes(Xb) if nlist > 256 and bhi > blo else None)
    lab = gather_rows(lab.to(torch.int32), ctx)
    t0 = record_phase(phases, "bucketing", bhi - blo, t0, X.device)
    order, off, _ = ops.label_sort(lab, nlist)  # stable counting sort by list
    order = order.long()
    counts = off[1:] - off[:-1]
    Xs = X.index_select(0, order).contiguous()
    xn = ops.row_sqnorm(Xs)
    # probe lists: nearest non-empty lists to each list's centroid (itself first)
    cn = torch.where(counts > 0, ops.row_sqnorm(C), torch.full((nlist,), float("inf"), device=X.device))
    _, probes = ops.knn(C, C, nprobe, inorm=cn, qnorm=torch.zeros(nlist, device=X.device))
    ok = (probes >= 0) & torch.isfinite(cn[probes.clamp_min(0)])
    probes = torch.where(ok, probes, torch.full_like(probes, -1))
    tile_q0, tile_list = ivf_tiles(counts, off)
    T = int(tile_list.shape[0])
    lo, hi = balanced_tile_range(tile_q0, tile_list, off, counts, probes, ctx.rank if world > 1 else 0, world)
    # fp16 centred candidates (knn_lists_f16_ok): a few extra neighbours, re-ranked exactly below
    kc = min(32, k + max(2, k // 4)) if ops.knn_lists_f16_ok(Xs, k, C) else k
    od, oi = ops.knn_lists(Xs, xn, off, probes.int(), tile_q0[lo:hi], tile_list[lo:hi], kc, centroids=C)
    r0 = int(tile_q0[lo]) if lo < T else N
    r1 = int(tile_q0[hi]) if hi < T else N
    d2, pos = refine_sorted(Xs[r0:r1], Xs, oi[r0:r1].long())
    if kc > k:
        d2, pos = d2[:, :k].contiguous(), pos[:, :k].contiguous()
    del od, oi
    d2 = gather_rows(d2, ctx)
    pos = gather_rows(pos, ctx)
    record_phase(phases, "knn_lists", r1 - r0, t0, X.device)
    if list_order:
        fin = torch.isfinite(d2)
        rowmax = torch.where(fin, d2, torch.zeros_like(d2)).max(1, keepdim=True).values
        d2 = torch.where(fin, d2, rowmax)
        return torch.sqrt(d2.clamp_min(0)), torch.where(pos >= 0, pos, torch.full_like(pos, -1)), order
    # back to the original row order; missing neighbours (tiny lists) -> -1 at the row's max distance
    idx = torch.where(pos >= 0, order[pos.clamp_min(0)], torch.full_like(pos, -1))
    fin = torch.isfinite(d2)
    rowmax = torch.where(fin, d2, torch.zeros_like(d2)).max(1, keepdim=True).values
    d2 = torch.where(fin, d2, rowmax)
    dist = torch.empty_like(d2)
    dist[order] = torch.sqrt(d2.clamp_min(0))
    out_i = torch.empty_like(idx)
    out_i[order] = idx
    return dist, out_i


def build_knn_graph(X: torch.Tensor, k: int, build_algo: str = "auto", build_kwds: Optional[dict] = None,
                    seed: int = 0, ctx: Any = None, list_order: bool = False, phases: Optional[dict] = None) -> Any:
    """(dist, idx); with ``list_order`` (dist, idx, order) where ``order`` is None unless the
    builder left the graph in a locality order (see ``knn_graph_ivf``)."""
    algo = (build_algo or "auto").lower()
    if algo == "auto":
        algo = "brute_force_knn" if X.shape[0] <= BRUTE_MAX_ROWS else "ivf"
    kw = dict(build_kwds or {})
    if algo in ("brute_force_knn", "brute", "exact"):
        import time

        t0 = time.perf_counter()
        d, i = knn_graph_brute(X, k, ctx)
        lo, hi = row_split(X.shape[0], ctx)
        record_phase(phases, "knn_brute", hi - lo, t0, X.device)
        return (d, i, None) if list_order else (d, i)
    if algo in ("ivf", "ivfflat", "ivf_flat", "nn_descent"):
        return knn_graph_ivf(X, k, nlist=kw.get("nlist"), nprobe=kw.get("nprobe"), seed=seed, ctx=ctx,
                             list_order=list_order, phases=phases)
    raise ValueError("Unsupported build_algo %r (auto, brute_force_knn, ivf)" % build_algo)
