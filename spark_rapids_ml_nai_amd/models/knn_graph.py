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
IVF_NPROBE = 16           # lists probed per query list (probe="list")
IVF_NPROBE_MAX = 128      # list-probing kernel's probe table (knn_graph.hip F_PMAX)
# per-query probing (probe="query", the default): every row scans the SRML_IVF_QPROBES lists whose
# centres are nearest to IT (not to its list's centre), chosen among the SRML_IVF_POOL x probes
# lists nearest to its list's centre; the device pair kernel keeps <= 32 per row
IVF_PROBE = os.environ.get("SRML_IVF_PROBE", "query")
IVF_QPROBES = int(os.environ.get("SRML_IVF_QPROBES", "32"))
IVF_POOL_MULT = int(os.environ.get("SRML_IVF_POOL", "8"))
IVF_QPROBES_DEV_MAX = 32
IVF_SEED_PROBES = int(os.environ.get("SRML_IVF_SEED_PROBES", "8"))  # list probes of the per-query seed pass
IVF_PAIR_BYTES = int(os.environ.get("SRML_IVF_PAIR_MB", "4096")) << 20  # per-chunk partial-list budget
IVF_PAIR_H16 = os.environ.get("SRML_IVF_PAIR_H16", "1") == "1"  # pre-centred fp16 items for the pair search
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
            sums = ops.zeros((nlist, n), dtype=torch.float64, device=X.device)
            counts = ops.zeros(nlist, dtype=torch.int64, device=X.device)
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


def row_tile_range(tile_q0: torch.Tensor, N: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous tile range of ``rank`` holding ~N / world rows (cuts on tile boundaries): the
    per-query probing work is about the same per row."""
    T = int(tile_q0.shape[0])
    if world <= 1 or T == 0:
        return 0, T
    targets = torch.tensor([N * r // world for r in range(world + 1)], dtype=tile_q0.dtype, device=tile_q0.device)
    cuts = torch.searchsorted(tile_q0, targets).cpu().tolist()
    cuts[0], cuts[-1] = 0, T
    return int(cuts[rank]), int(max(cuts[rank], cuts[rank + 1]))


def query_probe_search(Xs: torch.Tensor, xn: torch.Tensor, C: torch.Tensor, counts: torch.Tensor,
                       off: torch.Tensor, tile_q0: torch.Tensor, tile_list: torch.Tensor, tlo: int, thi: int, k: int,
                       kc: int, p: int, seed_probes: int = IVF_SEED_PROBES, pool_mult: int = IVF_POOL_MULT,
                       phases: Optional[dict] = None) -> Tuple[torch.Tensor, torch.Tensor, int, int]:
    """Per-query IVF probing over the query tiles ``tlo .. thi`` (rows r0 .. r1 of the list-sorted
    ``Xs``): (exact squared distances (r1 - r0, k), sorted positions int64, r0, r1).

    1. seed: list probing with ``seed_probes`` lists (every row of list c scans the lists nearest
       to c's centre; the dense tile kernel), re-ranked exactly: each row's k-th distance so far;
    2. pool: each list's ``pool_mult * p`` nearest lists by centre (one small C x C kNN); probes:
       each row's ``p`` nearest pool centres (``ops.knn_pool_probes``, fp16 MFMA tiles), minus the
       lists the seed already scanned;
    3. inverted search: the (row, list) pairs are grouped by list with the counting sort, every
       128-pair tile of list l is matched against l's items (``ops.knn_pairs``) keeping only items
       below the row's seeded threshold, then the seed's and the pairs' candidates are merged by
       the radix select and the ``kc`` best re-ranked exactly.
    Rows are processed in chunks that bound the partial lists to ``IVF_PAIR_BYTES``."""
    import time

    N = Xs.shape[0]
    nlist = C.shape[0]
    dev = Xs.device
    T = int(tile_q0.shape[0])
    r0 = int(tile_q0[tlo]) if tlo < T else N
    r1 = int(tile_q0[thi]) if thi < T else N
    if r1 <= r0:
        e = torch.empty((0, k), device=dev)
        return e, e.long(), r0, r1
    t0 = time.perf_counter()
    nonempty = int((counts > 0).sum())
    cn = torch.where(counts > 0, ops.row_sqnorm(C), torch.full((nlist,), float("inf"), device=dev))
    zero = ops.zeros(nlist, device=dev)
    # 1. seed: list probing, exact re-rank
    s1 = max(1, min(int(seed_probes), nonempty, IVF_NPROBE_MAX))
    _, probes1 = ops.knn(C, C, s1, inorm=cn, qnorm=zero)
    probes1 = torch.where(torch.isfinite(cn[probes1.clamp_min(0)]) & (probes1 >= 0), probes1,
                          torch.full_like(probes1, -1)).int()
    od, oi = ops.knn_lists(Xs, xn, off, probes1, tile_q0[tlo:thi], tile_list[tlo:thi], kc, centroids=C)
    d2s, poss = refine_sorted(Xs[r0:r1], Xs, oi[r0:r1].long())
    del od, oi
    # the fp16 keys of the pair search carry ~1e-3 relative rounding: a 1 % slack keeps every item
    # that can still enter the row's exact top k
    thr = torch.full((N,), float("inf"), dtype=torch.float32, device=dev)
    thr[r0:r1] = d2s[:, min(k, d2s.shape[1]) - 1] * 1.01 + 1e-30
    t0 = record_phase(phases, "query_seed", r1 - r0, t0, dev)
    # 2. probes
    cap = IVF_QPROBES_DEV_MAX if ops.knn_lists_f16_ok(Xs, kc, C) else nonempty
    p = max(1, min(int(p), nonempty, cap))
    P = max(p, min(nonempty, int(pool_mult) * p))
    _, pool = ops.knn(C, C, P, inorm=cn, qnorm=zero)
    probes = ops.knn_pool_probes(Xs, off, C, pool.int(), tile_q0[tlo:thi], tile_list[tlo:thi], p, r0, r1)
    t0 = record_phase(phases, "query_probes", r1 - r0, t0, dev)
    # 3. pairs, in row chunks; the items of the pair search are centred on their own list: one fp16
    # copy of the rows serves every pair tile (IVF_PAIR_H16=0: convert per tile instead)
    items_f16 = (ops.center_rows_f16(Xs, C, off) if IVF_PAIR_H16 and Xs.is_cuda and ops.knn_lists_f16_ok(Xs, kc, C)
                 else None)
    rows_per_chunk = max(128, IVF_PAIR_BYTES // (p * kc * 8))
    d_parts, p_parts = [], []
    ta = tlo
    while ta < thi:
        ca = int(tile_q0[ta])
        tb = min(thi, int(torch.searchsorted(tile_q0, torch.tensor([ca + rows_per_chunk], device=dev,
                                                                       dtype=tile_q0.dtype)).item()))
        tb = max(tb, ta + 1)
        cb = int(tile_q0[tb]) if tb < T else N
        pr = probes[ca - r0: cb - r0].long()
        rlist = torch.bucketize(torch.arange(ca, cb, device=dev), off[1:], right=True)
        seen = (probes1[rlist].long().unsqueeze(1) == pr.unsqueeze(2)).any(2)  # scanned by the seed
        flat = torch.where(seen | (pr < 0), torch.full_like(pr, -1), pr).reshape(-1)
        del seen, rlist, pr
        perm, poff, _ = ops.label_sort(flat, nlist)  # pairs grouped by probed list; dropped pairs trail
        perm = perm[: int(poff[-1])].long()
        qrows = (ca + perm // p).int()
        pt_q0, pt_list = ivf_tiles(poff[1:] - poff[:-1], poff)
        odp, oip = ops.knn_pairs(Xs, off, C, poff, qrows, perm.int(), pt_q0, pt_list, kc, (cb - ca) * p,
                                 thr_row=thr, items_f16=items_f16)
        del qrows, perm, flat
        vals = torch.cat([d2s[ca - r0: cb - r0], odp.view(cb - ca, p * kc)], 1)
        ids = torch.cat([poss[ca - r0: cb - r0], oip.view(cb - ca, p * kc).long()], 1)
        del odp, oip
        _, cand = ops.topk_rows(vals, kc, ids=ids)
        del vals, ids
        d2, pos = refine_sorted(Xs[ca:cb], Xs, cand)
        d_parts.append(d2[:, :k])
        p_parts.append(pos[:, :k])
        ta = tb
    record_phase(phases, "query_pairs", r1 - r0, t0, dev)
    return torch.cat(d_parts), torch.cat(p_parts), r0, r1


NND_ITERS = int(os.environ.get("SRML_NND_ITERS", "2"))  # refinement rounds of build_algo="nn_descent"
NND_CHUNK_ROWS = 1 << 21


def nn_descent_refine(Xs: torch.Tensor, d2: torch.Tensor, pos: torch.Tensor, k: int, iters: int = NND_ITERS,
                      a: int = 8, b: int = 8, R: int = 16, ctx: Any = None,
                      phases: Optional[dict] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """NN-descent refinement of an all-points graph (``pos``: N x k row ids of ``Xs``, ``d2``:
    their squared distances): per round, every row re-ranks exactly the union of its neighbours,
    its first ``a`` neighbours' first ``b`` neighbours and up to ``R`` reverse neighbours (rows
    that list it), de-duplicated, and keeps the k nearest. A neighbour's neighbour or a reverse
    neighbour is the join of NN-descent (Dong et al. 2011) evaluated from the row's side: every row
    writes only its own list, so no atomics. Reverse lists come from one stable grouping of the
    N k edges by target. Distributed (``ctx``): each rank refines a row block of the replicated
    graph, the blocks are all-gathered after every round.

    It pays off on a graph that is already good (per-query IVF: recall 0.64 -> 0.69 -> 0.71 in two
    rounds on 200k classification rows) and barely moves a poor one (list probing: 0.375 -> 0.380,
    the round-5 experiment's finding)."""
    import time

    t0 = time.perf_counter()
    N = Xs.shape[0]
    dev = Xs.device
    lo, hi = row_split(N, ctx)
    for _ in range(max(0, int(iters))):
        tgt = pos.reshape(-1)
        # reverse neighbours: edges grouped by target (stable: the source order is kept)
        if tgt.is_cuda and N <= int(ops.native.lib().srml_label_sort_kmax()):
            perm, off, _ = ops.label_sort(tgt.clamp_min(0).int(), N)
            perm = perm.long()
        else:
            srt, perm = torch.sort(tgt, stable=True)
            off = torch.searchsorted(srt, torch.arange(N + 1, device=dev, dtype=srt.dtype))
        d_parts, p_parts = [], []
        for c0 in range(lo, hi, NND_CHUNK_ROWS):
            c1 = min(hi, c0 + NND_CHUNK_ROWS)
            own = pos[c0:c1]
            non = pos.index_select(0, own[:, :a].clamp_min(0).reshape(-1))[:, :b].reshape(c1 - c0, a * b)
            non = torch.where(own[:, :a].repeat_interleave(b, 1) >= 0, non, torch.full_like(non, -1))
            st = off[c0:c1].unsqueeze(1) + torch.arange(R, device=dev)
            ok = st < off[c0 + 1: c1 + 1].unsqueeze(1)
            rev = torch.where(ok, perm[st.clamp_max(perm.numel() - 1)] // k, torch.full_like(st, -1))
            cand = torch.sort(torch.cat([own, non, rev], 1), dim=1).values
            dup = torch.zeros_like(cand, dtype=torch.bool)
            dup[:, 1:] = cand[:, 1:] == cand[:, :-1]
            cand = torch.where(dup, torch.full_like(cand, -1), cand)
            dd, pp = refine_sorted(Xs[c0:c1], Xs, cand)
            d_parts.append(dd[:, :k])
            p_parts.append(pp[:, :k])
        d2 = gather_rows(torch.cat(d_parts), ctx) if d_parts else d2[lo:hi]
        pos = gather_rows(torch.cat(p_parts), ctx) if p_parts else pos[lo:hi]
    record_phase(phases, "nn_descent", hi - lo, t0, dev)
    return d2, pos


def knn_graph_ivf(X: torch.Tensor, k: int, nlist: Optional[int] = None, nprobe: Optional[int] = None,
                  seed: int = 0, ctx: Any = None, list_order: bool = False, phases: Optional[dict] = None,
                  probe: Optional[str] = None, nnd_iters: int = 0) -> Any:
    """Approximate all-points graph: (euclidean distances [N, k], indices [N, k] int64).

    ``list_order=True`` returns ``(dist, idx, order)`` with the graph left in inverted-list order:
    row i of the graph is original row ``order[i]`` and the indices are list-order positions.
    Rows of one list are neighbours in space, so consumers that gather neighbour rows (the
    spectral SpMM, the layout epochs) read mostly-local memory instead of random rows."""
    import time

    N = X.shape[0]
    nlist = int(nlist) if nlist else max(1, int(round(N / IVF_LIST_ROWS)))
    nlist = max(1, min(nlist, N))
    probe = (probe or IVF_PROBE).lower()
    if probe not in ("query", "list"):
        raise ValueError("probe must be 'query' or 'list', got %r" % probe)
    if probe == "query":
        qprobes = int(nprobe) if nprobe else IVF_QPROBES
    nprobe = max(1, min(int(nprobe) if nprobe else IVF_NPROBE, nlist, IVF_NPROBE_MAX))
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
        if ctx is not None and ctx.world_size > 1:
            # the reorder ran on every rank alone and its cluster sums fold with fp64 atomics (order-
            # dependent rounding): rank 0's lists are THE lists, or ranks could mix list ids in the
            # all-gathered labels (one nlist x n broadcast)
            ctx.comm.broadcast(C, src=0)
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
    tile_q0, tile_list = ivf_tiles(counts, off)
    T = int(tile_list.shape[0])
    # fp16 centred candidates (knn_lists_f16_ok): a few extra neighbours, re-ranked exactly below
    kc = min(32, k + max(2, k // 4)) if ops.knn_lists_f16_ok(Xs, k, C) else k
    if probe == "query" and X.is_cuda and not ops.knn_lists_f16_ok(Xs, kc, C):
        probe = "list"  # no device pair kernel for these rows (n > 128 or k > 32): the list kernels
    if probe == "query":
        lo, hi = row_tile_range(tile_q0, N, ctx.rank if world > 1 else 0, world)
        d2, pos, r0, r1 = query_probe_search(Xs, xn, C, counts, off, tile_q0, tile_list, lo, hi, k, kc, qprobes,
                                             phases=phases)
    else:
        # probe lists: nearest non-empty lists to each list's centroid (itself first)
        cn = torch.where(counts > 0, ops.row_sqnorm(C), torch.full((nlist,), float("inf"), device=X.device))
        _, probes = ops.knn(C, C, nprobe, inorm=cn, qnorm=ops.zeros(nlist, device=X.device))
        ok = (probes >= 0) & torch.isfinite(cn[probes.clamp_min(0)])
        probes = torch.where(ok, probes, torch.full_like(probes, -1))
        lo, hi = balanced_tile_range(tile_q0, tile_list, off, counts, probes, ctx.rank if world > 1 else 0, world)
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
    if nnd_iters > 0:
        d2, pos = nn_descent_refine(Xs, d2, pos, k, iters=nnd_iters, ctx=ctx, phases=phases)
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
        # nn_descent: the per-query IVF graph refined by NN-descent rounds (build_kwds "nnd_iters")
        nnd = int(kw.get("nnd_iters", NND_ITERS)) if algo == "nn_descent" else int(kw.get("nnd_iters", 0))
        return knn_graph_ivf(X, k, nlist=kw.get("nlist"), nprobe=kw.get("nprobe"), seed=seed, ctx=ctx,
                             list_order=list_order, phases=phases, probe=kw.get("probe"), nnd_iters=nnd)
    raise ValueError("Unsupported build_algo %r (auto, brute_force_knn, ivf, nn_descent)" % build_algo)
