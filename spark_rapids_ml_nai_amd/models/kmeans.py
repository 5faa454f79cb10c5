"""Distributed KMeans (Lloyd) with random and k-means|| initialisation.

Reference: cuML ``KMeansMG.fit`` (``clustering.py:348-384``) — k-means||, Lloyd iterations with a
per-iteration centroid all-reduce. Per iteration and rank on MI355X:

1. ``nearest_centroid`` — fused MFMA distance GEMM + arg-min (no m x k matrix),
2. ``cluster_sums`` — per-cluster sums/counts (LDS-privatised or row-coalesced atomics),
3. ONE coalesced all-reduce of [sums (k·n), counts (k), inertia] in fp64 over RCCL,
4. centroid update / Spark convergence test (every centre moved <= tol) on the device.

Initialisation:
* ``random`` — k distinct global rows drawn with one seeded generator shared by all ranks;
  the owning rank contributes each row and an all-reduce assembles the centres;
* ``k-means||`` (``scalable-k-means++``) — ``init_steps`` rounds of D^2 over-sampling with
  factor ``oversampling_factor * k`` (device RNG), candidates all-gathered, weighted by the
  number of points they attract, then reduced to k centres with weighted k-means++ seeding +
  weighted Lloyd on the device (Spark's LocalKMeans step).
"""
from __future__ import annotations

import os
import time

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..utils.determinism import deterministic
from ..parallel.context import PartitionDescriptor, WorkerContext


def _global_rows(X: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext, idx: np.ndarray) -> torch.Tensor:
    """Gather rows with the given global indices onto every rank (owner contributes, all-reduce)."""
    n = X.shape[1]
    start = sum(s for r, s in desc.parts_rank_size if r < desc.rank)
    stop = start + X.shape[0]
    out = ops.zeros((len(idx), n), dtype=torch.float64, device=X.device)
    mine = np.nonzero((idx >= start) & (idx < stop))[0]
    if len(mine):
        rows = torch.from_numpy(idx[mine] - start).to(X.device)
        out[torch.from_numpy(mine).to(X.device)] = X.index_select(0, rows).double()
    ctx.comm.allreduce(out)
    return out


def sample_distinct(m: int, k: int, seed: int) -> np.ndarray:
    """``min(k, m)`` distinct integers of [0, m), sorted, in O(k) time and memory (draw, de-duplicate,
    redraw the shortfall); ``Generator.choice(m, k, replace=False)`` costs time in m (13 ms at 100M
    rows on the build host, 0.4 ms here). Every rank draws the same set from the same seed."""
    k = min(int(k), int(m))
    if 4 * k >= m:
        return np.sort(np.random.default_rng(seed).permutation(m)[:k])
    rng = np.random.default_rng(seed)
    got = np.unique(rng.integers(0, m, size=k))
    while got.size < k:
        got = np.unique(np.concatenate([got, rng.integers(0, m, size=2 * (k - got.size))]))
    if got.size > k:
        got = np.sort(rng.permutation(got)[:k])
    return got


def init_random(X: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext, k: int, seed: int) -> torch.Tensor:
    idx = sample_distinct(desc.m, k, seed)
    C = _global_rows(X, desc, ctx, idx)
    if C.shape[0] < k:  # fewer rows than clusters: duplicate
        C = C[torch.arange(k, device=C.device) % C.shape[0]]
    return C


def _weighted_lloyd(P: torch.Tensor, w: torch.Tensor, C: torch.Tensor, iters: int = 30) -> torch.Tensor:
    """Weighted Lloyd on the (small) candidate set (Spark's LocalKMeans step): the fused distance /
    arg-min kernel, the cluster-sum kernel over the pre-weighted rows; stops as soon as no
    candidate changes cluster (the centres are then a fixed point)."""
    Pf = P.float().contiguous()
    pn = ops.row_sqnorm(Pf) if Pf.is_cuda else (Pf * Pf).sum(1)
    k = C.shape[0]
    Pw = (P.double() * w.double().view(-1, 1)).float().contiguous()
    wd = w.double()
    C = C.double()
    prev = None
    for _ in range(iters):
        lab, _ = ops.nearest_centroid(Pf, C.float(), pn)
        if prev is not None and torch.equal(lab, prev):
            break
        prev = lab
        sums, _ = ops.cluster_sums(Pw, lab, k)
        cnt = ops.zeros(k, dtype=torch.float64, device=P.device).index_add_(0, lab.long(), wd)
        C = torch.where(cnt.view(-1, 1) > 0, sums / cnt.clamp_min(1e-300).view(-1, 1), C)
    return C


def init_kmeans_parallel(X: torch.Tensor, xnorm: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext,
                         k: int, seed: int, oversampling: float = 2.0, steps: int = 2,
                         XP: Optional[torch.Tensor] = None, trials: int = 1, mu: Optional[torch.Tensor] = None,
                         xnorm_split: Optional[torch.Tensor] = None, F16: Any = None) -> torch.Tensor:
    """k-means|| (scalable k-means++, reference cuML ``init="scalable-k-means++"`` / Spark
    ``initMode="k-means||"``): ``steps`` rounds of D^2 over-sampling (ell = oversampling * k rows
    per round, device RNG), candidates all-gathered, weighted by the rows they attract, then reduced
    to k centres by ``trials`` (Spark: 1) seeded weighted k-means++ draws on the device
    (``kmeanspp_gram``: distances from the candidates' MFMA Gram matrix) + weighted Lloyd, keeping
    the lowest cost.
    The distance passes over X use the split-bf16 MFMA kernel when the Lloyd loop will (``XP``),
    in its 3-product approximate form (D^2 sampling and candidate weights tolerate ~1e-5
    relative distance error; half the MFMA work of the exact Lloyd passes), or — ``F16`` given
    (``ops.F16Planes``) — the Lloyd loop's fp16 filter pass with radius 0 (its own arg-min, ~1e-3
    relative distance error at worst; only exact ties re-searched): near-equidistant random
    candidates would otherwise send most rows to the exact re-search."""
    dev = X.device
    m = X.shape[0]

    def nearest(C: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        if F16 is not None:  # D^2 sampling / weights: the filter's own arg-min, no re-search
            return ops.nearest_centroid_f16(F16, C.float(), approx=True)
        if XP is not None:  # sampling / weighting only need approximate distances
            return ops.nearest_centroid_split(XP, m, C.float(), xnorm if xnorm_split is None else xnorm_split,
                                              approx=True, mu=mu)
        return ops.nearest_centroid(X, C.float(), xnorm)

    rng = np.random.default_rng(seed)
    C = _global_rows(X, desc, ctx, np.array([int(rng.integers(0, desc.m))]))
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed) * 1000003 + ctx.rank)
    ell = oversampling * k
    # running (min d^2, arg-min) over all candidates so far: each pass only scores the centres
    # added by the previous round, and the candidate weights come from the same running arg-min
    best_d2 = best_lab = None
    new = C
    for r in range(max(1, steps) + 1):
        lab, d2 = nearest(new)
        off = C.shape[0] - new.shape[0]
        if best_d2 is None:
            best_d2, best_lab = d2, lab.long() + off
        else:
            better = d2 < best_d2
            best_d2 = torch.where(better, d2, best_d2)
            best_lab = torch.where(better, lab.long() + off, best_lab)
        if r == max(1, steps):
            break
        phi = best_d2.double().sum().view(1)
        ctx.comm.allreduce(phi)
        p = (ell * best_d2.double() / phi.clamp_min(1e-300)).clamp_max(1.0)
        pick = torch.rand(X.shape[0], generator=gen, device=dev, dtype=torch.float64) < p
        local = X[pick].double()
        parts = ctx.comm.allgatherv(local)
        new = torch.cat([q.to(dev) for q in parts], 0)
        if new.shape[0] == 0:
            break
        C = torch.cat([C, new], 0)
    # weight every candidate by the points it attracts
    w = ops.label_counts(best_lab, C.shape[0]).double()
    ctx.comm.allreduce(w)
    if C.shape[0] <= k:
        extra = init_random(X, desc, ctx, k - C.shape[0], seed + 1) if C.shape[0] < k else None
        return torch.cat([C, extra], 0) if extra is not None else C
    Cf = C.float().contiguous()
    G = ops.gram(Cf.T.contiguous()) if Cf.is_cuda else Cf.double() @ Cf.double().T  # C C^T (nc x nc)
    cn = ops.row_sqnorm(Cf) if Cf.is_cuda else (Cf * Cf).sum(1)
    best, best_cost = None, float("inf")
    for t in range(max(1, trials)):
        idx = ops.kmeanspp_gram(G, w, k, int(seed) * 7919 + t)
        Ct = _weighted_lloyd(C, w, C[idx])
        if trials <= 1:
            return Ct
        _, d2 = ops.nearest_centroid(Cf, Ct.float(), cn)
        cost = float((d2.double() * w).sum().item())
        if cost < best_cost:
            best, best_cost = Ct, cost
    return best


DELTA_FRAC = 0.2  # moved-row fraction below which the Lloyd sums are updated incrementally
# a full cluster-sum pass re-anchors the incrementally updated sums after this many delta updates
# (bounds the fp64 rounding of the +x / -x chains; cuML recomputes every iteration)
REANCHOR = max(1, int(os.environ.get("SRML_KMEANS_REANCHOR", "16")))


def _use_split(X: torch.Tensor, k: int) -> bool:
    """Split-bf16 distance GEMM (fp32-exact, 6 bf16 MFMA products = 6/16 of the fp32 MFMA cost)
    when the Lloyd step is GEMM-bound (k and n large) and the 1.5x-of-X planes fit in HBM.
    ``SRML_KMEANS_SPLIT=0/1`` forces it off/on."""
    import os
    env = os.environ.get("SRML_KMEANS_SPLIT")
    if env is not None:
        return env == "1"
    if not X.is_cuda or X.dtype != torch.float32:
        return False
    m, n = X.shape
    if k < 128 or n < 128:
        return False
    if m > ops.split_rows_per_launch(k):  # the 3-product / exact split kernels launch all rows at once
        return False
    need = 3 * 2 * ((m + 127) // 128 * 128) * ((n + 15) // 16 * 16)
    free, _ = torch.cuda.mem_get_info(X.device)
    return need < 0.6 * free


def _now(X: torch.Tensor) -> float:
    if X.is_cuda:  # this stream only: a device-wide sync would also wait for a streamed ingest's copies
        torch.cuda.current_stream(X.device).synchronize()
    return time.perf_counter()


LLOYD_BATCH = int(os.environ.get("SRML_LLOYD_BATCH", "4"))
# small-k MFMA loop: keep every row's label and, once under 1/4 of the rows move per step, sum only
# the moved rows' change: the one-hot GEMM runs on the tiles holding a moved row (=0: off)
LLOYD_SMALL_DELTA = os.environ.get("SRML_LLOYD_SMALL_DELTA", "1") == "1"


def _lloyd_small_loop(X: torch.Tensor, C: torch.Tensor, ctx: WorkerContext, k: int, max_iter: int,
                      tol2: float) -> Tuple[torch.Tensor, int, float]:
    """Device-resident small-k Lloyd loop (k <= 32, n <= 64): per iteration ONE fused step (labels,
    sums, counts, inertia into the all-reduce buffer), the all-reduce, and the device centre update
    (new centres, shift, convergence flag) — three launches, no host sync. The convergence flag is
    copied back asynchronously once per LLOYD_BATCH iterations and read one batch late (the steps
    launched after convergence return at once), like the device L-BFGS loop. With the label book
    (MFMA kernel, LLOYD_SMALL_DELTA) a step after one with few moved rows is a DELTA step: its
    one-hot GEMM sums only the moved rows' change (onehot(new) - onehot(old)) and is skipped on
    tiles without one, and the update adds the change to the running sums (the reduced buffer
    then carries changes on every rank alike: the mode follows the reduced moved count)."""
    n = X.shape[1]
    dev = X.device
    # MFMA kernel: no per-row outputs (0.8 GB of label / distance writes per 100M-row step saved),
    # and the loop runs in coordinates centred on the initial centres' mean (the kernel stages
    # x - mu; its per-wave fp32 sums then carry the data's spread, not its offset from the origin)
    rows_out = ops.lloyd_kernel() != "mfma"
    mu = None if rows_out else C.double().mean(0)
    C64 = (C.double() - mu).contiguous() if mu is not None else C.double().contiguous()
    C32 = C64.float().contiguous()
    cn = (C32 * C32).sum(1).contiguous()
    use_book = not rows_out and LLOYD_SMALL_DELTA
    buf = ops.zeros(k * n + k + 2, dtype=torch.float64, device=dev)
    mu32 = mu.float().contiguous() if mu is not None else None
    labels = dist = None
    if rows_out:
        labels = torch.empty(X.shape[0], dtype=torch.int32, device=dev)
        dist = torch.empty(X.shape[0], dtype=torch.float32, device=dev)
    flags = ops.zeros(3, dtype=torch.int32, device=dev)  # [done, iterations, delta mode]
    book = G = None
    if use_book:
        m = X.shape[0]
        book = (torch.empty(m, dtype=torch.int32, device=dev), flags[2:3])
        G = torch.empty(k * n + k, dtype=torch.float64, device=dev)
    stat = ops.zeros(2, dtype=torch.float64, device=dev)  # [inertia, max shift] of the last update
    host = ops.zeros((2, 3), dtype=torch.int32, pin_memory=True)
    stream = torch.cuda.current_stream(dev)
    pending: List[Any] = []
    it = j = 0
    while it < max_iter:
        for _ in range(min(max(1, LLOYD_BATCH), max_iter - it)):
            buf.zero_()
            ops.kmeans_lloyd_small(X, C32, cn, out=buf, done=flags, labels=labels, dist=dist, rows_out=rows_out,
                                   mu=mu32, book=book)
            ctx.comm.allreduce(buf)
            ops.kmeans_small_update(buf, k, n, C64, C32, cn, tol2, flags, stat, G=G)
            it += 1
        slot = host[j % 2]
        slot.copy_(flags, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        pending.append((ev, slot))
        j += 1
        if len(pending) >= 2:
            ev0, s0 = pending.pop(0)
            ev0.synchronize()
            if int(s0[0]):
                break
    fl = flags.cpu()
    if mu is not None:
        C64 = C64 + mu
    return C64, int(fl[1]), float(stat[0].item())


def _lloyd_f16_loop(X: torch.Tensor, F16: Any, C: torch.Tensor, ctx: WorkerContext, k: int, max_iter: int,
                    tol2: float) -> Tuple[torch.Tensor, int, float, int]:
    """Lloyd iterations on the fp16 certified filter with device bookkeeping: per iteration the
    search (``ops.nearest_centroid_f16``), the moved-row count, a delta or full cluster-sum update
    of the local [sums | counts | inertia] buffer, ONE all-reduce of it, and the in-place centre
    update whose (max shift, inertia) read-back is the iteration's convergence test. Returns
    (centres fp64, iterations, inertia of the last search, delta iterations)."""
    m, n = X.shape
    kn = k * n
    L = torch.empty(kn + k + 1, dtype=torch.float64, device=X.device)
    G = torch.empty_like(L)
    book = ops.LloydBook(X, k)
    C = C.to(device=X.device, dtype=torch.float64).contiguous()
    prev = None
    n_iter = n_delta = last_anchor = 0
    inertia = 0.0
    for it in range(max(0, max_iter)):
        n_iter = it + 1
        labels, d2 = ops.nearest_centroid_f16(F16, C)
        nm = book.moved(labels, prev) if prev is not None else -1
        if nm < 0 or nm > DELTA_FRAC * m or (n_delta and n_delta % REANCHOR == 0 and n_delta != last_anchor):
            book.full_into(X, labels, L)
            last_anchor = n_delta
        elif nm:
            book.delta_into(X, labels, prev, nm, L)
            n_delta += 1
        book.inertia_into(d2, L)
        G.copy_(L)
        ctx.comm.allreduce(G)
        shift, inertia = book.update(G, C)
        prev = labels
        if shift <= tol2:
            break
    return C, n_iter, inertia, n_delta


def kmeans_fit(X: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext, k: int, max_iter: int, tol: float,
               seed: int, init: str = "scalable-k-means++", oversampling: float = 2.0, init_steps: int = 2,
               timer: Any = None) -> Dict[str, Any]:
    n = X.shape[1]
    t_start = _now(X)
    # k > 256: 256 x 256 LDS-DMA kernel on the tiled plane layout (SRML_SPLIT_TILED=0: plain layout)
    tiled = k > 256 and os.environ.get("SRML_SPLIT_TILED", "1") == "1"
    use_split = _use_split(X, k)
    centred = use_split and tiled and X.is_cuda
    xnorm = None if centred else ops.row_sqnorm(X)  # the centred searches use ||x - mu||^2 only
    # filter-and-refine Lloyd search on the tiled planes: 3-product pass + exact re-search of the
    # near-tie rows (SRML_KMEANS_CERTIFIED=0: always the 6-product search). The split search runs
    # on centred data (planes of X - mu, centroids - mu, ||x - mu||^2): distances are unchanged,
    # and the dropped-product error bound scales with ||x - mu|| ||c - mu||, far below the gaps.
    certified = tiled and use_split and X.is_cuda and os.environ.get("SRML_KMEANS_CERTIFIED", "1") == "1"
    # SRML_KMEANS_FILTER=f16 (default): the certified filter is ONE fp16 MFMA product per (row,
    # centre) on a scaled fp16 plane of X - mu (ops.F16Planes; a third of the 3-product bf16
    # filter's MFMAs) with a radius ~2.8x wider; bf16: the 3-product split-bf16 filter
    mu = None
    xnorm_s = xnorm
    F16 = None
    if centred:
        mu = ops.col_moments(X, need_sq=False)[0].div_(max(X.shape[0], 1)).float()
        if certified and ops.kmeans_filter_mode() == "f16":
            F16 = ops.F16Planes(X, mu)
            if F16.ok:
                xnorm_s = F16.xnorm
            else:
                F16 = None
        if F16 is None:
            xnorm_s = ops.row_sqnorm(X, mu)
    XP = ops.split_bf16x3(X, tiled=tiled, mu=mu) if use_split and F16 is None else None
    t_prep = _now(X)
    if init in ("random",):
        C = init_random(X, desc, ctx, k, seed)
    elif init in ("scalable-k-means++", "k-means||", "k-means++"):
        C = init_kmeans_parallel(X, xnorm, desc, ctx, k, seed, oversampling, init_steps, XP=XP, mu=mu,
                                 xnorm_split=xnorm_s, F16=F16)
    else:
        raise ValueError("Unsupported init mode %s" % init)
    C = C.double()
    t_init = _now(X)
    tol2 = float(tol) ** 2
    n_iter = 0
    inertia = 0.0
    st0 = dict(ops._CERTIFY_STATS)
    # cluster sums are kept per rank and updated by the rows that changed cluster (+x into the new
    # cluster, -x out of the old; fp64) once fewer than DELTA_FRAC of them move — a late Lloyd
    # iteration moves ~1 % of the rows, so it reads ~1 % of X instead of all of it; a full pass
    # otherwise (and always in deterministic mode)
    prev = None
    sums_l = counts_l = None
    n_delta = 0
    last_anchor = 0
    # k <= 32, n <= 64 (the BASELINE k = 20 on 100M x 64): the fused one-pass step gives labels,
    # full cluster sums and the inertia together (no delta bookkeeping needed)
    fused_small = F16 is None and XP is None and ops.lloyd_small_ok(X, k) and not deterministic()
    # the fp16 certified filter on the device: the whole iteration's bookkeeping runs in native
    # kernels (ops.LloydBook), same delta / re-anchor schedule as the loop below
    booked = F16 is not None and X.is_cuda and not deterministic() and os.environ.get("SRML_LLOYD_BOOK", "1") == "1"
    if fused_small:
        C, n_iter, inertia = _lloyd_small_loop(X, C, ctx, k, max_iter, tol2)
    elif booked:
        C, n_iter, inertia, n_delta = _lloyd_f16_loop(X, F16, C, ctx, k, max_iter, tol2)
    for it in range(max(0, max_iter) if not (fused_small or booked) else 0):
        n_iter = it + 1
        if F16 is not None:
            labels, d2 = ops.nearest_centroid_f16(F16, C)  # fp64 centres: centred + rounded in its prep kernel
        elif XP is not None:
            labels, d2 = ops.nearest_centroid_split(XP, X.shape[0], C.float(), xnorm_s, X=X if certified else None,
                                                    mu=mu)
        else:
            labels, d2 = ops.nearest_centroid(X, C.float(), xnorm)
        moved = None
        if prev is not None and X.is_cuda and not deterministic():
            moved = torch.nonzero(labels != prev).view(-1)
            if moved.numel() > DELTA_FRAC * X.shape[0] or (n_delta and n_delta % REANCHOR == 0 and
                                                           n_delta != last_anchor):
                moved = None
        if moved is None:
            sums_l, counts_l = ops.cluster_sums(X, labels, k)
            last_anchor = n_delta
        elif moved.numel():
            ds, dc = ops.cluster_delta_sums(X, moved, labels.index_select(0, moved), prev.index_select(0, moved), k)
            sums_l += ds
            counts_l = counts_l + dc
            n_delta += 1
        prev = labels
        sums, counts = sums_l, counts_l
        buf = torch.cat([sums.view(-1), counts.double(), d2.double().sum().view(1)])
        ctx.comm.allreduce(buf)
        sums = buf[: k * n].view(k, n)
        counts = buf[k * n: k * n + k]
        inertia = float(buf[-1].item()) if it == max_iter - 1 else inertia
        newC = torch.where(counts.view(-1, 1) > 0, sums / counts.clamp_min(1.0).view(-1, 1), C)
        shift = float(((newC - C) ** 2).sum(1).max().item())
        C = newC
        if shift <= tol2:
            break
    del XP, F16
    t_end = _now(X)
    return {
        "cluster_centers_": C.cpu().numpy(),  # ndarray: 3M-float .tolist() cost 40 ms per fit
        "n_cols": int(n),
        "dtype": "float32" if X.dtype == torch.float32 else "float64",
        "n_iter": n_iter,
        # filter-and-refine Lloyd search: fraction of row assignments re-searched exactly
        "delta_iters": n_delta,  # iterations whose cluster sums were updated from the moved rows only
        # rank-local phase times (s): planes / means, seeding, Lloyd loop (each ends on a device sync;
        # the Lloyd loop syncs every iteration for its shift test anyway)
        "phase_s": [round(t_prep - t_start, 4), round(t_init - t_prep, 4), round(t_end - t_init, 4)],
        "refined_frac": round((ops._CERTIFY_STATS["refined"] - st0["refined"]) /
                              max(1, ops._CERTIFY_STATS["rows"] - st0["rows"]), 4) if certified else None,
    }


def kmeans_predict(X: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    """Labels of ``X`` under centres ``C``. Large batches with k > 256 on a GPU run the fit's
    certified search (centred split-bf16 planes, 3-product pass + exact re-search of near-tie rows:
    the exact search's labels); otherwise the fp32 MFMA search. ``SRML_KMEANS_PREDICT_SPLIT=0``
    forces the latter."""
    k = C.shape[0]
    if (X.is_cuda and k > 256 and X.shape[0] >= 65536 and _use_split(X, k)
            and os.environ.get("SRML_KMEANS_PREDICT_SPLIT", "1") == "1"):
        mu = ops.col_moments(X, need_sq=False)[0].div_(X.shape[0]).float()
        if ops.kmeans_filter_mode() == "f16":
            F16 = ops.F16Planes(X, mu)
            if F16.ok:
                return ops.nearest_centroid_f16(F16, C.float())[0]
        XP = ops.split_bf16x3(X, tiled=True, mu=mu)
        labels, _ = ops.nearest_centroid_split(XP, X.shape[0], C.float(), ops.row_sqnorm(X, mu), X=X, mu=mu)
        return labels
    labels, _ = ops.nearest_centroid(X, C)
    return labels


def kmeans_predict_streamed(host: Any, C: torch.Tensor, device: torch.device,
                            chunk_bytes: int = 0) -> torch.Tensor:
    """``kmeans_predict`` of a page-locked host matrix with its H2D streamed under the search
    (reference transform: ``clustering.py:493-499``, one cuML predict per batch): the rows cross
    PCIe in ~256 MB chunks on the copy stream (``ops.ingest.StreamedRows``) while the certified
    fp16 filter labels the chunks already on the device, so the transform costs about its H2D
    (``ops.ingest.RingRows``: three chunk buffers reused, not a device copy of the whole batch).

    Each chunk is centred on the centres' mean (the filter's operands are x - mu and c - mu; any
    mu keeps the labels exact, it only conditions the fp16 plane) with its own plane scale. Chunks
    the fp16 filter cannot take (no finite range) use ``kmeans_predict``. ``host`` may be a
    multi-batch ``ChunkedRows`` (the transform's Arrow batches, streamed batch by batch)."""
    from ..ops.ingest import RingRows

    if chunk_bytes <= 0:
        chunk_bytes = int(os.environ.get("SRML_PREDICT_CHUNK_MB", "256")) << 20
    # a ring of three chunk buffers: ~0.75 GB of HBM whatever the batch size, no 12 GB allocation
    S = RingRows(host, device, torch.float32, chunk_bytes=chunk_bytes, depth=3)
    Cf = C.float().to(device)
    mu = Cf.mean(0)
    labels = torch.empty(host.shape[0], dtype=torch.int32, device=device)
    for r0, r1, Xc in S.chunks():
        F16 = ops.F16Planes(Xc, mu)
        if F16.ok:
            labels[r0:r1] = ops.nearest_centroid_f16(F16, Cf)[0]
        else:
            labels[r0:r1] = kmeans_predict(Xc, Cf).to(torch.int32)
    return labels


def predict_streams(host: Any, k: int) -> bool:
    """Whether ``kmeans_predict_streamed`` takes this host batch: page-locked, large, k > 256 and
    the fp16 certified filter (``SRML_KMEANS_PREDICT_STREAM=0`` disables)."""
    from ..ops.ingest import is_pinned

    return ((isinstance(host, np.ndarray) or hasattr(host, "parts")) and host.ndim == 2
            and host.shape[0] >= 65536 and k > 256 and host.dtype == np.float32 and torch.cuda.is_available()
            and os.environ.get("SRML_KMEANS_PREDICT_STREAM", "1") == "1"
            and os.environ.get("SRML_KMEANS_PREDICT_SPLIT", "1") == "1"
            and ops.kmeans_filter_mode() == "f16" and is_pinned(host))
