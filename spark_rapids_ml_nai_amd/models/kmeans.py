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

from typing import Any, Dict, Optional

import numpy as np
import torch

from .. import ops
from ..parallel.context import PartitionDescriptor, WorkerContext


def _global_rows(X: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext, idx: np.ndarray) -> torch.Tensor:
    """Gather rows with the given global indices onto every rank (owner contributes, all-reduce)."""
    n = X.shape[1]
    start = sum(s for r, s in desc.parts_rank_size if r < desc.rank)
    stop = start + X.shape[0]
    out = torch.zeros((len(idx), n), dtype=torch.float64, device=X.device)
    mine = np.nonzero((idx >= start) & (idx < stop))[0]
    if len(mine):
        rows = torch.from_numpy(idx[mine] - start).to(X.device)
        out[torch.from_numpy(mine).to(X.device)] = X.index_select(0, rows).double()
    ctx.comm.allreduce(out)
    return out


def init_random(X: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext, k: int, seed: int) -> torch.Tensor:
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(desc.m, size=min(k, desc.m), replace=False))
    C = _global_rows(X, desc, ctx, idx)
    if C.shape[0] < k:  # fewer rows than clusters: duplicate
        C = C[torch.arange(k, device=C.device) % C.shape[0]]
    return C


def _weighted_kmeanspp(P: torch.Tensor, w: torch.Tensor, k: int, gen: torch.Generator) -> torch.Tensor:
    """Weighted k-means++ seeding of the (small) candidate set on the device."""
    npts = P.shape[0]
    Pf = P.float()
    first = int(torch.multinomial(w.float(), 1, generator=gen).item())
    centers = [first]
    d2 = ((Pf - Pf[first]) ** 2).sum(1)
    for _ in range(1, k):
        prob = (w * d2).double()
        tot = float(prob.sum().item())
        if tot <= 0:
            nxt = int(torch.randint(0, npts, (1,), generator=gen, device=P.device).item())
        else:
            nxt = int(torch.multinomial((prob / tot).float(), 1, generator=gen).item())
        centers.append(nxt)
        d2 = torch.minimum(d2, ((Pf - Pf[nxt]) ** 2).sum(1))
    return P[torch.tensor(centers, device=P.device)].clone()


def _weighted_lloyd(P: torch.Tensor, w: torch.Tensor, C: torch.Tensor, iters: int = 30) -> torch.Tensor:
    Pf = P.float().contiguous()
    pn = ops.row_sqnorm(Pf) if Pf.is_cuda else (Pf * Pf).sum(1)
    k = C.shape[0]
    for _ in range(iters):
        lab, _ = ops.nearest_centroid(Pf, C.float(), pn)
        lab = lab.long()
        sums = torch.zeros_like(C, dtype=torch.float64)
        sums.index_add_(0, lab, P.double() * w.double().view(-1, 1))
        cnt = torch.zeros(k, dtype=torch.float64, device=P.device).index_add_(0, lab, w.double())
        newC = torch.where(cnt.view(-1, 1) > 0, sums / cnt.clamp_min(1e-300).view(-1, 1), C.double())
        if torch.allclose(newC, C.double()):
            C = newC
            break
        C = newC
    return C


def init_kmeans_parallel(X: torch.Tensor, xnorm: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext,
                         k: int, seed: int, oversampling: float = 2.0, steps: int = 2) -> torch.Tensor:
    dev = X.device
    rng = np.random.default_rng(seed)
    C = _global_rows(X, desc, ctx, np.array([int(rng.integers(0, desc.m))]))
    gen = torch.Generator(device=dev)
    gen.manual_seed(int(seed) * 1000003 + ctx.rank)
    ell = oversampling * k
    for _ in range(max(1, steps)):
        _, d2 = ops.nearest_centroid(X, C.float(), xnorm)
        phi = d2.double().sum().view(1)
        ctx.comm.allreduce(phi)
        p = (ell * d2.double() / max(float(phi.item()), 1e-300)).clamp_max(1.0)
        pick = torch.rand(X.shape[0], generator=gen, device=dev, dtype=torch.float64) < p
        local = X[pick].double()
        parts = ctx.comm.allgatherv(local)
        C = torch.cat([C] + [q.to(dev) for q in parts], 0)
    # weight every candidate by the points it attracts
    lab, _ = ops.nearest_centroid(X, C.float(), xnorm)
    w = torch.bincount(lab.long(), minlength=C.shape[0]).double()
    ctx.comm.allreduce(w)
    if C.shape[0] <= k:
        extra = init_random(X, desc, ctx, k - C.shape[0], seed + 1) if C.shape[0] < k else None
        return torch.cat([C, extra], 0) if extra is not None else C
    # the candidate set is tiny (~ steps * oversampling * k points): run a few seeded k-means++
    # + weighted Lloyd trials on it and keep the lowest weighted cost (deterministic per seed)
    g2 = torch.Generator(device=dev)
    g2.manual_seed(int(seed))
    Cf = C.float().contiguous()
    cn = ops.row_sqnorm(Cf) if Cf.is_cuda else (Cf * Cf).sum(1)
    best, best_cost = None, float("inf")
    for _ in range(5):
        Ct = _weighted_lloyd(C, w, _weighted_kmeanspp(C, w, k, g2))
        _, d2 = ops.nearest_centroid(Cf, Ct.float(), cn)
        cost = float((d2.double() * w).sum().item())
        if cost < best_cost:
            best, best_cost = Ct, cost
    return best


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
    need = 3 * 2 * ((m + 127) // 128 * 128) * ((n + 15) // 16 * 16)
    free, _ = torch.cuda.mem_get_info(X.device)
    return need < 0.6 * free


def kmeans_fit(X: torch.Tensor, desc: PartitionDescriptor, ctx: WorkerContext, k: int, max_iter: int, tol: float,
               seed: int, init: str = "scalable-k-means++", oversampling: float = 2.0, init_steps: int = 2,
               timer: Any = None) -> Dict[str, Any]:
    n = X.shape[1]
    xnorm = ops.row_sqnorm(X)
    if init in ("random",):
        C = init_random(X, desc, ctx, k, seed)
    elif init in ("scalable-k-means++", "k-means||", "k-means++"):
        C = init_kmeans_parallel(X, xnorm, desc, ctx, k, seed, oversampling, init_steps)
    else:
        raise ValueError("Unsupported init mode %s" % init)
    C = C.double()
    tol2 = float(tol) ** 2
    # k > 256: 256 x 256 LDS-DMA kernel on the tiled plane layout (SRML_SPLIT_TILED=0: plain layout)
    tiled = k > 256 and os.environ.get("SRML_SPLIT_TILED", "1") == "1"
    XP = ops.split_bf16x3(X, tiled=tiled) if _use_split(X, k) else None
    n_iter = 0
    inertia = 0.0
    for it in range(max(0, max_iter)):
        n_iter = it + 1
        if XP is not None:
            labels, d2 = ops.nearest_centroid_split(XP, X.shape[0], C.float(), xnorm)
        else:
            labels, d2 = ops.nearest_centroid(X, C.float(), xnorm)
        sums, counts = ops.cluster_sums(X, labels, k)
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
    del XP
    return {
        "cluster_centers_": C.cpu().numpy(),  # ndarray: 3M-float .tolist() cost 40 ms per fit
        "n_cols": int(n),
        "dtype": "float32" if X.dtype == torch.float32 else "float64",
        "n_iter": n_iter,
    }


def kmeans_predict(X: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    labels, _ = ops.nearest_centroid(X, C)
    return labels
