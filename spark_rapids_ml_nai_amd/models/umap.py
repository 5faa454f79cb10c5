"""UMAP on MI355X: kNN graph -> fuzzy simplicial set -> spectral/random init -> SGD layout.

Semantics follow umap-learn / cuML UMAP (what the reference calls on one GPU, ``umap.py:924-958``):
* kNN graph: exact, from the fused MFMA distance + top-k kernel (``ops.knn``), self included;
* ``smooth_knn_dist`` (per-row bisection for sigma, rho = nearest non-zero distance with
  ``local_connectivity``) and the membership strengths exp(-(d - rho) / sigma) fused in one
  thread-per-row kernel (``ops.umap_smooth_knn``); torch reference on CPU;
* fuzzy union A + Aᵀ - A∘Aᵀ (``set_op_mix_ratio`` blends with the intersection): one thread per
  kNN edge finds the reverse edge in the neighbour's row and emits each union entry exactly
  once (``ops.umap_fuzzy_union_knn``), then one device sort of the edge keys;
* optional supervised intersection with a categorical target (far_dist 5, unknown 1) followed
  by ``reset_local_connectivity``;
* spectral init on the device for every n: top eigenvectors of D^-1/2 A D^-1/2 by the dense
  parallel-Jacobi kernel (n <= 2048) or block subspace iteration with the CSR SpMM kernel and
  split-K fp64 GEMMs (larger n); host ``eigsh`` only on CPU; scaled like umap-learn;
* SGD: ``srml_umap_epoch`` (edge-parallel HIP kernel, hash RNG negative sampling), alpha decays
  linearly, edges below max_w / n_epochs dropped, epochs_per_sample = n_epochs / (n_epochs·w/max_w);
* transform: kNN to the training data, local_connectivity - 1, l1-normalised weighted init
  from neighbour embeddings, n_epochs/3 (default 100 / 30) epochs at alpha/4 with the training
  embedding fixed.
"""
from __future__ import annotations

import math
import os
from typing import Any, Dict, Optional, Tuple

import numpy as np
import torch

from .. import ops

SMOOTH_K_TOLERANCE = 1e-5
MIN_K_DIST_SCALE = 1e-3
# IVF-built graphs stay in inverted-list order through the fuzzy set, spectral init and epochs
# (neighbour gathers become mostly local); the embedding is scattered back to row order at the end
LIST_ORDER = os.environ.get("SRML_UMAP_LIST_ORDER", "1") != "0"
# fit epochs on the symmetric fuzzy graph move heads only (ops.umap_epoch pull=True): each pair's
# two directed edges apply its attraction to both ends, without scattered tail atomics
PULL = os.environ.get("SRML_UMAP_PULL", "1") != "0"
# pull epochs draw negatives from a per-epoch randomly ordered snapshot, 8 edges per 64 B line
# (ops.umap_epoch neg_table): one memory request per 8 negative samples instead of 8
NEG_LINES = os.environ.get("SRML_UMAP_NEG_LINES", "1") != "0"
# Chebyshev filter degree of the device spectral init's subspace iteration (1 = plain iteration).
# Degree 4 at the 1e-6 Ritz stop: 20M blobs 97 -> 29 products, 20M classification rows 232 -> 58
# (fit 9.95 -> 6.32 s), trustworthiness unchanged (profiles/umap_spectral_cheb_r5.jsonl). Round 4's
# degree 8 at a stop near fp32 resolution ran to the product cap on the clustered 20M graph; the
# stop is now above fp32 noise and a stagnating Ritz change also ends the iteration.
CHEB_DEGREE = int(os.environ.get("SRML_UMAP_CHEB_DEGREE", "4"))
# Ritz-value stop of the spectral init (see _spectral_device): umap-learn's eigsh tolerance. At 20M
# rows 1e-4 / 1e-5 / 1e-6 take 34 / 42 / 46 products (1.00 / 1.21 / 1.32 s) for trustworthiness
# 0.7095 / 0.7092 / 0.7102 (profiles/northstar_r6_umap_spectral_tol*.jsonl)
SPECTRAL_TOL = float(os.environ.get("SRML_UMAP_SPECTRAL_TOL", "1e-4"))
SPECTRAL_DENSE_N = 2048  # device Jacobi on the dense normalised adjacency up to this many vertices
# per-phase {"rows": this rank's rows / edges, "s": seconds} of the last umap_fit in this process
LAST_PHASES: Dict[str, Any] = {}


def find_ab_params(spread: float, min_dist: float) -> Tuple[float, float]:
    """Fit 1 / (1 + a x^(2b)) to the target membership curve (umap-learn ``find_ab_params``)."""
    from scipy.optimize import curve_fit

    def curve(x: Any, a: float, b: float) -> Any:
        return 1.0 / (1.0 + a * x ** (2 * b))

    xv = np.linspace(0, spread * 3, 300)
    yv = np.zeros(xv.shape)
    yv[xv < min_dist] = 1.0
    yv[xv >= min_dist] = np.exp(-(xv[xv >= min_dist] - min_dist) / spread)
    params, _ = curve_fit(curve, xv, yv)
    return float(params[0]), float(params[1])


def knn_graph(Q: torch.Tensor, I: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(euclidean distances [mq, k] fp32, indices [mq, k] int64)."""
    inorm = ops.row_sqnorm(I)
    d2, idx = ops.knn(Q, I, k, inorm=inorm)
    # refine the selected distances directly to avoid expansion cancellation
    r = ops.knn_refine_sort(Q, I, idx)  # fused device kernel (k <= 64, fp32)
    if r is not None:
        return torch.sqrt(r[0].clamp_min(0)), r[1]
    step = max(1, (1 << 26) // max(1, k * Q.shape[1]))
    out = torch.empty_like(d2)
    for s in range(0, Q.shape[0], step):
        rows = I.index_select(0, idx[s: s + step].reshape(-1)).view(-1, idx.shape[1], Q.shape[1])
        out[s: s + step] = ((rows - Q[s: s + step].unsqueeze(1)) ** 2).sum(-1)
    d2, j = torch.sort(out, dim=1)
    idx = idx.gather(1, j)
    return torch.sqrt(d2.clamp_min(0)), idx


def smooth_knn_dist(dist: torch.Tensor, k: float, n_iter: int = 64, local_connectivity: float = 1.0,
                    bandwidth: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Vectorised umap-learn ``smooth_knn_dist``: (sigmas, rhos) for every row."""
    d = dist.double()
    m, kk = d.shape
    target = math.log2(k) * bandwidth
    nz = torch.where(d > 0, d, torch.full_like(d, float("inf")))
    nz_sorted, _ = torch.sort(nz, dim=1)
    n_nz = (d > 0).sum(1)
    index = int(math.floor(local_connectivity))
    interp = local_connectivity - index
    rho = ops.zeros(m, dtype=torch.float64, device=d.device)
    ok = n_nz >= local_connectivity
    if index > 0:
        base = nz_sorted[:, index - 1]
        rho_i = base.clone()
        if interp > 1e-5 and index < kk:
            rho_i = base + interp * (nz_sorted[:, index] - base)
        rho = torch.where(ok, rho_i, rho)
    else:
        rho = torch.where(ok, interp * nz_sorted[:, 0], rho)
    anyz = n_nz > 0
    rho = torch.where(~ok & anyz, nz_sorted.masked_fill(~torch.isfinite(nz_sorted), -1).max(1).values, rho)
    rho = torch.where(torch.isfinite(rho), rho, torch.zeros_like(rho))
    lo = ops.zeros(m, dtype=torch.float64, device=d.device)
    hi = torch.full((m,), float("inf"), dtype=torch.float64, device=d.device)
    mid = torch.ones(m, dtype=torch.float64, device=d.device)
    done = ops.zeros(m, dtype=torch.bool, device=d.device)
    dd = d[:, 1:] - rho.view(-1, 1)
    for _ in range(n_iter):
        psum = torch.where(dd > 0, torch.exp(-dd / mid.view(-1, 1)), torch.ones_like(dd)).sum(1)
        done = done | ((psum - target).abs() < SMOOTH_K_TOLERANCE)
        gt = psum > target
        new_hi = torch.where(gt, mid, hi)
        new_lo = torch.where(gt, lo, mid)
        new_mid = torch.where(gt, (lo + mid) / 2.0,
                              torch.where(torch.isinf(hi), mid * 2.0, (mid + hi) / 2.0))
        lo = torch.where(done, lo, new_lo)
        hi = torch.where(done, hi, new_hi)
        mid = torch.where(done, mid, new_mid)
        if bool(done.all()):
            break
    mean_row = d.mean(1)
    mean_all = d.mean()
    sigma = torch.where(rho > 0, torch.maximum(mid, MIN_K_DIST_SCALE * mean_row),
                        torch.maximum(mid, MIN_K_DIST_SCALE * mean_all))
    return sigma, rho


def membership_strengths(idx: torch.Tensor, dist: torch.Tensor, sigma: torch.Tensor, rho: torch.Tensor,
                         self_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    d = dist.double() - rho.view(-1, 1)
    w = torch.where(d <= 0, torch.ones_like(d), torch.exp(-d / sigma.view(-1, 1)))
    w = torch.where(sigma.view(-1, 1) == 0, torch.ones_like(w), w)
    if self_rows is not None:
        w = torch.where(idx == self_rows.view(-1, 1), torch.zeros_like(w), w)
    w = torch.where(idx < 0, torch.zeros_like(w), w)
    return w.float()


def _coalesce(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n: int) -> Tuple[Any, Any, Any, int]:
    key = rows.long() * n + cols.long()
    uk, inv = torch.unique(key, return_inverse=True)
    return uk // n, uk % n, inv, uk.numel()


def fuzzy_union(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n: int,
                set_op_mix_ratio: float = 1.0) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """P = mix·(A + Aᵀ - A∘Aᵀ) + (1 - mix)·(A∘Aᵀ) for an n x n COO matrix without duplicates."""
    keep = vals > 0
    rows, cols, vals = rows[keep], cols[keep], vals[keep]
    r2 = torch.cat([rows, cols])
    c2 = torch.cat([cols, rows])
    v2 = torch.cat([vals, vals]).double()
    ur, uc, inv, nu = _coalesce(r2, c2, v2, n)
    s = ops.zeros(nu, dtype=torch.float64, device=vals.device).index_add_(0, inv, v2)
    cnt = ops.zeros(nu, dtype=torch.int64, device=vals.device).index_add_(0, inv, torch.ones_like(inv))
    lp = ops.zeros(nu, dtype=torch.float64, device=vals.device).index_add_(0, inv, torch.log(v2))
    prod = torch.where(cnt >= 2, torch.exp(lp), torch.zeros_like(lp))
    out = set_op_mix_ratio * (s - prod) + (1.0 - set_op_mix_ratio) * prod
    keep = out > 0
    return ur[keep], uc[keep], out[keep].float()


def categorical_intersection(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, y: torch.Tensor,
                             n: int, unknown_dist: float = 1.0, far_dist: float = 5.0
                             ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    if vals.is_cuda:
        # the device union is (row, col)-sorted with a symmetric pattern: native kernel, same edges
        r64 = rows.long()
        if r64.numel() < 2 or bool((r64[1:] >= r64[:-1]).all()):
            out = ops.umap_categorical(r64, cols.long(), vals, y, n, unknown_dist, far_dist)
            keep = out > 0
            return r64[keep], cols.long()[keep], out[keep]
    yr, yc = y[rows], y[cols]
    unknown = (yr == -1) | (yc == -1)
    differ = (yr != yc) & ~unknown
    v = vals.double()
    v = torch.where(unknown, v * math.exp(-unknown_dist), v)
    v = torch.where(differ, v * math.exp(-far_dist), v)
    # reset_local_connectivity: normalise rows by their max, then fuzzy union again
    rmax = ops.zeros(n, dtype=torch.float64, device=v.device).scatter_reduce_(0, rows.long(), v, "amax",
                                                                               include_self=True)
    v = v / rmax[rows.long()].clamp_min(1e-30)
    return fuzzy_union(rows, cols, v.float(), n)


def _spectral_host(rows: np.ndarray, cols: np.ndarray, vals: np.ndarray, n: int, dim: int, seed: int) -> np.ndarray:
    import scipy.sparse as sp
    from scipy.sparse.linalg import eigsh

    A = sp.coo_matrix((vals.astype(np.float64), (rows, cols)), shape=(n, n)).tocsr()
    deg = np.asarray(A.sum(axis=1)).ravel()
    dinv = 1.0 / np.sqrt(np.maximum(deg, 1e-30))
    D = sp.diags(dinv)
    L = sp.identity(n) - D @ A @ D
    k = dim + 1
    if n <= 2000 or n < 4 * k:
        w, v = np.linalg.eigh(L.toarray())
    else:
        num_lanczos = max(2 * k + 1, int(np.sqrt(n)))
        rng = np.random.default_rng(seed)
        w, v = eigsh(L, k, which="SM", ncv=num_lanczos, tol=1e-4, v0=np.ones(n) + 0.01 * rng.standard_normal(n),
                     maxiter=n * 5)
    order = np.argsort(w)[1:k]
    return v[:, order]


def _allreduce(t: torch.Tensor, ctx: Any) -> torch.Tensor:
    if ctx is not None and ctx.world_size > 1:
        ctx.comm.allreduce(t)
    return t


def _cholqr2(Y: torch.Tensor, ctx: Any = None) -> torch.Tensor:
    """Orthonormal basis of a tall-skinny device block: two CholeskyQR passes (fp64 Gram on the
    device, p x p Cholesky on the host); Householder QR only if the Gram is numerically singular.
    Distributed (``ctx``): Y is this rank's row block; the p x p Grams are all-reduced (every rank
    applies the same R^-1 to its rows)."""
    W = Y
    dist = ctx is not None and ctx.world_size > 1
    for _ in range(2):
        Wd = W.double()
        # Gram of a tall-skinny block: the streaming SYRK kernel (fp32 in, fp64 out); a library
        # fp64 GEMM with K = n rows picks a non-split-K tile and took 53 ms at 2M x 11
        Gt = ops.gram(W.float()) if (W.is_cuda and W.shape[0]) else Wd.T @ Wd
        G = _allreduce(Gt.contiguous(), ctx).cpu().numpy()
        try:
            L = np.linalg.cholesky((G + G.T) * 0.5)
        except np.linalg.LinAlgError:
            L = None
        d = np.diag(L) if L is not None else None
        if L is None or d.min() <= 1e-6 * d.max():
            if dist:  # a singular block shared by the ranks: orthonormalise the gathered block
                from .knn_graph import gather_rows, row_split

                full = torch.linalg.qr(gather_rows(Y.contiguous(), ctx))[0]
                lo, hi = row_split(full.shape[0], ctx)
                return full[lo:hi].contiguous()
            return torch.linalg.qr(Y)[0]
        Rinv = torch.from_numpy(np.linalg.solve(L, np.eye(L.shape[0])).T.copy()).to(Y.device)
        W = ops.dgemm(Wd, Rinv).to(Y.dtype)
    return W


def _spectral_device(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n: int, dim: int, seed: int,
                     iters: int = 300, tol: float = 1e-6, min_iters: int = 20, ctx: Any = None,
                     phases: Optional[dict] = None) -> torch.Tensor:
    """Top eigenvectors of D^-1/2 A D^-1/2 by subspace iteration: the SpMM is the in-tree CSR
    kernel (``ops.csr_spmm``, one row group per graph row), orthonormalisation is CholeskyQR2.
    The (row, col)-sorted union edges ARE the CSR (no sparse-tensor coalesce); the iteration
    stops once the Ritz values of the leading dim + 1 directions move by <= ``tol`` (checked at
    every re-orthonormalisation, from the product the next step needs anyway) — umap-learn's
    eigsh runs at tol 1e-4 and the layout only needs a starting point. The Ritz values come from
    fp32 products, so a tolerance near fp32 resolution (1e-8 before) made the stop a coin toss:
    164 products in one 20M fit and the 300 cap in the next.

    Distributed (``ctx``, graph replicated): rank r owns a contiguous row block of the operator
    and of the subspace block. Every product all-gathers the n x p block (the SpMM gathers
    arbitrary neighbour rows), multiplies the rank's rows only, and the p x p Ritz / Gram
    matrices are all-reduced: the SpMM, Gram and GEMM work divides by W, the subspace stays
    bit-identical across ranks."""
    from ..core.base import CSR
    from .knn_graph import gather_rows, record_phase, row_split

    import time

    t0 = time.perf_counter()
    dev = vals.device
    r64 = rows.long()
    if r64.numel() > 1 and not bool((r64[1:] >= r64[:-1]).all()):
        # (row, col) order: the in-tree LSD radix sort of the packed keys carries the values
        keys = (r64 * n + cols.long()).contiguous()
        vals = vals.float().contiguous().clone()
        ops.radix_sort_pairs(keys, vals, max(1, int(n * n).bit_length()))
        r64, cols = keys // n, keys % n
    # rows are sorted: the CSR row pointer is a binary search per row boundary (no atomics), and
    # the degrees are the row sums of the same CSR (one pass of the SpMM kernel against a ones
    # column; an fp64 index_add over the ~15 n edges cost 0.3 s of atomics at n = 20M)
    indptr = torch.searchsorted(r64.contiguous(), torch.arange(n + 1, device=dev, dtype=torch.int64))
    lo, hi = row_split(n, ctx)
    e0, e1 = int(indptr[lo]), int(indptr[hi])
    ip_l = (indptr[lo: hi + 1] - e0).contiguous()
    ci = cols[e0:e1].to(torch.int32).contiguous()
    vl = vals[e0:e1]
    rl = r64[e0:e1]
    A = CSR(indptr=ip_l, indices=ci, data=vl.float().contiguous(), shape=(hi - lo, n))
    deg = gather_rows(ops.csr_row_sums(A), ctx)  # fp64 per-row accumulation, this rank's rows
    dinv = 1.0 / torch.sqrt(deg.clamp_min(1e-30))
    mv = (dinv[rl] * vl.double() * dinv[ci.long()]).float().contiguous()
    M = CSR(indptr=ip_l, indices=ci, data=mv, shape=(hi - lo, n))
    # block size: dim + 1 wanted vectors + 8 guards, rounded up to the SpMM kernel's 16 columns
    # (64 B W rows: one memory line per gathered neighbour, and a faster-converging subspace)
    p = min(n, 16 if dim + 9 <= 16 else dim + 9)
    # device RNG: a host randn of 20M x 16 plus its copy took 0.9 s of the 20M fit; every rank
    # draws the whole block (same seed) and keeps its rows
    g = torch.Generator(device=dev).manual_seed(int(seed))
    Y = torch.randn((n, p), generator=g, device=dev)
    Y[:, 0] = torch.sqrt(deg).float()
    Y = Y[lo:hi].contiguous()
    Y = _cholqr2(Y, ctx)

    def amul(V: torch.Tensor) -> torch.Tensor:
        Vf = gather_rows(V.contiguous(), ctx)
        return 0.5 * (ops.csr_spmm(M, Vf) + V)  # (M + I) / 2: eigenvalues in [0, 1], order kept

    def ritz_matrix(Yb: torch.Tensor, Zb: torch.Tensor) -> np.ndarray:
        T = ops.dgemm(Yb.double().contiguous(), Zb.double().contiguous(), ta=True)
        return _allreduce(T.contiguous(), ctx).cpu().numpy()

    prev = None
    it = 0
    best = float("inf")
    stall = 0
    if CHEB_DEGREE > 1:
        # Chebyshev-filtered subspace iteration: each step applies T_d on [0, b] (b = the block's
        # smallest Ritz value, an upper bound of the unwanted spectrum), which damps the unwanted
        # directions like ~exp(-d sqrt(2 gap)) instead of (1 - gap)^d for d plain products
        while it < iters:
            Z = amul(Y)
            it += 1
            T = ritz_matrix(Y, Z)
            allr = np.sort(np.linalg.eigvalsh((T + T.T) * 0.5))[::-1]
            ritz = allr[: dim + 1]
            if prev is not None:
                rel = float(np.max(np.abs(ritz - prev))) / max(float(np.max(np.abs(ritz))), 1e-30)
                # a change that stops shrinking for 4 checks near the tolerance is fp32 noise
                stall = stall + 1 if rel >= 0.5 * best and rel <= 20.0 * tol else 0
                best = min(best, rel)
                if it >= min_iters and (rel <= tol or stall >= 4):
                    break
            prev = ritz
            bcut = float(min(max(allr[-1], 0.0), allr[dim]))
            if bcut >= 0.995 or it + CHEB_DEGREE > iters:
                Y = _cholqr2(Z, ctx)  # spectrum too clustered for the filter: a plain step
                continue
            e, c = 0.5 * bcut, 0.5 * bcut
            Y0, Y1 = Y, (Z - c * Y) / e
            for _ in range(CHEB_DEGREE - 1):
                Y0, Y1 = Y1, 2.0 * (amul(Y1) - c * Y1) / e - Y0
                it += 1
            Y = _cholqr2(Y1, ctx)
    while CHEB_DEGREE <= 1 and it < iters:
        Z = amul(Y)
        it += 1
        if it % 5 == 1:  # Y is orthonormal here: Ritz values of the current subspace
            T = ritz_matrix(Y, Z)
            ritz = np.sort(np.linalg.eigvalsh((T + T.T) * 0.5))[::-1][: dim + 1]
            if prev is not None and it >= min_iters and \
                    np.max(np.abs(ritz - prev)) <= tol * max(float(np.max(np.abs(ritz))), 1e-30):
                Y = Z
                break
            prev = ritz
        Y = Z
        if it % 5 == 0:
            Y = _cholqr2(Y, ctx)
    Y = _cholqr2(Y, ctx)
    Z = amul(Y)
    # Y^T Z: K = n rows in the millions -> the split-K fp64 MFMA GEMM (ordered fold)
    Yd = Y.double().contiguous()
    w, V = np.linalg.eigh(ritz_matrix(Y, Z))
    order = np.argsort(w)[::-1][1: dim + 1].copy()
    out = gather_rows(ops.dgemm(Yd, torch.from_numpy(np.ascontiguousarray(V[:, order])).to(dev)).float().contiguous(),
                      ctx)
    record_phase(phases, "spectral", hi - lo, t0, dev)
    if phases is not None:
        phases["spectral"]["products"] = it + 1
    return out


def _spectral_dense_device(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n: int, dim: int) -> torch.Tensor:
    """Small graphs on the device: dense D^-1/2 A D^-1/2 and all its eigenpairs by the parallel
    Jacobi kernel (``ops.syevj``); the top non-trivial eigenvectors of M are the smallest
    non-trivial ones of the normalised Laplacian (umap-learn's spectral_layout)."""
    dev = vals.device
    deg = ops.zeros(n, dtype=torch.float64, device=dev).index_add_(0, rows.long(), vals.double())
    dinv = 1.0 / torch.sqrt(deg.clamp_min(1e-30))
    M = ops.zeros((n, n), dtype=torch.float64, device=dev)
    M.index_put_((rows.long(), cols.long()), dinv[rows.long()] * vals.double() * dinv[cols.long()], accumulate=True)
    M = 0.5 * (M + M.T)
    w, V = ops.syevj(M)  # descending
    return V[:, 1: dim + 1].float().contiguous()


def spectral_init(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, n: int, dim: int, seed: int,
                  ctx: Any = None, phases: Optional[dict] = None) -> torch.Tensor:
    """Spectral layout (identical on every rank of a distributed fit: the large-graph subspace
    iteration runs row-partitioned over the ranks, the small cases are computed redundantly)."""
    dev = vals.device
    dist = ctx is not None and ctx.world_size > 1
    if n > SPECTRAL_DENSE_N and (dev.type == "cuda" or dist):
        coords = _spectral_device(rows, cols, vals, n, dim, seed, tol=SPECTRAL_TOL, ctx=ctx, phases=phases)
    elif dev.type != "cuda":
        coords = torch.from_numpy(_spectral_host(rows.cpu().numpy(), cols.cpu().numpy(), vals.cpu().numpy(), n, dim,
                                                 seed)).float().to(dev)
    else:
        coords = _spectral_dense_device(rows, cols, vals, n, dim)
    expansion = 10.0 / coords.abs().max().clamp_min(1e-30)
    g = torch.Generator(device=dev).manual_seed(int(seed) + 1)
    return coords * expansion + torch.randn(coords.shape, generator=g, device=dev) * 1e-4


def make_epochs_per_sample(w: torch.Tensor, n_epochs: int) -> torch.Tensor:
    n_samples = n_epochs * (w / w.max())
    return torch.where(n_samples > 0, float(n_epochs) / n_samples.clamp_min(1e-30), torch.full_like(w, -1.0))


def optimize_layout(emb_head: torch.Tensor, emb_tail: torch.Tensor, head: torch.Tensor, tail: torch.Tensor,
                    w: torch.Tensor, n_epochs: int, a: float, b: float, gamma: float, initial_alpha: float,
                    negative_sample_rate: float, move_other: bool, seed: int, ctx: Any = None,
                    pull: bool = False, phases: Optional[dict] = None) -> torch.Tensor:
    """SGD epochs over the fuzzy-graph edges.

    Distributed (``ctx.world_size > 1``, identical graph and layout on every rank): rank r
    keeps the edges e with e % world == r, runs its epoch on its replica of the layout and the
    replicas are re-synchronised by ONE all-reduce of the layout deltas per epoch (N x dim fp32;
    160 MB at the 20M-row north-star — a few hundred microseconds over the xGMI mesh). The
    summed deltas are the union of every rank's Hogwild updates, as on one device.
    """
    w = torch.where(w < w.max() / float(n_epochs), torch.zeros_like(w), w)
    keep = w > 0
    head, tail, w = head[keep], tail[keep], w[keep]
    eps = make_epochs_per_sample(w, n_epochs).float()  # normalised by the GLOBAL max weight
    world = ctx.world_size if ctx is not None else 1
    if world > 1:
        shard = slice(ctx.rank, None, world)
        head, tail, eps = head[shard], tail[shard], eps[shard]
        seed = (int(seed) + 0x9E3779B1 * ctx.rank) & 0x7FFFFFFF
    head, tail, eps = head.int().contiguous(), tail.int().contiguous(), eps.contiguous()
    if phases is not None:
        phases["epochs"] = {"rows": int(head.shape[0])}  # this rank's edges
    eps_neg = (eps / float(negative_sample_rate)).contiguous()
    next_sample = eps.clone()
    next_neg = eps_neg.clone()
    same = emb_head.data_ptr() == emb_tail.data_ptr()
    neg = None
    nt = emb_tail.shape[0]
    if NEG_LINES and pull and same and emb_tail.is_cuda and nt >= 4096 and emb_tail.shape[1] <= 4:
        # negatives from a per-epoch snapshot in a random vertex order, 8 edges per 64 B line
        g = torch.Generator(device=emb_tail.device).manual_seed(int(seed) + 7)
        ids = torch.randperm(nt, generator=g, device=emb_tail.device)[: (nt // 8) * 8].int().contiguous()
        neg = (torch.empty((ids.shape[0], emb_tail.shape[1]), dtype=torch.float32, device=emb_tail.device), ids)
    for n in range(n_epochs):
        alpha = initial_alpha * (1.0 - float(n) / float(n_epochs))
        before = (emb_head.clone(), None if same or not move_other else emb_tail.clone()) if world > 1 else None
        if neg is not None:
            ops.umap_neg_table(emb_tail, neg[1], neg[0])
        ops.umap_epoch(head, tail, eps, next_sample, next_neg, eps_neg, emb_head, emb_tail, a, b, gamma, alpha, n,
                       move_other, seed, pull=pull, neg_table=neg)
        if before is not None:
            for cur, old in ((emb_head, before[0]), (emb_tail, before[1])):
                if old is None:
                    continue
                cur.sub_(old)
                ctx.comm.allreduce(cur)
                cur.add_(old)
    return emb_head


def _n_epochs_default(n: int) -> int:
    return 500 if n <= 10000 else 200


def umap_fit(X: torch.Tensor, params: Dict[str, Any], y: Optional[torch.Tensor] = None, ctx: Any = None) -> np.ndarray:
    """Embedding (N x n_components, float32) of the rows of X.

    ``ctx`` with ``world_size > 1`` (X replicated on every rank): every phase shards over the
    ranks — the IVF quantiser's Lloyd iterations (1/W of the training sample each, sums
    all-reduced), the bucketing (1/W of the rows each, labels all-gathered), the kNN lists (a
    work-balanced range of query tiles, rows all-gathered), the spectral subspace iteration
    (row-partitioned SpMM, all-gathered block per product, all-reduced p x p Grams) and the SGD
    epochs (edge-parallel, one RCCL all-reduce of the layout deltas per epoch,
    ``optimize_layout``); only the fuzzy union (kNN-structured, ~0.06 s at 20M) is computed on
    every rank. ``LAST_PHASES`` holds this rank's per-phase rows and seconds of the last fit.
    """
    import time

    phases: Dict[str, Any] = {}
    LAST_PHASES.clear()
    t_ph = time.perf_counter()
    N = X.shape[0]
    k = int(min(params.get("n_neighbors", 15), N))
    dim = int(params.get("n_components", 2))
    metric = params.get("metric", "euclidean")
    seed = params.get("random_state")
    seed = int(seed) if seed is not None else int(np.random.randint(0, 2 ** 31 - 1))
    dist_ctx = ctx if (ctx is not None and ctx.world_size > 1) else None
    if dist_ctx is not None:
        seed = int(dist_ctx.comm.broadcast_object(seed, 0))
    a, b = params.get("a"), params.get("b")
    if a is None or b is None:
        a, b = find_ab_params(float(params.get("spread", 1.0)), float(params.get("min_dist", 0.1)))
    Xf = X.float().contiguous()
    if metric in ("cosine", "correlation"):
        if metric == "correlation":
            Xf = Xf - Xf.mean(1, keepdim=True)
        Xf = Xf / Xf.norm(dim=1, keepdim=True).clamp_min(1e-30)
    elif metric not in ("euclidean", "l2", "sqeuclidean"):
        raise ValueError("Unsupported UMAP metric %r" % metric)
    pre = params.get("precomputed_knn")
    order = None  # graph row i is original row order[i] (IVF list order), None: original order
    if pre is not None:
        idx = torch.as_tensor(np.asarray(pre[0]), dtype=torch.int64, device=X.device)[:, :k]
        dist = torch.as_tensor(np.asarray(pre[1]), dtype=torch.float32, device=X.device)[:, :k]
    else:
        from .knn_graph import build_knn_graph

        g = build_knn_graph(Xf, k, params.get("build_algo", "auto"), params.get("build_kwds"), seed, ctx,
                            list_order=LIST_ORDER, phases=phases)
        dist, idx, order = g if LIST_ORDER else (g[0], g[1], None)
        t_ph = time.perf_counter()  # the graph's phases are logged inside (synchronised)
        if metric in ("cosine", "correlation"):
            dist = 0.5 * dist * dist  # 1 - cos for unit rows
        elif metric == "sqeuclidean":
            dist = dist * dist
    lc = float(params.get("local_connectivity", 1.0))
    mix = float(params.get("set_op_mix_ratio", 1.0))
    if X.is_cuda:  # fused kernels: smooth_knn_dist + membership, then the kNN-structured union
        _, _, w = ops.umap_smooth_knn(dist, idx, float(k), local_connectivity=lc, self_rows=True)
        rows, cols, vals = ops.umap_fuzzy_union_knn(idx, w, mix)
    else:
        sigma, rho = smooth_knn_dist(dist, float(k), local_connectivity=lc)
        self_rows = torch.arange(N, device=X.device)
        w = membership_strengths(idx, dist, sigma, rho, self_rows)
        rows = self_rows.view(-1, 1).expand_as(idx).reshape(-1)
        cols = idx.reshape(-1)
        rows, cols, vals = fuzzy_union(rows, cols.clamp_min(0), w.reshape(-1), N, mix)
    if y is not None:
        yy = y.to(X.device).long().view(-1)
        if order is not None:
            yy = yy[order]
        rows, cols, vals = categorical_intersection(rows, cols, vals, yy, N)
    n_epochs = params.get("n_epochs")
    n_epochs = int(n_epochs) if n_epochs else _n_epochs_default(N)
    init = params.get("init", "spectral")
    from .knn_graph import record_phase

    record_phase(phases, "fuzzy_union", N, t_ph, X.device)
    # every rank computes the same initial layout (the spectral iteration row-partitioned)
    if isinstance(init, str) and init == "spectral" and N > dim + 1:
        emb = spectral_init(rows, cols, vals, N, dim, seed, ctx=dist_ctx, phases=phases)
    else:
        g = torch.Generator(device=X.device).manual_seed(seed)
        emb = torch.rand((N, dim), generator=g, device=X.device) * 20.0 - 10.0
    mn, mx = emb.min(0).values, emb.max(0).values
    emb = (10.0 * (emb - mn) / (mx - mn).clamp_min(1e-30)).float().contiguous()
    if dist_ctx is not None and dist_ctx.world_size > 1:
        # the ranks' layouts agree by construction (identical collectives); one N x dim broadcast
        # makes rank 0's layout THE layout whatever a rank-local rounding did
        dist_ctx.comm.broadcast(emb, src=0)
    t_ep = time.perf_counter()
    optimize_layout(emb, emb, rows, cols, vals, n_epochs, a, b, float(params.get("repulsion_strength", 1.0)),
                    float(params.get("learning_rate", 1.0)), float(params.get("negative_sample_rate", 5)), True, seed,
                    ctx=dist_ctx, pull=PULL, phases=phases)
    record_phase(phases, "epochs", phases.get("epochs", {}).get("rows", 0), t_ep, X.device)
    LAST_PHASES.update(phases)
    if order is not None:
        out = torch.empty_like(emb)
        out[order] = emb
        emb = out
    return emb.cpu().numpy()


def umap_transform(X: torch.Tensor, raw: torch.Tensor, embedding: torch.Tensor, params: Dict[str, Any]) -> np.ndarray:
    Nn = X.shape[0]
    Ntr = raw.shape[0]
    k = int(min(params.get("n_neighbors", 15), Ntr))
    metric = params.get("metric", "euclidean")
    seed = params.get("random_state")
    seed = int(seed) if seed is not None else 42
    a, b = params.get("a"), params.get("b")
    if a is None or b is None:
        a, b = find_ab_params(float(params.get("spread", 1.0)), float(params.get("min_dist", 0.1)))
    Xf, Rf = X.float().contiguous(), raw.float().contiguous()
    if metric in ("cosine", "correlation"):
        if metric == "correlation":
            Xf, Rf = Xf - Xf.mean(1, keepdim=True), Rf - Rf.mean(1, keepdim=True)
        Xf = Xf / Xf.norm(dim=1, keepdim=True).clamp_min(1e-30)
        Rf = Rf / Rf.norm(dim=1, keepdim=True).clamp_min(1e-30)
    dist, idx = knn_graph(Xf, Rf, k)
    if metric in ("cosine", "correlation"):
        dist = 0.5 * dist * dist
    elif metric == "sqeuclidean":
        dist = dist * dist
    adj_lc = max(0.0, float(params.get("local_connectivity", 1.0)) - 1.0)
    if X.is_cuda:
        _, _, w = ops.umap_smooth_knn(dist, idx, float(k), local_connectivity=adj_lc, self_rows=False)
    else:
        sigma, rho = smooth_knn_dist(dist, float(k), local_connectivity=adj_lc)
        w = membership_strengths(idx, dist, sigma, rho)
    wn = w / w.sum(1, keepdim=True).clamp_min(1e-30)
    emb_tr = embedding.float().contiguous()
    init = (wn.unsqueeze(-1) * emb_tr[idx.clamp_min(0)]).sum(1).contiguous()
    n_epochs = params.get("n_epochs")
    n_epochs = int(n_epochs) // 3 if n_epochs else (100 if Nn <= 10000 else 30)
    if n_epochs <= 0:
        return init.cpu().numpy()
    rows = torch.arange(Nn, device=X.device).view(-1, 1).expand_as(idx).reshape(-1)
    cols = idx.reshape(-1).clamp_min(0)
    vals = w.reshape(-1)
    emb = optimize_layout(init, emb_tr.clone(), rows, cols, vals, n_epochs, a, b,
                          float(params.get("repulsion_strength", 1.0)), float(params.get("learning_rate", 1.0)) / 4.0,
                          float(params.get("negative_sample_rate", 5)), False, seed)
    return emb.cpu().numpy()
