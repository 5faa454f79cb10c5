"""Distributed least squares: OLS, Ridge and ElasticNet/Lasso with Spark's objective.

Reference: cuML ``LinearRegressionMG`` (eig), ``RidgeMG`` (alpha x M) and ``CDMG``
(``regression.py:498-613``). Spark semantics (``WeightedLeastSquares`` / LBFGS-OWLQN objective)
are implemented exactly, in the standardised space:

    min_w~  1/2 w~' A~ w~ - b~' w~ + lam_eff [ a * sum p1_j |w~_j| + (1-a)/2 * sum p2_j w~_j^2 ]

with x~_j = x_j / sigma_j, y~ = y / sigma_y, A~ / b~ the (centred when fitIntercept) second
moments, lam_eff = regParam / sigma_y, p = 1 with standardization else 1/sigma_j (L1) and
1/sigma_j^2 (L2). Back-transform: w_j = w~_j sigma_y / sigma_j, b = ybar - xbar·w.

Device work per rank is two streaming passes over the resident shard — ``col_moments`` (sum,
sum of squares) and the fused-centring MFMA ``gram`` + ``xtv`` (X^T y) — and ONE coalesced
RCCL all-reduce of [X'X, X'y] (fp64). The n x n solve runs on the replicated statistics:
Cholesky for OLS/Ridge, cyclic coordinate descent on the Gram matrix ("covariance updates",
O(n^2) per epoch, independent of m) for ElasticNet/Lasso. All param maps of a fitMultiple
share the statistics (one pass over the data for every model).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict, List, Optional

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext


@dataclass
class LSQStats:
    m: int
    xbar: np.ndarray
    xstd: np.ndarray
    ybar: float
    ystd: float
    cov: np.ndarray  # centred scatter / m  (n x n)
    raw2: np.ndarray  # uncentred second moment / m
    xy_c: np.ndarray  # centred cross moment / m
    xy_raw: np.ndarray  # uncentred cross moment / m
    yy_raw: float


def lsq_stats(X: torch.Tensor, y: torch.Tensor, m_total: int, ctx: WorkerContext) -> LSQStats:
    n = X.shape[1]
    dev = X.device
    s, q = ops.col_moments(X)
    yd = y.double()
    ys = torch.stack([yd.sum(), (yd * yd).sum()])
    small = torch.cat([s, q, ys])
    ctx.comm.allreduce(small)
    s, q, ys = small[:n], small[n: 2 * n], small[2 * n:]
    mean = s / m_total
    G = ops.gram(X, mean)  # centred scatter (fp64)
    xty = ops.xtv(X, y.view(-1, 1)).view(-1)  # raw X'y (fp64)
    big = torch.cat([G.view(-1), xty])
    ctx.comm.allreduce(big)
    G = big[: n * n].view(n, n)
    xty = big[n * n:]
    meanh = mean.cpu().numpy()
    mt = float(m_total)
    var = np.maximum(q.cpu().numpy() / mt - meanh * meanh, 0.0)
    ybar = float(ys[0].item()) / mt
    yvar = max(float(ys[1].item()) / mt - ybar * ybar, 0.0)
    cov = G.cpu().numpy() / mt
    xy_raw = xty.cpu().numpy() / mt
    xy_c = xy_raw - meanh * ybar
    raw2 = cov + np.outer(meanh, meanh)
    return LSQStats(m_total, meanh, np.sqrt(var), ybar, float(np.sqrt(yvar)), cov, raw2, xy_c, xy_raw,
                    float(ys[1].item()) / mt)


def _cholesky_solve(A: np.ndarray, b: np.ndarray) -> np.ndarray:
    try:
        L = np.linalg.cholesky(A)
        z = np.linalg.solve(L, b)
        return np.linalg.solve(L.T, z)
    except np.linalg.LinAlgError:
        # singular normal equations: minimum-norm least-squares solution (eigen-solver fallback)
        w, V = np.linalg.eigh(A)
        tol = max(w.max(), 0.0) * A.shape[0] * np.finfo(np.float64).eps
        inv = np.where(w > tol, 1.0 / np.where(w > tol, w, 1.0), 0.0)
        return V @ (inv * (V.T @ b))


def coordinate_descent(A: np.ndarray, b: np.ndarray, l1: np.ndarray, l2: np.ndarray, max_iter: int, tol: float,
                       w0: Optional[np.ndarray] = None) -> np.ndarray:
    """min 1/2 w'Aw - b'w + sum l1_j |w_j| + 1/2 sum l2_j w_j^2  by cyclic CD on the Gram matrix."""
    n = A.shape[0]
    w = np.zeros(n) if w0 is None else w0.copy()
    grad = A @ w  # maintained A w
    diag = np.diag(A) + l2
    for _ in range(max(1, max_iter)):
        max_delta = 0.0
        max_w = 0.0
        for j in range(n):
            if diag[j] <= 0:
                continue
            rho = b[j] - grad[j] + A[j, j] * w[j]
            if rho > l1[j]:
                nw = (rho - l1[j]) / diag[j]
            elif rho < -l1[j]:
                nw = (rho + l1[j]) / diag[j]
            else:
                nw = 0.0
            d = nw - w[j]
            if d != 0.0:
                grad += d * A[:, j]
                w[j] = nw
                max_delta = max(max_delta, abs(d))
            max_w = max(max_w, abs(nw))
        if max_delta <= tol * max(max_w, 1e-300):
            break
    return w


def lsq_solve(st: LSQStats, reg: float, l1_ratio: float, fit_intercept: bool, standardization: bool,
              max_iter: int, tol: float) -> Dict[str, Any]:
    n = st.xbar.shape[0]
    xstd = st.xstd
    nz = xstd > 0
    safe = np.where(nz, xstd, 1.0)
    if st.ystd == 0.0 and fit_intercept:
        # constant label: Spark returns zero coefficients and intercept = label mean
        return {"coef_": [0.0] * n, "intercept_": st.ybar}
    ystd = st.ystd if st.ystd > 0 else 1.0
    if fit_intercept:
        A = st.cov / np.outer(safe, safe)
        b = st.xy_c / (safe * ystd)
    else:
        A = st.raw2 / np.outer(safe, safe)
        b = st.xy_raw / (safe * ystd)
    A[~nz, :] = 0.0
    A[:, ~nz] = 0.0
    b[~nz] = 0.0
    lam = reg / ystd
    l1 = lam * l1_ratio * (np.ones(n) if standardization else 1.0 / safe)
    l2 = lam * (1.0 - l1_ratio) * (np.ones(n) if standardization else 1.0 / (safe * safe))
    if reg == 0.0 or l1_ratio == 0.0:
        Areg = A + np.diag(l2)
        Areg[~nz, ~nz] = 1.0
        wt = _cholesky_solve(Areg, b)
    else:
        wt = coordinate_descent(A, b, l1, l2, max_iter, tol)
    wt[~nz] = 0.0
    w = wt * ystd / safe
    intercept = float(st.ybar - st.xbar @ w) if fit_intercept else 0.0
    return {"coef_": w.tolist(), "intercept_": intercept}


def linear_predict(X: torch.Tensor, coef: torch.Tensor, intercept: float) -> torch.Tensor:
    return ops.xw(X, coef.view(-1, 1)).view(-1) + intercept
