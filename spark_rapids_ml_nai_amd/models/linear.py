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
RCCL all-reduce of [X'X, X'y] (fp64). The n x n solve runs on the replicated statistics, on
the device: blocked Cholesky (``srml_potrf_f64``, MFMA trailing updates) for OLS/Ridge, with the
Jacobi eigensolver's minimum-norm solution for singular systems; cyclic coordinate descent on
the Gram matrix ("covariance updates", O(n^2) per epoch, independent of m, one kernel launch —
``srml_cd_gram_f64``) for ElasticNet/Lasso. All param maps of a fitMultiple share the
statistics (one pass over the data for every model).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Any, Dict

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext


@dataclass
class LSQStats:
    """Replicated second-order statistics (fp64 tensors on the rank's device)."""

    m: int
    xbar: torch.Tensor
    sumsq: torch.Tensor  # global column sums of squares
    scatter: torch.Tensor  # global centred scatter (n x n, NOT divided by m)
    xty: torch.Tensor  # global raw X^T y
    ybar: float
    ystd: float
    yy_raw: float

    @property
    def xstd(self) -> torch.Tensor:
        return (self.sumsq / float(self.m) - self.xbar * self.xbar).clamp_min(0.0).sqrt()

    @property
    def cov(self) -> torch.Tensor:
        """centred scatter / m"""
        return self.scatter / float(self.m)

    @property
    def xy_raw(self) -> torch.Tensor:
        """uncentred cross moment / m"""
        return self.xty.view(-1) / float(self.m)

    @property
    def xy_c(self) -> torch.Tensor:
        """centred cross moment / m"""
        return self.xy_raw - self.xbar * self.ybar

    @property
    def raw2(self) -> torch.Tensor:
        """uncentred second moment / m"""
        return self.cov + torch.outer(self.xbar, self.xbar)


def lsq_stats(X: torch.Tensor, y: torch.Tensor, m_total: int, ctx: WorkerContext, stream: Any = None) -> LSQStats:
    """One pass (overlapped with the H2D when ``stream`` is given) + two all-reduces."""
    from .stats import scatter_stats

    st = scatter_stats(X, ctx, m_total, stream=stream, y=y, need_sq=True)
    mt = float(m_total)
    ybar = st.y_sum / mt
    yvar = max(st.y_sumsq / mt - ybar * ybar, 0.0)
    return LSQStats(m_total, st.mean, st.sumsq, st.scatter, st.xty.view(-1), ybar, float(np.sqrt(yvar)),
                    st.y_sumsq / mt)


def _min_norm_prox(A: torch.Tensor, b: torch.Tensor, max_iter: int = 40, rtol: float = 1e-13) -> torch.Tensor:
    """Minimum-norm solution of singular PSD normal equations by the proximal-point (iterated
    Tikhonov) recursion x <- (A + d I)^-1 (b + d x) from x = 0: null-space components stay zero,
    an eigen-direction with eigenvalue l converges at rate d / (l + d). One Cholesky of A + d I
    (d = 1e-7 max diag A, well conditioned), then two triangular sweeps per step — the n > 4096
    counterpart of the eigen path (cuML's eigDC fallback, regression.py:508-560). The rounding
    component of b in the null space grows the iterate by ~eps |b| / d per step; the recursion
    stops when the step size stops shrinking geometrically (that drift dominates), so the result
    agrees with the eigen pseudo-inverse to ~1e-8 relative; eigenvalues below ~1e-5 max diag are
    only partly resolved (directions that ill-posed have no stable min-norm answer in fp64)."""
    n = A.shape[0]
    d = max(float(A.diagonal().max()), 1e-300) * 1e-7
    L, ok = ops.spd_factor(A + d * torch.eye(n, dtype=A.dtype, device=A.device))
    if not ok:
        return _min_norm_eig(A, b)
    x = ops.spd_factor_solve(L, b)
    prev = float("inf")
    for _ in range(max_iter):
        x1 = ops.spd_factor_solve(L, b + d * x)
        step = float(torch.linalg.vector_norm(x1 - x))
        x = x1
        if step <= rtol * float(torch.linalg.vector_norm(x1)) or step > 0.5 * prev:
            break
        prev = step
    return x


def _min_norm_solve(A: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """Singular normal equations: minimum-norm least-squares solution (device Jacobi eigensolver
    up to n = 4096, the proximal-point Cholesky recursion beyond)."""
    if A.is_cuda and A.shape[0] > 4096:
        return _min_norm_prox(A, b)
    return _min_norm_eig(A, b)


def _min_norm_eig(A: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    w, V = ops.syevj(A) if A.is_cuda and A.shape[0] <= 4096 else torch.linalg.eigh(A)
    tol = max(float(w.max()), 0.0) * A.shape[0] * float(np.finfo(np.float64).eps)
    inv = torch.where(w > tol, 1.0 / torch.where(w > tol, w, torch.ones_like(w)), torch.zeros_like(w))
    Vtb = ops.dgemm(V, b.view(-1, 1), ta=True).view(-1)
    return ops.dgemm(V, (inv * Vtb).view(-1, 1)).view(-1)


def lsq_solve(st: LSQStats, reg: float, l1_ratio: float, fit_intercept: bool, standardization: bool,
              max_iter: int, tol: float) -> Dict[str, Any]:
    n = st.xbar.shape[0]
    dev = st.xbar.device
    if st.ystd == 0.0 and fit_intercept:
        # constant label: Spark returns zero coefficients and intercept = label mean
        return {"coef_": [0.0] * n, "intercept_": st.ybar}
    ystd = st.ystd if st.ystd > 0 else 1.0
    # Penalties of the reference's solvers (regression.py:508-560: cuML RidgeMG with alpha * m, CD
    # with alpha / l1_ratio; i.e. sklearn Ridge / Lasso / ElasticNet): in raw units
    #   1/(2m) ||y - Xw - b||^2 + reg * (l1_ratio ||s w||_1 + (1 - l1_ratio)/2 ||s w||^2),
    # s = feature std (standardization) or 1. Solved here in standardised units (w_t = w s_x / ystd,
    # objective scaled by 1/ystd^2), which moves one 1/ystd onto the L1 weight and none onto L2.
    direct = reg == 0.0 or l1_ratio == 0.0
    if dev.type == "cuda":
        # one kernel forms the scaled system (+ diag(l2 + 1 - keep) for the direct solvers: constant
        # columns get identity rows and a zero rhs) and the per-feature vectors [safe|keep|b|l1|l2]
        A = torch.empty((n, n), dtype=torch.float64, device=dev)
        vec = torch.empty(5 * n, dtype=torch.float64, device=dev)
        ops.native.call("srml_lsq_prepare", st.scatter.data_ptr(), n, st.xbar.data_ptr(), st.sumsq.data_ptr(),
                        st.xty.data_ptr(), float(st.m), float(st.ybar), float(ystd), float(reg), float(l1_ratio),
                        int(fit_intercept), int(standardization), int(direct), A.data_ptr(), vec.data_ptr(),
                        ops.native.stream(dev))
        safe, keep, b, l1, l2 = vec.view(5, n)
        Areg = A
    else:
        xstd = st.xstd
        nz = xstd > 0
        safe = torch.where(nz, xstd, torch.ones_like(xstd))
        denom = torch.outer(safe, safe)
        A = (st.cov if fit_intercept else st.raw2) / denom
        b = (st.xy_c if fit_intercept else st.xy_raw) / (safe * ystd)
        keep = nz.double()
        A = A * torch.outer(keep, keep)
        b = b * keep
        lam = reg / ystd
        ones = torch.ones(n, dtype=torch.float64, device=dev)
        l1 = lam * l1_ratio * (ones if standardization else 1.0 / safe)
        l2 = reg * (1.0 - l1_ratio) * (ones if standardization else 1.0 / (safe * safe))
        Areg = A + torch.diag(l2 + (1.0 - keep)) if direct else A
    if direct:
        wt, ok = ops.spd_solve(Areg, b)
        if not ok:
            wt = _min_norm_solve(Areg, b)
    else:
        wt, _ = ops.cd_gram(A, b, l1, l2, max_iter, tol)
    if dev.type == "cuda":
        out = torch.empty(n + 1, dtype=torch.float64, device=dev)
        ops.native.call("srml_lsq_finish", ops._c(wt.double()).data_ptr(), n, vec.data_ptr(), st.xbar.data_ptr(),
                        float(ystd), float(st.ybar), int(fit_intercept), out.data_ptr(), ops.native.stream(dev))
        h = out.cpu().tolist()
        return {"coef_": h[:n], "intercept_": float(h[n])}
    wt = wt * keep
    w = wt * ystd / safe
    intercept = float(st.ybar - float((st.xbar * w).sum())) if fit_intercept else 0.0
    return {"coef_": w.cpu().tolist(), "intercept_": intercept}


def linear_predict(X: torch.Tensor, coef: torch.Tensor, intercept: float) -> torch.Tensor:
    return ops.xw(X, coef.view(-1, 1)).view(-1) + intercept
