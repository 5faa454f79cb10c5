"""Distributed logistic regression (binomial + multinomial, L2 / L1 / elastic-net) with Spark's
objective.

Reference: cuML ``LogisticRegressionMG`` (QN: L-BFGS / OWL-QN, ``lbfgs_memory=10``,
``penalty_normalized=False``) driven from ``classification.py:957-1151``, with standardisation
done by the reference in cupy and the moments exchanged as JSON through the Spark driver.

MI355X design:
* every objective/gradient evaluation is ONE fused pass over the resident shard: binary
  ``srml_logreg_binary2_f32`` (margin, softplus loss, residual and X^T r from registers),
  multinomial ``srml_mlogit_f32`` (K margins, softmax, K gradient rows from one read of each row),
  CSR kernels for sparse input, an LDS-accumulating pass for fp64 / wide rows; then ONE RCCL
  all-reduce of [grad (K n), grad_b (K), loss] in fp64;
* the quasi-Newton iteration (L-BFGS memory 10; OWL-QN for L1 / elastic-net) runs ON THE DEVICE
  (``models/qn.py`` + ``ops/csrc/qn.hip``): no host round trip per evaluation; all ranks advance
  identical optimiser states from the identical all-reduced sums;
* standardisation never rewrites X: it is folded into the coefficients (z = X (w~/sigma) + b)
  and the chain rule, with the column moments from one ``col_moments`` pass + all-reduce.

Objective (Spark): 1/m sum_i loss_i + reg * [ (1-a)/2 sum_j q2_j w_j^2 + a sum_j q1_j |w_j| ]
with q = sigma (standardization=True) or 1, intercepts unpenalised.
"""
from __future__ import annotations

import os

from typing import Any, Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext
from .qn import QNProblem, minimize


def _problem(n: int, m_total: int, stats: Dict[str, Any], reg: float, l1_ratio: float, fit_intercept: bool,
             standardization: bool, max_iter: int, tol: float, K: int) -> Tuple[QNProblem, np.ndarray, np.ndarray]:
    """Spark's objective as a QN problem on the sigma-scaled coefficients: (problem, theta0,
    inv_sigma)."""
    sigma = stats["sigma"]
    inv_sigma = np.where(sigma > 0, 1.0 / np.where(sigma > 0, sigma, 1.0), 0.0)
    q1 = sigma if standardization else np.ones(n)
    q2 = sigma * sigma if standardization else np.ones(n)
    # penalties act on scaled coefficients w~ = w * sigma
    pen_l2 = reg * (1.0 - l1_ratio) * np.where(sigma > 0, q2 / np.where(sigma > 0, sigma * sigma, 1.0), 0.0)
    pen_l1 = reg * l1_ratio * np.where(sigma > 0, q1 / np.where(sigma > 0, sigma, 1.0), 0.0)
    nb = K if fit_intercept else 0
    theta0 = np.zeros(K * n + nb)
    if fit_intercept:
        counts = stats["class_counts"]
        if K == 1:
            p1 = counts[1] / max(counts.sum(), 1.0) if len(counts) > 1 else 0.5
            p1 = min(max(p1, 1e-12), 1 - 1e-12)
            theta0[K * n] = np.log(p1 / (1 - p1))
        else:
            lc = np.log(np.maximum(counts[:K], 1.0))
            theta0[K * n:] = lc - lc.mean()
    P = QNProblem(n=n, K=K, fit_intercept=fit_intercept, m_total=float(m_total),
                  l2=np.concatenate([np.tile(pen_l2, K), np.zeros(nb)]),
                  l1=np.concatenate([np.tile(pen_l1 if l1_ratio > 0 and reg > 0 else np.zeros(n), K), np.zeros(nb)]),
                  inv_sigma=inv_sigma, max_iter=max(0, int(max_iter)), tol=float(tol), M=10)
    return P, theta0, inv_sigma


def _result(res: Dict[str, Any], base: Dict[str, Any], ctx: WorkerContext, n: int, K: int, fit_intercept: bool,
            inv_sigma: np.ndarray, path: str) -> Dict[str, Any]:
    theta = res["theta"]
    if ctx.world_size > 1:  # every rank holds the same state; make the model bit-identical anyway
        th = torch.from_numpy(theta).to(ctx.device)
        ctx.comm.broadcast(th, 0)
        theta = th.cpu().numpy()
    W = theta[: K * n].reshape(K, n) * inv_sigma
    b = theta[K * n:] if fit_intercept else np.zeros(K)
    if fit_intercept and K > 1:
        b = b - b.mean()  # Spark centres multinomial intercepts
    out = dict(base)
    out.update(coef_=W.tolist(), intercept_=[float(v) for v in b], num_iters=int(res["iter"]),
               objective=float(res["f"]))
    out["_solver"] = {"n_evals": int(res["n_evals"]), "status": res["status"], "path": path}
    if res.get("n_margin_only"):  # evaluations that read the cached margins instead of X
        out["_solver"]["n_margin_only"] = int(res["n_margin_only"])
    return out


def _one_class(classes: list, base: Dict[str, Any], n: int) -> Dict[str, Any]:
    cv = classes[0]
    if cv not in (0.0, 1.0):
        raise RuntimeError("class value must be either 1. or 0. when dataset has one label")
    out = dict(base)
    out.update(coef_=[[0.0] * n], intercept_=[float("inf") if cv == 1.0 else float("-inf")], num_iters=0,
               objective=0.0)
    return out


def logistic_fit(X: Any, y: torch.Tensor, m_total: int, ctx: WorkerContext, reg: float, l1_ratio: float,
                 fit_intercept: bool, standardization: bool, max_iter: int, tol: float,
                 n_classes: Optional[int] = None, sparse: bool = False,
                 stats: Optional[Dict[str, Any]] = None) -> Dict[str, Any]:
    n = X.shape[1]
    if stats is None:
        stats = logistic_stats(X, y, m_total, ctx, sparse)
    classes = stats["classes"]
    C = n_classes if n_classes is not None else stats["num_classes"]
    K = 1 if C <= 2 else C
    dtype = "float32" if (X.dtype if not sparse else X.data.dtype) == torch.float32 else "float64"
    base = {"classes_": [float(c) for c in classes], "n_cols": int(n), "dtype": dtype}
    # one-class edge case (Spark: +-inf intercept, zero coefficients)
    if len(classes) == 1 and fit_intercept:
        return _one_class(classes, base, n)
    P, theta0, inv_sigma = _problem(n, m_total, stats, reg, l1_ratio, fit_intercept, standardization, max_iter, tol, K)
    y32 = y if y.dtype == torch.float32 else y.to(torch.float32)
    y32 = y32.contiguous()

    ws = ops.logreg_workspace(X) if not sparse and K == 1 else None  # this fit's own partial rows

    def evaluate(w: torch.Tensor, b: torch.Tensor, flag: Optional[torch.Tensor], out: torch.Tensor,
                 zc: Optional[tuple] = None) -> None:
        ops.logistic_loss_grad(X, y32, w, b, K, out, flag, ws=ws, zcache=zc)

    allreduce = ctx.comm.allreduce if ctx.distributed else None
    path = ops.logistic_path(X, K)
    fold = evaluate_partials = None
    if ws is not None and allreduce is None and path == "fused_binary_f32":
        # one rank: the evaluation leaves its per-block partial rows and the fused optimiser step
        # folds them (one launch per evaluation instead of three)
        parts, wst = ops.logreg_fold_layout(X)
        fold = (ws, parts, wst)
        _scratch = ops.zeros(K * n + 2, dtype=torch.float64, device=X.device)

        def evaluate_partials(w: torch.Tensor, b: torch.Tensor, flag: Optional[torch.Tensor],
                              zc: Optional[tuple] = None) -> None:
            ops.logistic_loss_grad(X, y32, w, b, K, _scratch, flag, ws=ws, leave_partials=True, zcache=zc)
    # stream-ordered device evaluations (no host sync; allocations come from the graph's pool) may
    # be replayed from a HIP graph — when launches are what the batch costs: a graph is captured
    # and instantiated per fit (5.4 ms at the 125k x 3000 shard), while an evaluation reading more
    # than GRAPH_MAX_BYTES of X runs far longer than its five launches take to issue
    graph_safe = (path in ("fused_binary_f32", "fused_multinomial_f32", "csr_binary", "two_pass_multinomial_f32",
                           "two_pass_binary_f32") or path.startswith("lds_binary")) and _eval_bytes(X) <= GRAPH_MAX_BYTES
    # line-search margin cache: binary fits on the narrow / prefetching kernels. Every rank's optimiser
    # must run the same state machine, so the ranks agree (a rank without rows has nothing to cache)
    zok = ((path == "fused_binary_f32" and (X.shape[0] == 0 or ops.logreg_zcache_ok(X)))
           or (path == "two_pass_multinomial_f32" and ops.XW_MFMA_MIN_K <= K <= 16))
    if allreduce is not None:
        flag_t = torch.tensor([1.0 if zok else 0.0], dtype=torch.float64, device=X.device)
        ctx.comm.allreduce(flag_t, op="min")
        zok = bool(flag_t.item() > 0)
    zbuf = ops.zeros(2 * X.shape[0] * K, dtype=torch.float64, device=X.device) if zok else None
    res = minimize(P, theta0, evaluate, allreduce, y.device, batch=8 if not path.startswith("torch") else 2,
                   graph_safe=graph_safe, fold=fold, evaluate_partials=evaluate_partials, zcache=zbuf)
    return _result(res, base, ctx, n, K, fit_intercept, inv_sigma, path)


GRAPH_MAX_BYTES = int(os.environ.get("SRML_QN_GRAPH_MAX_MB", "64")) << 20


def _eval_bytes(X: Any) -> int:
    """Bytes of X one loss/gradient evaluation streams (dense values, or CSR values + indices)."""
    if hasattr(X, "data") and hasattr(X, "indices") and not isinstance(X, torch.Tensor):
        return int(X.data.numel() * X.data.element_size() + X.indices.numel() * X.indices.element_size())
    return int(X.numel() * X.element_size())


MAX_BATCH = 12  # models per fused multi-model pass (register-resident weights, like the multinomial pass)


def logistic_fit_multi(X: Any, y: torch.Tensor, m_total: int, ctx: WorkerContext, settings: List[Dict[str, Any]],
                       sparse: bool = False, stats: Optional[Dict[str, Any]] = None) -> List[Dict[str, Any]]:
    """fitMultiple for LogisticRegression (SURVEY §2.6 hyper-parameter batching): binary problems
    on the device run in batches of <= 12 that share every pass over X (margins of all models in
    one skinny-GEMM pass, residuals, one X^T R pass: ``ops.logistic_loss_grad_multi``) and one
    batched optimiser launch per evaluation (``minimize_batch``); anything else (multinomial,
    sparse, fp64, CPU, a single setting) fits one setting at a time. ``settings`` entries:
    reg, l1_ratio, fit_intercept, standardization, max_iter, tol."""
    n = X.shape[1]
    if stats is None:
        stats = logistic_stats(X, y, m_total, ctx, sparse)
    K = 1 if stats["num_classes"] <= 2 else stats["num_classes"]
    if sparse or K != 1 or len(settings) < 2 or not ops.mbin_supported(X, min(len(settings), MAX_BATCH)):
        return [logistic_fit(X, y, m_total, ctx, s["reg"], s["l1_ratio"], s["fit_intercept"], s["standardization"],
                             s["max_iter"], s["tol"], sparse=sparse, stats=stats) for s in settings]
    from .qn import minimize_batch

    classes = stats["classes"]
    base = {"classes_": [float(c) for c in classes], "n_cols": int(n), "dtype": "float32"}
    y32 = (y if y.dtype == torch.float32 else y.to(torch.float32)).contiguous()
    allreduce = ctx.comm.allreduce if ctx.distributed else None
    out: List[Optional[Dict[str, Any]]] = [None] * len(settings)
    todo = []
    for i, s in enumerate(settings):
        if len(classes) == 1 and s["fit_intercept"]:
            out[i] = _one_class(classes, base, n)
        else:
            todo.append(i)
    for g0 in range(0, len(todo), MAX_BATCH):
        grp = todo[g0: g0 + MAX_BATCH]
        probs = [_problem(n, m_total, stats, settings[i]["reg"], settings[i]["l1_ratio"], settings[i]["fit_intercept"],
                          settings[i]["standardization"], settings[i]["max_iter"], settings[i]["tol"], 1) for i in grp]

        def evaluate(WB: torch.Tensor, OUT: torch.Tensor) -> None:
            ops.logistic_loss_grad_multi(X, y32, WB, OUT)

        res = minimize_batch([p[0] for p in probs], [p[1] for p in probs], evaluate, allreduce, y.device)
        for i, (P, _, inv_sigma), r in zip(grp, probs, res):
            out[i] = _result(r, base, ctx, n, 1, P.fit_intercept, inv_sigma, "batched_binary_f32")
    return [o for o in out if o is not None]


def logistic_stats(X: Any, y: torch.Tensor, m_total: int, ctx: WorkerContext, sparse: bool) -> Dict[str, Any]:
    """Column std-devs (population, Spark's featuresStd) and label histogram, all-reduced once."""
    n = X.shape[1]
    if sparse:
        s, q = ops.csr_col_moments(X)
    else:
        s, q = ops.col_moments(X)
    yl = y.long()
    if torch.any(y < 0) or torch.any(y != torch.floor(y)):
        bad = y[(y < 0) | (y != torch.floor(y))][0].item()
        if bad < 0:
            raise RuntimeError(f"Labels MUST be in [0, 2147483647), but got {bad}")
        raise RuntimeError(f"Labels MUST be Integers, but got {bad}")
    mx = torch.tensor([float(yl.max().item()) if yl.numel() else 0.0], dtype=torch.float64, device=y.device)
    ctx.comm.allreduce(mx, op="max")
    ncls = int(mx.item()) + 1
    hist = ops.label_counts(yl, ncls).double()
    buf = torch.cat([s, q, hist])
    ctx.comm.allreduce(buf)
    s, q, hist = buf[:n], buf[n: 2 * n], buf[2 * n:]
    mean = (s / m_total).cpu().numpy()
    var = np.maximum((q / m_total).cpu().numpy() - mean * mean, 0.0)
    # Spark uses the unbiased std for featuresStd
    var = var * m_total / max(m_total - 1, 1)
    counts = hist.cpu().numpy()
    classes = [float(c) for c in np.nonzero(counts > 0)[0]]
    return {"sigma": np.sqrt(var), "mean": mean, "class_counts": counts, "classes": classes,
            "num_classes": max(2, ncls)}


def logistic_scores(X: torch.Tensor, coef: torch.Tensor, intercept: torch.Tensor) -> torch.Tensor:
    """Margins (rows, K): one pass of the skinny xw kernel with the bias epilogue."""
    return ops.xw(X, coef.T.contiguous(), intercept)
