"""Quasi-Newton minimiser (L-BFGS, OWL-QN for L1 terms) for the GLM solvers, with its state on the
device.

Reference: cuML's QN solver (``LogisticRegressionMG``, ``lbfgs_memory=10``) called from
``python/src/spark_rapids_ml/classification.py:1051-1065``; it iterates on the host with a device
round trip per evaluation. Here (``ops/csrc/qn.hip``) one single-block kernel advances the
optimiser after every summed loss/gradient evaluation, so a fit is a host-free stream of

    eval(w, b) -> out    [fused pass over the resident shard]
    allreduce(out)       [RCCL, world > 1]
    qn_step(out)         [line search / history / direction / next trial point]

and the host only polls the ``done`` flag every ``batch`` evaluations (asynchronously: the flag of
batch j is read while batch j + 1 is already queued). Evaluations early-exit once ``done`` is set.

Problem form (optimiser coordinates theta; ``inv_sigma`` maps them to the model space):

    f(theta) = loss_sum(W, b) / m + 1/2 sum l2_i theta_i^2 + sum l1_i |theta_i|
    W[k, j] = theta[k*n + j] * inv_sigma[j],   b[k] = theta[K*n + k]   (if fit_intercept)

``HostQN`` is the same state machine in numpy (CPU path and the oracle of the kernel tests).
Convergence follows cuML's QN (the reference backend): max|pg| <= tol * max(|f|, tol), or
|f_{k-10} - f_k| <= delta * max(|f|, tol) with delta = 0.01 tol, or k >= max_iter, or a failed line
search (the last accepted point is returned).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Callable, List, Optional

import numpy as np
import torch

from .. import ops

QN_GRAPH = os.environ.get("SRML_QN_GRAPH", "1") != "0"
# multi-rank fits: capture the batch INCLUDING its all-reduces (RCCL collectives recorded into the
# HIP graph, replayed identically on every rank); SRML_QN_GRAPH_COMM=0 keeps them eager
QN_GRAPH_COMM = os.environ.get("SRML_QN_GRAPH_COMM", "1") != "0"
# the optimiser step for N <= 16384: "mb" (default) = four multi-block launches (srml_qn_step_mb;
# a one-rank binary LogReg fit folds the evaluation's partial rows in the first: srml_qn_step_mbf);
# "fused" = ONE launch with software grid barriers (srml_qn_step_fused, folds likewise);
# "single" = the one-block kernel
QN_STEP = os.environ.get("SRML_QN_STEP", "mb")
QN_MB = QN_STEP in ("fused", "mb")
GRAPH_STATS = {"captures": 0, "replays": 0}  # observability / tests
STATUS = {0: "running", 1: "converged (gradient)", 2: "converged (objective change)", 3: "max iterations",
          4: "line search failed", 5: "barrier timeout"}
F_DONE, F_STATUS, F_ITER, F_NEVAL, F_LS, F_COUNT, F_HEAD, F_STARTED, F_BRACKET, F_ZMODE, F_ZSEL, F_NCHEAP, F_ZC = \
    range(13)
SC_F, SC_ALPHA, SC_DGINIT, SC_GAMMA, SC_GINF, SC_ALPHA1, SC_BETA = range(7)
# line-search margin cache (binary LogisticRegression on the multi-block step, Armijo, no L1): a
# rejected trial's margins make the rest of its backtracking margins-only evaluations (qn.hip F_ZMODE)
QN_ZCACHE = os.environ.get("SRML_QN_ZCACHE", "1") != "0"


@dataclass
class QNProblem:
    n: int
    K: int
    fit_intercept: bool
    m_total: float
    l2: np.ndarray  # [N] penalty coefficients on theta (0 for intercepts)
    l1: np.ndarray  # [N]
    inv_sigma: np.ndarray  # [n]
    max_iter: int
    tol: float
    M: int = 10
    max_ls: int = 20
    past: int = 10
    c1: float = 1e-4
    c2: float = 0.9
    wolfe: bool = False  # cuML's default line search is backtracking Armijo (LBFGS_LS_BT_ARMIJO)
    delta: Optional[float] = None

    @property
    def Kn(self) -> int:
        return self.K * self.n

    @property
    def N(self) -> int:
        return self.Kn + (self.K if self.fit_intercept else 0)

    @property
    def use_l1(self) -> bool:
        return bool(np.any(self.l1 > 0))

    @property
    def delta_(self) -> float:
        return 0.01 * self.tol if self.delta is None else float(self.delta)

    @property
    def out_len(self) -> int:
        return self.Kn + self.K + 1


def _interp_width(f0: float, ft: float, dgtest: float) -> float:
    """Backtracking factor from the minimiser of the quadratic through phi(0) = f0,
    phi'(0) alpha = dgtest (< 0) and phi(alpha) = ft, safeguarded to [0.1, 0.5] (Nocedal & Wright
    §3.5). Halving alone spent ~14 evaluations on the over-long second L-BFGS step."""
    den = 2.0 * (ft - f0 - dgtest)
    w = -dgtest / den if den > 0 else 0.5
    if not np.isfinite(w):
        return 0.5
    return float(min(0.5, max(0.1, w)))


# ------------------------------------------------------------------------------------------
class HostQN:
    """numpy reference of the device state machine (identical decisions; dense two-loop-free
    compact-form direction computed directly from the stored pairs)."""

    def __init__(self, P: QNProblem, theta0: np.ndarray) -> None:
        self.P = P
        N = P.N
        self.x = np.zeros(N)
        self.g = np.zeros(N)
        self.pg = np.zeros(N)
        self.d = np.zeros(N)
        self.xt = np.asarray(theta0, dtype=np.float64).copy()
        self.S: list = []
        self.Y: list = []
        self.f = 0.0
        self.alpha = 0.0
        self.dginit = 0.0
        self.gamma = 1.0
        self.iter = 0
        self.n_evals = 0
        self.ls = 0
        self.bracket = False
        self.started = False
        self.done = False
        self.status = 0
        self.fh = np.zeros(max(P.past, 1))
        self._isg_full = np.tile(P.inv_sigma, P.K)

    def wb(self) -> np.ndarray:
        """Evaluation parameters [W (K*n, class-major) | b (K)] in the model space."""
        P = self.P
        out = np.zeros(P.Kn + P.K)
        out[: P.Kn] = self.xt[: P.Kn] * self._isg_full
        if P.fit_intercept:
            out[P.Kn:] = self.xt[P.Kn:]
        return out

    @staticmethod
    def _pseudo(x: np.ndarray, g: np.ndarray, c: np.ndarray) -> np.ndarray:
        pg = g.copy()
        pos, neg, zero = x > 0, x < 0, x == 0
        pg[pos] += c[pos]
        pg[neg] -= c[neg]
        gp, gm = g + c, g - c
        z = zero & (c > 0)
        pz = np.where(gp < 0, gp, np.where(gm > 0, gm, 0.0))
        pg[z] = pz[z]
        return pg

    def _set_trial(self) -> None:
        P = self.P
        t = self.x + self.alpha * self.d
        if P.use_l1:
            orth = np.where(self.x != 0, np.sign(self.x), -np.sign(self.pg))
            mask = (P.l1 > 0) & (t * orth <= 0)
            t[mask] = 0.0
        self.xt = t

    def step(self, out: np.ndarray) -> None:
        P = self.P
        if self.done:
            return
        out = np.asarray(out, dtype=np.float64)
        Kn, N = P.Kn, P.N
        xt = self.xt
        gt = np.empty(N)
        gt[:Kn] = out[:Kn] / P.m_total * self._isg_full + P.l2[:Kn] * xt[:Kn]
        gt[Kn:] = out[Kn:N] / P.m_total
        ft = out[Kn + P.K] / P.m_total + 0.5 * float(np.sum(P.l2 * xt * xt)) + float(np.sum(P.l1 * np.abs(xt)))
        self.n_evals += 1
        if self.started:
            accept, width = True, 1.0
            if not np.isfinite(ft):
                accept, width = False, 0.5
            else:
                dgtest = float(self.pg @ (xt - self.x)) if P.use_l1 else self.alpha * self.dginit
                if ft > self.f + P.c1 * dgtest:
                    accept, width = False, _interp_width(self.f, ft, dgtest)
                elif P.wolfe and not P.use_l1 and not self.bracket and float(gt @ self.d) < P.c2 * self.dginit:
                    accept, width = False, 2.1
            if not accept:
                self.ls += 1
                if self.ls >= P.max_ls:
                    self.status, self.done = 4, True
                    return
                if width < 1.0:
                    self.bracket = True
                self.alpha *= width
                self._set_trial()
                return
        pg = self._pseudo(xt, gt, P.l1 if P.use_l1 else np.zeros(N))
        if self.started:
            s, y = xt - self.x, gt - self.g
            ys, yy = float(s @ y), float(y @ y)
            if yy > 0 and ys > 1e-10 * yy:
                self.S.append(s)
                self.Y.append(y)
                if len(self.S) > P.M:
                    self.S.pop(0)
                    self.Y.pop(0)
                self.gamma = ys / yy
            self.iter += 1
        self.x, self.g, self.f, self.pg = xt.copy(), gt, ft, pg
        self.ls, self.bracket = 0, False
        status = 0
        fmag = max(abs(ft), P.tol)
        if np.max(np.abs(pg)) <= P.tol * fmag if N else True:
            status = 1
        if P.past > 0:
            k = self.iter
            if status == 0 and self.started and k >= P.past and abs(self.fh[k % P.past] - ft) <= P.delta_ * fmag:
                status = 2
            self.fh[k % P.past] = ft
        if status == 0 and self.iter >= P.max_iter:
            status = 3
        self.started = True
        if status:
            self.status, self.done = status, True
            return
        d = -self._h_times(pg)
        if P.use_l1:
            d[(P.l1 > 0) & (d * pg >= 0)] = 0.0
        dg = float(pg @ d)
        if not dg < 0:
            d = -pg
            dg = -float(pg @ pg)
            self.S, self.Y, self.gamma = [], [], 1.0
        self.d = d
        self.dginit = dg
        self.alpha = 1.0 / max(np.sqrt(float(d @ d)), 1e-300) if not self.S else 1.0
        self._set_trial()

    def _h_times(self, v: np.ndarray) -> np.ndarray:
        """Compact L-BFGS inverse-Hessian product (Byrd, Nocedal, Schnabel 1994)."""
        if not self.S:
            return v.copy()
        S = np.stack(self.S)
        Y = np.stack(self.Y)
        g = self.gamma
        SY = S @ Y.T
        R = np.triu(SY)
        Dg = np.diag(np.diag(SY))
        p1, p2 = S @ v, Y @ v
        from scipy.linalg import solve_triangular

        t = solve_triangular(R, p1, lower=False)
        a = solve_triangular(R.T, (Dg + g * (Y @ Y.T)) @ t - g * p2, lower=True)
        return g * v + S.T @ a - g * (Y.T @ t)

    def theta(self) -> np.ndarray:
        return self.x.copy()


# ------------------------------------------------------------------------------------------
class _QnArgs(ctypes.Structure):
    _fields_ = [("N", ctypes.c_long), ("Kn", ctypes.c_long), ("n", ctypes.c_int), ("K", ctypes.c_int),
                ("M", ctypes.c_int), ("past", ctypes.c_int), ("max_iter", ctypes.c_int), ("max_ls", ctypes.c_int),
                ("l1", ctypes.c_int), ("wolfe", ctypes.c_int), ("tol", ctypes.c_double), ("delta", ctypes.c_double),
                ("inv_m", ctypes.c_double), ("c1", ctypes.c_double), ("c2", ctypes.c_double)] + \
               [(nm, ctypes.c_void_p) for nm in ("x", "g", "pg", "d", "xt", "gt", "S", "Y", "SY", "YY", "fh", "sc",
                                                 "l2", "l1c", "isg", "fl", "wb", "out", "probe")]


class DeviceQN:
    """Optimiser state in device memory, advanced by ``srml_qn_step`` (one launch per evaluation)."""

    def __init__(self, P: QNProblem, theta0: np.ndarray, device: torch.device, wb: Optional[torch.Tensor] = None,
                 out: Optional[torch.Tensor] = None, flags: Optional[torch.Tensor] = None) -> None:
        """``wb`` / ``out`` / ``flags``: optional preallocated (contiguous) views, so a batch of
        problems shares one trial-point matrix, one result matrix and one flag block."""
        from ..ops import native

        self.P = P
        self.device = device
        N, M = P.N, P.M
        if M > int(native.lib().srml_qn_max_history()):
            raise ValueError("L-BFGS memory %d exceeds the kernel's capacity" % M)
        f64 = dict(dtype=torch.float64, device=device)
        self.vec = ops.zeros((6 + 2 * M) * N, **f64)  # x g pg d xt gt S Y
        v = self.vec
        self.x, self.g, self.pg, self.d, self.xt, self.gt = (v[i * N:(i + 1) * N] for i in range(6))
        self.S = v[6 * N: (6 + M) * N]
        self.Y = v[(6 + M) * N:]
        self.small = ops.zeros(2 * M * M + max(P.past, 1) + 8, **f64)  # SY YY fh sc
        self.coef = torch.from_numpy(np.concatenate([P.l2, P.l1, P.inv_sigma]).astype(np.float64)).to(device)
        self.flags = flags if flags is not None else ops.zeros(16, dtype=torch.int32, device=device)
        self.wb = wb if wb is not None else ops.zeros(P.Kn + P.K, **f64)
        self.out = out if out is not None else ops.zeros(P.out_len, **f64)
        assert self.wb.numel() == P.Kn + P.K and self.out.numel() == P.out_len and self.flags.numel() == 16
        th = torch.from_numpy(np.asarray(theta0, dtype=np.float64)).to(device)
        self.xt.copy_(th)
        isg = torch.from_numpy(np.tile(P.inv_sigma, P.K)).to(device)
        self.wb[: P.Kn] = th[: P.Kn] * isg
        if P.fit_intercept:
            self.wb[P.Kn:] = th[P.Kn:]
        a = _QnArgs()
        a.N, a.Kn, a.n, a.K, a.M, a.past = N, P.Kn, P.n, P.K, M, P.past
        a.max_iter, a.max_ls, a.l1, a.wolfe = int(P.max_iter), int(P.max_ls), int(P.use_l1), int(P.wolfe)
        a.tol, a.delta, a.inv_m, a.c1, a.c2 = float(P.tol), P.delta_, 1.0 / float(P.m_total), P.c1, P.c2
        sm = self.small
        MM = M * M
        ptrs = dict(x=self.x, g=self.g, pg=self.pg, d=self.d, xt=self.xt, gt=self.gt, S=self.S, Y=self.Y,
                    SY=sm[:MM], YY=sm[MM: 2 * MM], fh=sm[2 * MM: 2 * MM + max(P.past, 1)],
                    sc=sm[2 * MM + max(P.past, 1):], l2=self.coef[:N], l1c=self.coef[N: 2 * N],
                    isg=self.coef[2 * N:], fl=self.flags, wb=self.wb, out=self.out)
        for k, t in ptrs.items():
            setattr(a, k, t.data_ptr())

        if os.environ.get("SRML_QN_PROBE") == "1":  # per-section wall-clock stamps of the step kernel
            self.probe = ops.zeros(16, dtype=torch.int64, device=device)
            a.probe = self.probe.data_ptr()
        self._args = a
        self._keep = ptrs
        self._mb = None
        lib = native.lib()
        # the one-launch step spins on software grid barriers: only when all its blocks are
        # guaranteed co-resident (occupancy x CUs), else the multi-launch step
        self._fused = QN_MB and QN_STEP == "fused" and bool(lib.srml_qn_fused_resident(N))
        self.fold: Optional[tuple] = None  # (partial-row workspace, rows, stride) the fused step folds
        if QN_MB and N <= 16384 and os.environ.get("SRML_QN_PROBE") != "1":
            size = int(lib.srml_qn_fused_scratch() if self._fused else lib.srml_qn_mb_scratch())
            self._mb = ops.zeros(size, **f64)  # zeroed: the fused step's barrier words start at 0
        assert ctypes.sizeof(_QnArgs) == int(native.lib().srml_qn_args_size()), "QnArgs layout mismatch"

    @property
    def w_dev(self) -> torch.Tensor:
        return self.wb[: self.P.Kn]

    @property
    def b_dev(self) -> torch.Tensor:
        return self.wb[self.P.Kn:]

    def step(self) -> None:
        from ..ops import native

        if self._mb is not None and self._fused:
            ws, parts, wst = self.fold if self.fold is not None else (None, 0, 0)
            native.call("srml_qn_step_fused", ctypes.addressof(self._args), self._mb.data_ptr(),
                        ws.data_ptr() if ws is not None else None, int(parts), int(wst), native.stream(self.device))
        elif self._mb is not None and self.fold is not None:
            ws, parts, wst = self.fold
            native.call("srml_qn_step_mbf", ctypes.addressof(self._args), self._mb.data_ptr(), ws.data_ptr(),
                        int(parts), int(wst), native.stream(self.device))
        elif self._mb is not None:
            native.call("srml_qn_step_mb", ctypes.addressof(self._args), self._mb.data_ptr(), native.stream(self.device))
        else:
            native.call("srml_qn_step", ctypes.addressof(self._args), native.stream(self.device))

    def theta(self) -> np.ndarray:
        return self.x.cpu().numpy().copy()

    def zcache_supported(self) -> bool:
        """The margin cache needs the multi-block or single-block step (the one-launch fused step
        ignores its flags), a backtracking Armijo search and no L1 (the orthant projection is not
        linear in the step)."""
        return not (self._mb is not None and self._fused) and not self.P.use_l1 and not self.P.wolfe

    def enable_zcache(self, zbuf: torch.Tensor) -> tuple:
        """Switch the margin cache on (``zbuf``: 2 m fp64): returns the evaluation's (flags, buffer,
        scalars) triple for ``ops.logistic_loss_grad(zcache=...)``."""
        self.flags[F_ZC] = 1
        return (self.flags, zbuf, self._keep["sc"])

    def info(self) -> dict:
        fl = self.flags.cpu().numpy()
        sc = self._keep["sc"].cpu().numpy()
        return {"iter": int(fl[F_ITER]), "n_evals": int(fl[F_NEVAL]), "status": STATUS.get(int(fl[F_STATUS]), "?"),
                "f": float(sc[SC_F]), "done": bool(fl[F_DONE]), "n_margin_only": int(fl[F_NCHEAP])}


# ------------------------------------------------------------------------------------------
def _graph_capturable(allreduce: Callable) -> bool:
    """Whether a bound ``Communicator.allreduce`` can be recorded into a HIP graph: RCCL
    collectives can (one-shot and host-staged gloo ones cannot: a per-call epoch / a host copy)."""
    comm = getattr(allreduce, "__self__", None)
    if comm is None or getattr(comm, "backend", "none") != "nccl":
        return False
    from ..parallel import oneshot

    return oneshot.comm_mode() == "rccl"


def _comm_poll(allreduce: Optional[Callable]) -> Optional[Callable[[], None]]:
    """The non-blocking error poll of the communicator behind a bound ``allreduce`` (if any)."""
    return getattr(getattr(allreduce, "__self__", None), "poll", None)


def minimize(P: QNProblem, theta0: np.ndarray, evaluate: Callable[[torch.Tensor, torch.Tensor, Optional[torch.Tensor],
                                                                   torch.Tensor], None],
             allreduce: Optional[Callable[[torch.Tensor], None]], device: torch.device,
             batch: int = 8, graph_safe: bool = False, fold: Optional[tuple] = None,
             evaluate_partials: Optional[Callable] = None, zcache: Optional[torch.Tensor] = None) -> dict:
    """Run the QN iteration. ``evaluate(w, b, flag, out)`` must ADD the summed data-term
    [grad_w (K*n) | grad_b (K) | loss] of this rank's rows at (w, b) into ``out`` (device
    tensors; ``flag`` is the device done-flag it may use to early-exit, None on the host path).
    ``allreduce(out)`` sums ``out`` over ranks in place (None for one rank). ``graph_safe``: the
    evaluation is stream-ordered device work only (no host sync, no allocation), so a one-rank fit
    may capture the batch in a HIP graph (``SRML_QN_GRAPH=0`` disables).

    ``fold`` = (workspace, rows, stride) with ``evaluate_partials(w, b, flag)``: a one-rank fit
    whose evaluation can leave per-block partial rows in the workspace instead of summing into
    ``out``; the fused device step then folds them itself (one launch less per evaluation).

    ``zcache`` (2 m fp64, binary LogisticRegression on the prefetching kernel): the line-search
    margin cache — ``evaluate`` / ``evaluate_partials`` then take a ``zc`` keyword (see
    ``DeviceQN.enable_zcache``) and a rejected trial's backtracking costs margins-only passes.

    Returns {theta, f, iter, n_evals, status}.
    """
    if device.type != "cuda":
        st = HostQN(P, theta0)
        out = ops.zeros(P.out_len, dtype=torch.float64, device=device)
        cap = max(1, P.max_iter) * (P.max_ls + 1) + 2
        while not st.done and st.n_evals < cap:
            wb = torch.from_numpy(st.wb()).to(device)
            out.zero_()
            evaluate(wb[: P.Kn], wb[P.Kn:], None, out)
            if allreduce is not None:
                allreduce(out)
            st.step(out.cpu().numpy())
        return {"theta": st.theta(), "f": st.f, "iter": st.iter, "n_evals": st.n_evals,
                "status": STATUS[st.status if st.done else 3]}
    q = DeviceQN(P, theta0, device)
    zc = None
    if zcache is not None and QN_ZCACHE and q.zcache_supported():
        zc = q.enable_zcache(zcache)
    if fold is not None and evaluate_partials is not None and allreduce is None and q._mb is not None:
        q.fold = fold
        evaluate = lambda w, b, flag, out, **kw: evaluate_partials(w, b, flag, **kw)  # noqa: E731
    zkw = {"zc": zc} if zc is not None else {}
    poll = _comm_poll(allreduce)
    flag = q.flags[F_DONE: F_DONE + 1]
    host_flag = ops.zeros(2, dtype=torch.int32, pin_memory=True)
    events: list = []
    # a margins-only trial accepted costs one more (full) evaluation of its iteration
    cap = max(1, P.max_iter) * (P.max_ls + (2 if zc is not None else 1)) + 2
    evals = 0
    stream = torch.cuda.current_stream(device)
    j = 0

    def run_batch() -> None:
        for _ in range(batch):
            evaluate(q.w_dev, q.b_dev, flag, q.out, **zkw)
            if allreduce is not None:
                allreduce(q.out)
            q.step()

    # one-rank fits on a single-launch evaluation replay the batch as ONE HIP graph: 2 x batch
    # kernels with no per-launch host work (the first batch runs eagerly: one-time kernel set-up)
    graph = None
    use_graph = graph_safe and QN_GRAPH and (allreduce is None or (QN_GRAPH_COMM and _graph_capturable(allreduce)))
    while evals < cap:
        if graph is not None:
            graph.replay()
            GRAPH_STATS["replays"] += 1
        else:
            run_batch()
            if use_graph and evals + batch < cap:
                # raw capture on a side stream (torch.cuda.graph's context manager also runs
                # gc.collect + empty_cache: milliseconds inside the fit)
                graph = torch.cuda.CUDAGraph()
                side = torch.cuda.Stream(device)
                side.wait_stream(stream)
                try:
                    with torch.cuda.stream(side):
                        graph.capture_begin()
                        try:
                            run_batch()
                        finally:
                            graph.capture_end()
                    GRAPH_STATS["captures"] += 1
                except RuntimeError:
                    if allreduce is None:
                        raise
                    # a backend that cannot record its collective: the remaining batches run
                    # eagerly (the failed capture executed nothing)
                    graph, use_graph = None, False
                    GRAPH_STATS["comm_capture_failed"] = GRAPH_STATS.get("comm_capture_failed", 0) + 1
                stream.wait_stream(side)
                # capture records without running: the captured batch is still to be executed
                # (replayed at the top of the next pass)
        evals += batch
        slot = host_flag[j % 2: j % 2 + 1]
        slot.copy_(flag, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        events.append((ev, slot))
        j += 1
        if poll is not None:
            poll()  # a collective of an earlier batch lost a peer: raise instead of iterating on NaN
        if len(events) >= 2:
            ev0, s0 = events.pop(0)
            ev0.synchronize()
            if int(s0.item()):
                break
    torch.cuda.synchronize(device)
    res = q.info()
    if res["status"] == "barrier timeout":
        if q._mb is not None and q._fused:  # leave the barrier words at zero, as every launch must
            from ..ops import native

            off = int(native.lib().srml_qn_fused_barrier_offset())
            q._mb[off: off + 1].zero_()
        raise RuntimeError("device L-BFGS step: a grid barrier timed out (blocks not co-resident)")
    res["theta"] = q.theta()
    if not res["done"]:
        res["status"] = "evaluation cap"
    return res


def minimize_batch(Ps: List[QNProblem], theta0s: List[np.ndarray],
                   evaluate: Callable[[torch.Tensor, torch.Tensor], None],
                   allreduce: Optional[Callable[[torch.Tensor], None]], device: torch.device,
                   batch: int = 8) -> List[dict]:
    """Hyper-parameter batching: B independent binary problems of one width advance together.
    ``evaluate(WB, OUT)`` must ADD the data terms of all B models at the rows of WB (B, n + 1) into
    OUT (B, n + 2) — one pass over X for the whole batch; the B optimiser steps run as ONE launch
    (``srml_qn_step_batch``, a block per problem). Problems that converged keep their state while
    the others continue; the loop ends when every done flag is set."""
    from ..ops import native

    B = len(Ps)
    n = Ps[0].n
    assert all(P.K == 1 and P.n == n for P in Ps), "batched QN needs binary problems of one width"
    f64 = dict(dtype=torch.float64, device=device)
    WB = ops.zeros((B, n + 1), **f64)
    OUT = ops.zeros((B, n + 2), **f64)
    FL = ops.zeros((B, 16), dtype=torch.int32, device=device)
    qs = [DeviceQN(P, th, device, wb=WB[j], out=OUT[j], flags=FL[j]) for j, (P, th) in enumerate(zip(Ps, theta0s))]
    raw = b"".join(bytes(q._args) for q in qs)
    args_dev = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
    st = native.stream(device)
    host = ops.zeros(2, dtype=torch.int32, pin_memory=True)
    cap = max(max(1, P.max_iter) * (P.max_ls + 1) + 2 for P in Ps)
    evals, j = 0, 0
    events: list = []
    stream = torch.cuda.current_stream(device)
    poll = _comm_poll(allreduce)
    while evals < cap:
        for _ in range(batch):
            evaluate(WB, OUT)
            if allreduce is not None:
                allreduce(OUT)
            native.call("srml_qn_step_batch", args_dev.data_ptr(), B, st)
        evals += batch
        slot = host[j % 2: j % 2 + 1]
        slot.copy_(FL[:, F_DONE].min().view(1), non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        events.append((ev, slot))
        j += 1
        if poll is not None:
            poll()
        if len(events) >= 2:
            ev0, s0 = events.pop(0)
            ev0.synchronize()
            if int(s0.item()):
                break
    torch.cuda.synchronize(device)
    out = []
    for q in qs:
        r = q.info()
        r["theta"] = q.theta()
        if not r["done"]:
            r["status"] = "evaluation cap"
        out.append(r)
    return out
