"""Device primitives. GPU tensors -> hand-written gfx950 HIP kernels (``libsrml_ops.so``);
CPU tensors -> PyTorch reference implementations of the same math (used by GPU-less CI and as
the numerics oracle in the kernel tests).
"""
from __future__ import annotations

import math
import os
from typing import Any, Dict, Iterator, Optional, Tuple

import numpy as np
import torch

from . import native
from ..utils.determinism import deterministic

__all__ = ["col_moments", "gram", "xw", "dgemm", "sign_flip", "is_native", "xtv", "row_sqnorm",
           "logreg_binary_loss_grad", "nearest_centroid", "cluster_sums", "csr_logreg_binary_loss_grad",
           "csr_spmm", "csr_spmtm", "csr_col_moments", "logistic_loss_grad"]


def is_native(t: torch.Tensor) -> bool:
    return t.is_cuda


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------------------------------
def col_moments(X: torch.Tensor, need_sq: bool = True,
                out: Optional[Tuple[torch.Tensor, Optional[torch.Tensor]]] = None
                ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Per-column fp64 (sum, sum of squares) of a row-major (m, n) matrix. ``out`` = (sum, sumsq)
    fp64 accumulators to ADD into (the kernel folds with atomics: a streamed pass over row chunks
    needs no per-chunk zero fill or add)."""
    m, n = X.shape
    if not X.is_cuda:
        Xd = X.double()
        if out is not None:
            out[0].add_(Xd.sum(0))
            if need_sq:
                out[1].add_((Xd * Xd).sum(0))
            return out
        return Xd.sum(0), (Xd * Xd).sum(0) if need_sq else None
    X = _c(X)
    if out is not None:
        s, q = out[0], (out[1] if need_sq else None)
        if s.dtype != torch.float64 or not s.is_contiguous() or (q is not None and (q.dtype != torch.float64
                                                                                    or not q.is_contiguous())):
            raise ValueError("col_moments(out=): contiguous fp64 accumulators")
    else:
        s = zeros(n, dtype=torch.float64, device=X.device)
        q = zeros(n, dtype=torch.float64, device=X.device) if need_sq else None
    name = "srml_col_moments_f32" if X.dtype == torch.float32 else "srml_col_moments_f64"
    if X.dtype not in (torch.float32, torch.float64):
        raise TypeError("col_moments supports fp32/fp64")
    native.call(name, X.data_ptr(), m, n, X.stride(0), s.data_ptr(), q.data_ptr() if q is not None else None,
                native.stream(X.device))
    return s, q


def gram(X: torch.Tensor, mean: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
         finalize: bool = True) -> torch.Tensor:
    """out (fp64 n x n) += (X - mean)^T (X - mean); returns out (full symmetric matrix).

    ``finalize=False`` (streaming, one call per row chunk): only the upper triangle of ``out``
    is accumulated, in place; call ``gram_mirror(out)`` once after the last chunk."""
    m, n = X.shape
    if out is None:
        out = zeros((n, n), dtype=torch.float64, device=X.device)
    if not X.is_cuda or X.dtype != torch.float32:
        Xc = X - mean.to(X.dtype) if mean is not None else X
        if X.is_cuda:
            # fp64 inputs: f64 path on the f64 MFMA dgemm (A^T A)
            dgemm(_c(Xc), _c(Xc), ta=True, tb=False, alpha=1.0, beta=1.0, out=out)
        else:
            Xc = Xc.double()
            out += Xc.T @ Xc
        return out
    X = _c(X)
    mu = _c(mean.to(torch.float32)) if mean is not None else None
    st = native.stream(X.device)
    ws, wsc = None, 0
    if deterministic():  # per-chunk partial tiles folded in order (<= 64 chunks, <= 1 GB)
        wsc = int(max(1, min(64, (1 << 30) // (8 * n * n))))
        ws = torch.empty(wsc * n * n, dtype=torch.float64, device=X.device)
    wsp = ws.data_ptr() if ws is not None else None
    if not finalize:
        native.call("srml_gram_f32_ex", X.data_ptr(), m, n, X.stride(0), mu.data_ptr() if mu is not None else None,
                    out.data_ptr(), wsp, wsc, st)
        return out
    # the kernel accumulates only the upper triangle; mirror into a temporary, then add
    up = torch.zeros_like(out)
    native.call("srml_gram_f32_ex", X.data_ptr(), m, n, X.stride(0), mu.data_ptr() if mu is not None else None,
                up.data_ptr(), wsp, wsc, st)
    native.call("srml_mirror_upper_f64", up.data_ptr(), n, st)
    out += up
    return out


def gram_mirror(G: torch.Tensor) -> torch.Tensor:
    """Complete a streaming (upper-triangle) Gram accumulation into the full symmetric matrix."""
    if not G.is_cuda:
        iu = torch.triu_indices(G.shape[0], G.shape[0], 1)
        G[iu[1], iu[0]] = G[iu[0], iu[1]]
        return G
    native.call("srml_mirror_upper_f64", G.data_ptr(), G.shape[0], native.stream(G.device))
    return G


_XW_WIDTHS = (1, 2, 3, 4, 8, 16, 32)


def xw(X: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = X @ W (+ bias): X (m, n), W (n, k). fp32: one bandwidth-bound pass over X per 32
    output columns (``srml_xw_f32``); fp64: the f64-MFMA GEMM (``srml_dgemm``)."""
    m, n = X.shape
    k = W.shape[1]
    if not X.is_cuda:
        out = X.to(W.dtype) @ W
        return out + bias if bias is not None else out
    if X.dtype == torch.float64:
        out = torch.empty((m, k), dtype=torch.float64, device=X.device)
        if bias is not None:
            out.copy_(bias.to(device=X.device, dtype=torch.float64).view(1, k).expand(m, k))
        dgemm(_c(X), W.to(device=X.device, dtype=torch.float64), beta=1.0 if bias is not None else 0.0, out=out)
        return out
    if X.dtype != torch.float32:
        raise TypeError("xw supports fp32/fp64 inputs, got %s" % X.dtype)
    if k > 32:
        cols = [xw(X, W[:, c0: c0 + 32], bias[c0: c0 + 32] if bias is not None else None) for c0 in range(0, k, 32)]
        return torch.cat(cols, 1)
    X = _c(X)
    if k >= XW_MFMA_MIN_K:
        return xw_t(X, W.t().to(torch.float32).contiguous(), bias)
    kk = next(w for w in _XW_WIDTHS if w >= k)
    Wp = zeros((n, kk), dtype=torch.float32, device=X.device)
    Wp[:, :k] = W.to(torch.float32)
    bp = None
    if bias is not None:
        bp = zeros(kk, dtype=torch.float32, device=X.device)
        bp[:k] = bias.to(torch.float32)
    out = torch.empty((m, kk), dtype=torch.float32, device=X.device)
    native.call("srml_xw_f32", X.data_ptr(), m, n, X.stride(0), Wp.data_ptr(), kk,
                bp.data_ptr() if bp is not None else None, out.data_ptr(), kk, native.stream(X.device))
    return out[:, :k] if kk != k else out


# K from which the skinny products run on the fp32 MFMA kernels (tools/skinny_bench.py at 1M x 3000:
# the VALU X W kernel re-reads W from LDS per element and loses to the MFMA one from K = 3 up).
XW_MFMA_MIN_K = 3
XTV_MFMA_MIN_K = 5


def xw_t(X: torch.Tensor, Wt: torch.Tensor, bias: Optional[torch.Tensor] = None,
         out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 out (m, K) = X Wt^T (+ bias) for K <= 32 on the exact-fp32 MFMA (``srml_xw_t_f32``):
    Wt (K, n) fp32 with unit column stride (any row stride), one bandwidth-bound pass over X."""
    m, n = X.shape
    K = Wt.shape[0]
    if out is None:
        out = torch.empty((m, K), dtype=torch.float32, device=X.device)
    if not X.is_cuda:
        out.copy_(X.float() @ Wt.float().t() + (bias.float() if bias is not None else 0.0))
        return out
    if K > 32 or Wt.dtype != torch.float32 or Wt.stride(1) != 1 or out.stride(1) != 1:
        raise ValueError("xw_t: Wt must be fp32 (K <= 32, n) with unit column stride")
    X = _c(X)
    bp = _c(bias.to(device=X.device, dtype=torch.float32)) if bias is not None else None
    native.call("srml_xw_t_f32", X.data_ptr(), m, n, X.stride(0), Wt.data_ptr(), K, Wt.stride(0),
                bp.data_ptr() if bp is not None else None, out.data_ptr(), out.stride(0), native.stream(X.device))
    return out


def dgemm(A: torch.Tensor, B: torch.Tensor, ta: bool = False, tb: bool = False, alpha: float = 1.0,
          beta: float = 0.0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp64 out = alpha op(A) op(B) + beta out (row-major)."""
    M = A.shape[1] if ta else A.shape[0]
    K = A.shape[0] if ta else A.shape[1]
    N = B.shape[0] if tb else B.shape[1]
    if out is None:
        out = zeros((M, N), dtype=torch.float64, device=A.device)
        beta = 0.0
    if not A.is_cuda:
        a = A.double().T if ta else A.double()
        b = B.double().T if tb else B.double()
        res = alpha * (a @ b)
        if beta != 0.0:
            res = res + beta * out
        out.copy_(res)
        return out
    A = _c(A.double())
    B = _c(B.double())
    if out.stride(1) != 1:
        raise ValueError("dgemm: out must have unit column stride")
    st = native.stream(A.device)
    tiles = ((M + 63) // 64) * ((N + 63) // 64)
    splits = _dgemm_splits(M, N, K, tiles)
    if splits > 1:
        ws = torch.empty(splits * M * N, dtype=torch.float64, device=A.device)
        native.call("srml_dgemm_splitk", int(ta), int(tb), M, N, K, float(alpha), A.data_ptr(), A.stride(0),
                    B.data_ptr(), B.stride(0), float(beta), out.data_ptr(), out.stride(0), splits, ws.data_ptr(), st)
        return out
    native.call("srml_dgemm", int(ta), int(tb), M, N, K, float(alpha), A.data_ptr(), A.stride(0), B.data_ptr(),
                B.stride(0), float(beta), out.data_ptr(), out.stride(0), st)
    return out


def _dgemm_splits(M: int, N: int, K: int, tiles: int) -> int:
    """K splits for the fp64 GEMM: enough 64x64 tiles x splits to cover the 256 CUs ~4x, each
    split >= 64 deep, workspace (splits x M x N fp64) <= 256 MB."""
    if tiles >= 512 or K < 128:
        return 1
    want = (1024 + tiles - 1) // tiles
    by_k = K // 64
    by_mem = max(1, (256 << 20) // max(1, 8 * M * N))
    return max(1, min(want, by_k, by_mem))


def sign_flip(U: torch.Tensor) -> torch.Tensor:
    """In place: make the max-|x| entry of every column of U (rows, cols) positive."""
    rows, cols = U.shape
    if not U.is_cuda or U.dtype != torch.float64 or not U.is_contiguous():
        idx = U.abs().argmax(0)
        s = torch.sign(U[idx, torch.arange(cols, device=U.device)])
        s[s == 0] = 1
        U.mul_(s)
        return U
    native.call("srml_sign_flip_f64", U.data_ptr(), rows, cols, U.stride(0), native.stream(U.device))
    return U


# ------------------------------------------------------------------------------------------
# GLM / KMeans primitives
# ------------------------------------------------------------------------------------------
def xtv(X: torch.Tensor, V: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out (n, k) fp64 += X^T V for X (m, n) fp32 and V (m, k) (k <= 4 native; wider -> chunks)."""
    m, n = X.shape
    V2 = V.reshape(m, -1)
    k = V2.shape[1]
    if out is None:
        out = zeros((n, k), dtype=torch.float64, device=X.device)
    if not X.is_cuda:
        out += X.double().T @ V2.double()
        return out
    if X.dtype == torch.float64:
        dgemm(_c(X), _c(V2.to(torch.float64)), ta=True, beta=1.0, out=out)  # split-K f64 MFMA
        return out
    if X.dtype != torch.float32:
        raise TypeError("xtv supports fp32/fp64 inputs, got %s" % X.dtype)
    X = _c(X)
    if k >= XTV_MFMA_MIN_K:
        for c0 in range(0, k, 16):
            kk = min(16, k - c0)
            Vc = _c(V2[:, c0: c0 + kk].to(torch.float32))
            oc = out[:, c0: c0 + kk]
            native.call("srml_xtv_mfma_f32", X.data_ptr(), m, n, X.stride(0), Vc.data_ptr(), kk, Vc.stride(0),
                        oc.data_ptr(), oc.stride(0), oc.stride(1), None, native.stream(X.device))
        return out
    if k <= 4 and out.is_contiguous() and out.dtype == torch.float64:
        # the kernel folds into out with fp64 atomics: accumulate in place (a streamed X^T y over
        # row chunks then needs no per-chunk temporary, zero fill or add)
        Vc = _c(V2.to(torch.float32))
        native.call("srml_xtv_f32", X.data_ptr(), m, n, X.stride(0), Vc.data_ptr(), k, Vc.stride(0), out.data_ptr(),
                    native.stream(X.device))
        return out
    for c0 in range(0, k, 4):
        kk = min(4, k - c0)
        Vc = _c(V2[:, c0: c0 + kk].to(torch.float32))
        tmp = zeros((n, kk), dtype=torch.float64, device=X.device)
        native.call("srml_xtv_f32", X.data_ptr(), m, n, X.stride(0), Vc.data_ptr(), kk, Vc.stride(0), tmp.data_ptr(),
                    native.stream(X.device))
        out[:, c0: c0 + kk] += tmp
    return out


def row_sqnorm(X: torch.Tensor, mu: Optional[torch.Tensor] = None) -> torch.Tensor:
    """||x_r||^2 per row: fp32 for fp32 inputs, fp64 for fp64 inputs on the device.
    ``mu`` (fp32 inputs): ||x_r - mu||^2 (centred norms of the KMeans split search)."""
    m, n = X.shape
    if mu is not None:
        muf = _c(mu.float().view(-1))
        if not X.is_cuda or X.dtype != torch.float32:
            return ((X.float() - muf) ** 2).sum(1)
        X = _c(X)
        out = torch.empty(m, dtype=torch.float32, device=X.device)
        native.call("srml_row_sqnorm_centered_f32", X.data_ptr(), m, n, X.stride(0), muf.data_ptr(), out.data_ptr(),
                    native.stream(X.device))
        return out
    if X.is_cuda and X.dtype == torch.float64:
        X = _c(X)
        out = torch.empty(m, dtype=torch.float64, device=X.device)
        native.call("srml_row_sqnorm_f64", X.data_ptr(), m, n, X.stride(0), out.data_ptr(), native.stream(X.device))
        return out
    if not X.is_cuda or X.dtype != torch.float32:
        return (X.float() * X.float()).sum(1)
    X = _c(X)
    out = torch.empty(m, dtype=torch.float32, device=X.device)
    native.call("srml_row_sqnorm_f32", X.data_ptr(), m, n, X.stride(0), out.data_ptr(), native.stream(X.device))
    return out


def logreg_binary_loss_grad(X: torch.Tensor, y: torch.Tensor, w: torch.Tensor, b: float,
                            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp64 [grad_w (n), grad_b, loss_sum] of sum_r softplus(z_r) - y_r z_r, z = X w + b (one pass).
    ``out`` (device, n + 2 fp64): reused result buffer (zeroed here)."""
    m, n = X.shape
    if not X.is_cuda or X.dtype != torch.float32 or n > 4096:
        Xd = X.double()
        z = Xd @ w.double().to(X.device) + b
        yd = y.double()
        p = torch.sigmoid(z)
        r = p - yd
        loss = torch.nn.functional.softplus(z).sum() - (yd * z).sum()
        return torch.cat([Xd.T @ r, r.sum().view(1), loss.view(1)])
    X = _c(X)
    out = zeros(n + 2, dtype=torch.float64, device=X.device) if out is None else zero_(out)
    wf = _c(w.to(device=X.device, dtype=torch.float64))
    yf = _c(y.to(torch.float32))
    ws = logreg_workspace(X)
    native.call("srml_logreg_binary3_f32", X.data_ptr(), m, n, X.stride(0), yf.data_ptr(), wf.data_ptr(), float(b),
                None, None, out.data_ptr(), ws.data_ptr() if ws is not None else None, 0, native.stream(X.device))
    return out


def logreg_fold_layout(X: Any) -> Tuple[int, int]:
    """(partial rows, row stride in floats) of ``logreg_workspace(X)``."""
    m, n = X.shape
    return int(native.lib().srml_logreg_fold_parts(m)), ((n + 3) & ~3) + 4


def logreg_workspace(X: Any) -> Optional[torch.Tensor]:
    """Partial-row workspace of the fused binary evaluation for this shard (one per fit: the
    block partials and their fold are two launches), or None when its kernel needs none."""
    if _is_csr(X) or not X.is_cuda or X.dtype != torch.float32:
        return None
    m, n = X.shape
    # the layout the evaluation will see: X itself, or the (aligned, ld = n) copy _c makes
    ptr, ld = (X.data_ptr(), X.stride(0)) if X.is_contiguous() else (0, n)
    nf = int(native.lib().srml_logreg_fold_ws(m, n, ld, ptr))
    return torch.empty(nf, dtype=torch.float32, device=X.device) if nf > 0 else None


def logreg_zcache_ok(X: Any) -> bool:
    """Whether the binary evaluation of this shard runs a kernel with the optimiser's line-search
    margin cache (``srml_logreg_zcache_ok``: the narrow n <= 512 / prefetching 1024 < n <= 4096
    kernels)."""
    if _is_csr(X) or not X.is_cuda or X.dtype != torch.float32 or deterministic():
        return False
    m, n = X.shape
    ptr, ld = (X.data_ptr(), X.stride(0)) if X.is_contiguous() else (0, n)
    return bool(int(native.lib().srml_logreg_zcache_ok(m, n, ld, ptr)))


def nearest_centroid(X: torch.Tensor, C: torch.Tensor, xnorm: Optional[torch.Tensor] = None,
                     cnorm: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(labels int32 [m], squared distance fp32 [m]) of each row's nearest centroid (fused, no m x k matrix)."""
    m, n = X.shape
    k = C.shape[0]
    if X.is_cuda and X.dtype == torch.float64:
        X = _c(X)
        Cd = _c(C.to(device=X.device, dtype=torch.float64))
        cn = (Cd * Cd).sum(1) if cnorm is None or cnorm.dtype != torch.float64 else _c(cnorm)
        xn = xnorm if xnorm is not None and xnorm.dtype == torch.float64 else row_sqnorm(X)
        labels = torch.empty(m, dtype=torch.int32, device=X.device)
        dist = torch.empty(m, dtype=torch.float32, device=X.device)
        native.call("srml_nearest_centroid_f64", X.data_ptr(), m, n, X.stride(0), Cd.data_ptr(), k, Cd.stride(0),
                    cn.data_ptr(), _c(xn).data_ptr(), labels.data_ptr(), dist.data_ptr(), None,
                    native.stream(X.device))
        return labels, dist
    if cnorm is None:
        cnorm = (C.float() * C.float()).sum(1)
    if not X.is_cuda or X.dtype != torch.float32:
        labels = torch.empty(m, dtype=torch.int32, device=X.device)
        dist = torch.empty(m, dtype=torch.float32, device=X.device)
        bs = max(1, (1 << 24) // max(k, 1))
        for s in range(0, m, bs):
            xb = X[s: s + bs].float()
            d = cnorm.view(1, -1) - 2.0 * (xb @ C.float().T)
            v, i = d.min(1)
            xn = (xb * xb).sum(1) if xnorm is None else xnorm[s: s + bs]
            labels[s: s + bs] = i.int()
            dist[s: s + bs] = (v + xn).clamp_min(0)
        return labels, dist
    X = _c(X)
    C = _c(C.to(torch.float32))
    cn = _c(cnorm.to(torch.float32))
    if lloyd_small_ok(X, k, search_only=True):  # small k: one pass, VALU distances (MFMA tiles idle)
        return kmeans_lloyd_small(X, C, cn, with_sums=False)[:2]
    best = torch.full((m,), -1, dtype=torch.int64, device=X.device)  # 0xFFFF... as uint64
    st = native.stream(X.device)
    native.call("srml_nearest_centroid_f32", X.data_ptr(), m, n, X.stride(0), C.data_ptr(), k, C.stride(0),
                cn.data_ptr(), best.data_ptr(), st)
    if xnorm is None:
        xnorm = row_sqnorm(X)
    labels = torch.empty(m, dtype=torch.int32, device=X.device)
    dist = torch.empty(m, dtype=torch.float32, device=X.device)
    native.call("srml_nn_finalize", best.data_ptr(), m, xnorm.data_ptr(), labels.data_ptr(), dist.data_ptr(), st)
    return labels, dist


def split_bf16x3(X: torch.Tensor, row_multiple: int = 128, tiled: bool = False,
                 mu: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Exact three-way bf16 split of a fp32 matrix: planes P[3][rows_pad][kp] (bf16) with
    X = P[0] + P[1] + P[2] (each plane the round-to-nearest bf16 of the remaining residual),
    rows padded to ``row_multiple`` and columns to a multiple of 16 with zeros.

    ``tiled`` (GPU only): the LDS-DMA kernel's layout P[3][rows_pad/256][kp/16][256][16] — each
    (256-row tile, 16-wide k step) block one contiguous, bank-swizzled 8 KiB image.
    ``mu``: planes of X - mu (centred; fp32 subtraction fused into the split)."""
    m, n = X.shape
    kp = (n + 15) // 16 * 16
    if tiled and X.is_cuda and X.dtype == torch.float32:
        rows_pad = max(256, (m + 255) // 256 * 256)
        X = X if X.stride(1) == 1 else X.contiguous()
        P = torch.empty((3, rows_pad // 256, kp // 16, 256, 16), dtype=torch.bfloat16, device=X.device)
        if mu is not None:
            muf = _c(mu.float().view(-1))
            native.call("srml_split_bf16x3_tiled_centered", X.data_ptr(), m, n, X.stride(0), muf.data_ptr(), kp,
                        rows_pad, P.data_ptr(), native.stream(X.device))
        else:
            native.call("srml_split_bf16x3_tiled", X.data_ptr(), m, n, X.stride(0), kp, rows_pad, P.data_ptr(),
                        native.stream(X.device))
        return P
    if mu is not None:
        X = X.float() - mu.float().view(1, -1)
    rows_pad = max(row_multiple, (m + row_multiple - 1) // row_multiple * row_multiple)
    if not X.is_cuda or X.dtype != torch.float32:
        P = zeros((3, rows_pad, kp), dtype=torch.bfloat16, device=X.device)
        r = X.float()
        for p in range(3):
            P[p, :m, :n] = r.to(torch.bfloat16)
            r = r - P[p, :m, :n].float()
        return P
    X = X if X.stride(1) == 1 else X.contiguous()
    P = torch.empty((3, rows_pad, kp), dtype=torch.bfloat16, device=X.device)
    native.call("srml_split_bf16x3", X.data_ptr(), m, n, X.stride(0), kp, rows_pad, P.data_ptr(),
                native.stream(X.device))
    return P


CERTIFY_TAU = 2.0 ** -13  # dropped-product bound of the 3-product search (3 * 2^-16, 8x slack), per ||x|| ||c||


def split_bf16x3_rows(X: torch.Tensor, rows: torch.Tensor, mu: torch.Tensor) -> torch.Tensor:
    """``split_bf16x3(X[rows], tiled=True, mu=mu)`` without the gathered copy of the rows
    (``srml_split_bf16x3_tiled_centered_rows`` reads them through the index list)."""
    m, n = int(rows.shape[0]), X.shape[1]
    if not X.is_cuda or X.dtype != torch.float32 or X.stride(1) != 1:
        return split_bf16x3(X.index_select(0, rows.long()), tiled=True, mu=mu)
    kp = (n + 15) // 16 * 16
    rows_pad = max(256, (m + 255) // 256 * 256)
    P = torch.empty((3, rows_pad // 256, kp // 16, 256, 16), dtype=torch.bfloat16, device=X.device)
    muf = _c(mu.float().view(-1))
    ri = _c(rows.to(torch.int32))
    native.call("srml_split_bf16x3_tiled_centered_rows", X.data_ptr(), X.stride(0), ri.data_ptr(), m, n,
                muf.data_ptr(), kp, rows_pad, P.data_ptr(), native.stream(X.device))
    return P


def certify_tau(n: int) -> float:
    """Worst-case |d~ - d| of the 3-product search vs the fp32 6-product search, relative to
    ||x|| ||c||: the dropped products (``CERTIFY_TAU``) plus the fp32 accumulation error of BOTH
    searches over n terms (each <= n * 2^-24 * sum|x_i c_i| <= n * 2^-24 ||x|| ||c||, the standard
    gamma_n bound with Cauchy-Schwarz). With this radius a certified row provably gets the label
    the exact search gives it; without the n term the guarantee would only be empirical."""
    return CERTIFY_TAU + 2.0 * float(n) * 2.0 ** -24


def _nearest_centroid_certified(XP: torch.Tensor, X: torch.Tensor, m: int, k: int, CP: torch.Tensor,
                                cn: torch.Tensor, xnorm: torch.Tensor, st: int, mu: Optional[torch.Tensor]
                                ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Filter-and-refine arg-min: the 3-product search (half the MFMAs of the fp32-exact one)
    keeps every row's best and second-best distance; rows whose gap exceeds twice the error
    radius (``certify_tau(n)``: dropped products + worst-case fp32 accumulation of both searches)
    are certified — the exact search provably picks the same centroid — and only the remaining
    near-tie rows are re-searched with the 6-product kernel (their labels and distances are then
    bit-identical to the exact path)."""
    dev = XP.device
    nslot = int(native.lib().srml_nearest_centroid_split_top2_nslot(k))
    keys = torch.empty(m * nslot, dtype=torch.int64, device=dev)
    lob = torch.empty(m * nslot, dtype=torch.float32, device=dev)
    xrows, kp, crows = XP.shape[1] * 256, XP.shape[2] * 16, CP.shape[1] * 256
    xn = _c(xnorm.float())
    tau = certify_tau(int(X.shape[1]) if X is not None else kp)
    cg = (2.0 * tau) * cn.clamp_min(0).sqrt()  # error radius per unit ||x||, per centroid
    native.call("srml_nearest_centroid_split_top2", XP.data_ptr(), m, xrows, kp, CP.data_ptr(), k, crows,
                cn.data_ptr(), cg.data_ptr(), xn.data_ptr(), keys.data_ptr(), lob.data_ptr(), st)
    labels = torch.empty(m, dtype=torch.int32, device=dev)
    dist = torch.empty(m, dtype=torch.float32, device=dev)
    flagged = torch.empty(m, dtype=torch.int32, device=dev)
    cnt = zeros(1, dtype=torch.int32, device=dev)
    native.call("srml_split_top2_select", keys.data_ptr(), lob.data_ptr(), m, nslot, xn.data_ptr(), cg.data_ptr(),
                labels.data_ptr(), dist.data_ptr(), flagged.data_ptr(), cnt.data_ptr(), st)
    del keys, lob
    nf = int(cnt.item())
    _CERTIFY_STATS["rows"] += m
    _CERTIFY_STATS["refined"] += nf
    if nf:
        rows = flagged[:nf]
        XPr = split_bf16x3_rows(X, rows, mu)
        best = torch.full((nf,), -1, dtype=torch.int64, device=dev)
        native.call("srml_nearest_centroid_split_tiled_np", XPr.data_ptr(), nf, XPr.shape[1] * 256, kp,
                    CP.data_ptr(), k, crows, cn.data_ptr(), best.data_ptr(), 6, st)
        native.call("srml_split_scatter_refined", best.data_ptr(), rows.data_ptr(), nf, xn.data_ptr(),
                    labels.data_ptr(), dist.data_ptr(), st)
    return labels, dist


_CERTIFY_STATS = {"rows": 0, "refined": 0}  # filter-and-refine counters (diagnostics / tests)


# ---- fp16 certified filter -----------------------------------------------------------------
F16_U = 2.0 ** -11  # unit roundoff of fp16
F16_A = 2.0 ** -14  # absolute error of an fp16 element below the normal range (flushed or subnormal), scaled units


def certify_tau16(n: int) -> float:
    """Radius of the one-product fp16 filter relative to ||x - mu|| ||c - mu||, against the TRUE
    distances of the fp32 centred operands (the re-search evaluates its candidates in fp64): the fp16
    rounding of both operands (2u + u^2, u = 2^-11; the absolute subnormal term and the fp32 rounding
    of ||c - mu||^2 are separate, ``f16_radius_terms``), the fp32 accumulation of the filter's n
    exact fp16 products (<= n 2^-24 ||x|| ||c||, Cauchy-Schwarz), times 1.01 (fp32 evaluation of
    the norms and of the test itself)."""
    return 1.01 * (2.0 * F16_U + F16_U * F16_U + 1.01 * float(n) * 2.0 ** -24)


def f16_radius_terms(n: int, scale: float, tau: float) -> Tuple[float, float, float]:
    """(xadd, z, z2) of the fp16 filter's certificate: with a = 2^-14 / scale (per-element absolute
    error outside the normal range) the dot-product error gains 2 a sqrt(n) (1 + u)(||v|| + ||w||) + 2 n a^2
    on top of tau ||v|| ||w||; written per candidate j as (||v|| + xadd) g_j + z ||v|| + z2 with
    g_j = 2 tau ||w_j||, i.e. xadd = z / (2 tau)."""
    a = F16_A / scale
    z = 2.02 * a * math.sqrt(n) * (1.0 + F16_U)
    z2 = 2.02 * float(n) * a * a
    # ||c_j - mu||^2 enters d~_j as an fp32 rounding of its fp64 value: <= 2^-24 ||w_j||^2
    # <= (2^-24 wmax / (2 tau)) g_j with wmax = sqrt(n) 2^15 / scale (no element of s w reaches 2^15
    # without raising the overflow flag)
    wmax = math.sqrt(n) * 32768.0 / scale
    return (z + 2.0 ** -24 * wmax) / (2.0 * tau), z, z2


class F16Planes:
    """The fp16 filter's operand for one X: ONE tiled fp16 plane of s (x - mu) (2 B per element
    instead of the 3-product search's 4 staged / 6 stored), the centred row norms and s.

    s is a power of two putting max |x - mu| in [2^13, 2^14) (fp16 max 65504): one pass over X
    computes the centred norms and that maximum (``srml_row_sqnorm_centered_amax_f32``), and one
    host read of it picks s. ``ok`` is False when the data have no finite non-zero range (the
    caller then keeps the bf16 3-product filter)."""

    def __init__(self, X: torch.Tensor, mu: torch.Tensor) -> None:
        m, n = X.shape
        self.X, self.m, self.n = X, m, n
        self.mu = _c(mu.float().view(-1))
        dev = X.device
        st = native.stream(dev)
        self.xnorm = torch.empty(m, dtype=torch.float32, device=dev)
        amax = zeros(1, dtype=torch.int32, device=dev)
        native.call("srml_row_sqnorm_centered_amax_f32", X.data_ptr(), m, n, X.stride(0), self.mu.data_ptr(),
                    self.xnorm.data_ptr(), amax.data_ptr(), st)
        a = float(amax.view(torch.float32).item())
        self.ok = math.isfinite(a) and a > 0.0
        self.scale = 1.0
        self.P = None
        if not self.ok:
            return
        e = math.frexp(a)[1] - 1  # a in [2^e, 2^(e+1))
        if not -100 <= 13 - e <= 100:
            self.ok = False
            return
        self.scale = 2.0 ** (13 - e)
        self.kp = (n + 15) // 16 * 16
        self.rows_pad = max(256, (m + 255) // 256 * 256)
        self.P = torch.empty((self.rows_pad // 256, self.kp // 16, 256, 16), dtype=torch.float16, device=dev)
        self.ovf = zeros(1, dtype=torch.int32, device=dev)
        native.call("srml_split_f16_tiled_centered", X.data_ptr(), m, n, X.stride(0), self.mu.data_ptr(), self.kp,
                    self.rows_pad, self.scale, self.P.data_ptr(), self.ovf.data_ptr(), st)
        self.tau = certify_tau16(n)
        self.xadd, self.z, self.z2 = f16_radius_terms(n, self.scale, self.tau)


F16_CAND_CAP = 64  # candidate-list capacity per re-searched row (more: that row scans every centre)


def _f16_centre_planes(F: F16Planes, C: torch.Tensor, approx: bool) -> Tuple[torch.Tensor, ...]:
    """The centre side of an fp16 search on F's scaled plane: centred centres W = C - mu, their
    norms cn (fp64 sum, one fp32 rounding; allocated for the padded tile rows, entries past k
    unset), the radius terms cg, the [ovf, flagged count] counters zeroed — one launch — and the
    tiled fp16 plane CP of scale * W (X's own plane never overflows; only the centres can)."""
    k, dev = C.shape[0], F.X.device
    st = native.stream(dev)
    Cd = _c(C.to(dev)) if C.dtype in (torch.float32, torch.float64) else _c(C.to(dev, torch.float32))
    crows = max(256, (k + 255) // 256 * 256)
    W = torch.empty((k, F.n), dtype=torch.float32, device=dev)
    cn = torch.empty(crows, dtype=torch.float32, device=dev)
    cg = torch.empty(k, dtype=torch.float32, device=dev)
    zero2 = torch.empty(2, dtype=torch.int32, device=dev)  # [ovf, flagged count]
    native.call("srml_f16_centre_prep", Cd.data_ptr(), int(Cd.dtype == torch.float64), k, F.n, F.mu.data_ptr(),
                float(2.0 * F.tau), int(bool(approx)), W.data_ptr(), cn.data_ptr(), cg.data_ptr(), zero2.data_ptr(), st)
    CP = torch.empty((crows // 256, F.kp // 16, 256, 16), dtype=torch.float16, device=dev)
    native.call("srml_split_f16_tiled_centered", W.data_ptr(), k, F.n, W.stride(0), None, F.kp, crows, F.scale,
                CP.data_ptr(), zero2[0:1].data_ptr(), st)
    return W, cn, cg, zero2, CP, crows


def nearest_f16_labels(F: F16Planes, C: torch.Tensor) -> Optional[torch.Tensor]:
    """int32 arg-min labels of F's rows over the centres C on the fp16 planes (approximate: the
    filter's arg-min, lowest index on ties) in ONE pass per 256-row tile over all centres
    (``srml_nearest_f16_rowloop``: no per-(row, centre tile) slots), or None when the planes are not
    128 halves wide (the caller takes ``nearest_centroid_f16(approx=True)``)."""
    if F.kp != 128 or os.environ.get("SRML_F16_ROWLOOP", "1") == "0":
        return None
    dev = F.X.device
    # (the centre plane's overflow flag is not read: the callers' centres are Lloyd means of rows
    # of X — convex combinations inside the range the plane's scale was chosen for)
    _, cn, _, _, CP, crows = _f16_centre_planes(F, C, True)
    labels = torch.empty(F.m, dtype=torch.int32, device=dev)
    rc = native.lib().srml_nearest_f16_rowloop(F.P.data_ptr(), F.m, F.rows_pad, F.kp, CP.data_ptr(), C.shape[0],
                                                crows, cn.data_ptr(), float(-2.0 / (F.scale * F.scale)),
                                                labels.data_ptr(), native.stream(dev))
    if rc == -2:
        return None
    if rc != 0:
        raise RuntimeError("srml_nearest_f16_rowloop failed (%d)" % rc)
    return labels


def nearest_centroid_f16(F: F16Planes, C: torch.Tensor, approx: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
    """(labels, squared distances) of F.X's rows under centres C by the fp16 certified filter:
    one fp16 MFMA product per (row, centre) on the scaled planes (a third of the 3-product bf16
    filter's MFMAs, half its staged bytes) keeps each row's best and the lowest lower bound of the
    others under the radius ``certify_tau16`` / ``f16_radius_terms`` (proven against the true
    distances of the fp32 centred operands). Rows it cannot certify are re-searched: a second fp16
    pass over just those rows lists every centre whose lower bound does not exceed the row's
    certified upper bound on its best distance (the true arg-min is always listed), and those
    candidates are evaluated exactly in fp64 (``srml_kmeans_cand_exact``). Labels are therefore the
    exact arg-min (lowest index on exact ties) for every row; a certified row's distance is the
    filter's (within its radius: inertia / D^2 weights), a re-searched row's the fp64 one.
    ``approx=True`` (k-means|| D^2 sampling and candidate weights): radius 0 — every row takes the
    filter's arg-min and only exact ties of the filtered distances are re-searched."""
    m, k, dev = F.m, C.shape[0], F.X.device
    st = native.stream(dev)
    W, cn, cg, zero2, CP, crows = _f16_centre_planes(F, C, approx)
    ovf = zero2[0:1]
    xadd, z, z2 = (0.0, 0.0, 0.0) if approx else (F.xadd, F.z, F.z2)
    dscale = -2.0 / (F.scale * F.scale)
    nslot = int(native.lib().srml_nearest_centroid_f16_top2_nslot(k))
    labels = torch.empty(m, dtype=torch.int32, device=dev)
    dist = torch.empty(m, dtype=torch.float32, device=dev)
    flagged = torch.empty(m, dtype=torch.int32, device=dev)
    thr = torch.empty(m, dtype=torch.float32, device=dev)
    cnt = zero2[1:2]  # zeroed by the centre prep
    # row chunks of whole 256-row tiles within the 2^32 work-item grid (512-thread blocks x
    # centre tiles); the select appends each chunk's uncertified rows (chunk-relative) to flagged
    step = split_rows_per_launch(k)
    for r0 in range(0, m, step):
        mc = min(step, m - r0)
        keys = torch.empty(mc * nslot, dtype=torch.int64, device=dev)
        lob = torch.empty(mc * nslot, dtype=torch.float32, device=dev)
        Pc = F.P[r0 // 256: (r0 + mc + 255) // 256]
        xn = F.xnorm[r0: r0 + mc]
        native.call("srml_nearest_centroid_f16_top2", Pc.data_ptr(), mc, Pc.shape[0] * 256, F.kp, CP.data_ptr(), k,
                    crows, cn.data_ptr(), cg.data_ptr(), xn.data_ptr(), dscale, xadd, keys.data_ptr(), lob.data_ptr(),
                    st)
        c0 = int(cnt.item()) if r0 else 0
        native.call("srml_split_top2_select_f16_thr", keys.data_ptr(), lob.data_ptr(), mc, nslot, xn.data_ptr(),
                    cg.data_ptr(), xadd, z, z2, ovf.data_ptr(), labels[r0:].data_ptr(), dist[r0:].data_ptr(),
                    flagged.data_ptr(), cnt.data_ptr(), thr.data_ptr(), st)
        if r0:
            nc = int(cnt.item())
            flagged[c0:nc] += r0
        del keys, lob
    nf = int(cnt.item())
    _CERTIFY_STATS["rows"] += m
    _CERTIFY_STATS["refined"] += nf
    if nf:
        rows = flagged[:nf]
        X = F.X
        assert X.stride(1) == 1
        cap = F16_CAND_CAP
        cand = torch.empty(nf * cap, dtype=torch.int32, device=dev)
        stepr = split_rows_per_launch(k)
        plane = F.P is not None and os.environ.get("SRML_F16_GATHER", "plane") == "plane"
        # plane gather: the same launch gathers the rows' norms and zeroes their candidate counters
        ccount = torch.empty(nf, dtype=torch.int32, device=dev) if plane else zeros(nf, dtype=torch.int32,
                                                                                          device=dev)
        scratch = None if plane else zeros(1, dtype=torch.int32, device=dev)
        for q0 in range(0, nf, stepr):
            nq = min(stepr, nf - q0)
            rq = rows[q0: q0 + nq]
            rp = max(256, (nq + 255) // 256 * 256)
            Pr = torch.empty((rp // 256, F.kp // 16, 256, 16), dtype=torch.float16, device=dev)
            if plane:
                # the flagged rows' slots of the filter's own plane (32 B per k step, no re-conversion)
                xr = torch.empty(nq, dtype=torch.float32, device=dev)
                native.call("srml_f16_plane_gather_rows_ex", F.P.data_ptr(), F.rows_pad, F.kp, rq.data_ptr(), nq, rp,
                            Pr.data_ptr(), F.xnorm.data_ptr(), xr.data_ptr(), ccount[q0:].data_ptr(), st)
            else:
                native.call("srml_split_f16_tiled_centered_rows", X.data_ptr(), X.stride(0), rq.data_ptr(), nq, F.n,
                            F.mu.data_ptr(), F.kp, rp, F.scale, Pr.data_ptr(), scratch.data_ptr(), st)
                xr = F.xnorm.index_select(0, rq.long())
            native.call("srml_nearest_centroid_f16_cand", Pr.data_ptr(), nq, rp, F.kp, CP.data_ptr(), k, crows,
                        cn.data_ptr(), cg.data_ptr(), xr.data_ptr(), dscale, xadd, thr[q0:].data_ptr(),
                        ccount[q0:].data_ptr(), cand[q0 * cap:].data_ptr(), cap, st)
            del Pr
        native.call("srml_kmeans_cand_exact", X.data_ptr(), X.stride(0), F.mu.data_ptr(), W.data_ptr(), W.stride(0),
                    F.n, k, rows.data_ptr(), nf, ccount.data_ptr(), cand.data_ptr(), cap, labels.data_ptr(),
                    dist.data_ptr(), st)
    return labels, dist


def quantizer_planes(X: torch.Tensor) -> Optional[F16Planes]:
    """fp16 filter planes of X for APPROXIMATE nearest-centroid labels (IVF coarse quantisers, whose
    lists only need a good bucketing, not the exact arg-min), or None off the fp32 device path."""
    if not X.is_cuda or X.dtype != torch.float32 or X.dim() != 2 or X.shape[1] < 16 or X.stride(1) != 1:
        return None
    mu = col_moments(X, need_sq=False)[0].div_(max(X.shape[0], 1)).float()
    F = F16Planes(X, mu)
    return F if F.ok else None


def nearest_list(X: torch.Tensor, C: torch.Tensor, F: Optional[F16Planes] = None,
                 xnorm: Optional[torch.Tensor] = None) -> torch.Tensor:
    """int32 labels of X's rows under centres C for bucketing: the fp16 filter's own arg-min (one fp16
    MFMA product per pair, ``nearest_centroid_f16(approx=True)``) when ``F`` (planes of X) is given
    and C has > 256 rows; else the fp32 MFMA search."""
    if F is not None and C.shape[0] > 256:
        lab = nearest_f16_labels(F, C)
        return lab if lab is not None else nearest_centroid_f16(F, C, approx=True)[0]
    return nearest_centroid(X, C, xnorm)[0]


def split_rows_per_launch(k: int) -> int:
    """Rows of one 256 x 256-tile split / fp16 filter launch: 512-thread blocks x ceil(k / 256)
    centre tiles per 256-row tile must stay within the 2^32 work-item grid of a dispatch."""
    ct = max(1, (int(k) + 255) // 256)
    return max(256, (0xFFFFFFFF // 512 // ct) * 256)


def kmeans_filter_mode() -> str:
    """``SRML_KMEANS_FILTER``: ``f16`` (default: one-product fp16 certified filter) or ``bf16``
    (3-product split-bf16 certified filter)."""
    v = os.environ.get("SRML_KMEANS_FILTER", "f16").lower()
    if v not in ("f16", "bf16"):
        raise ValueError("SRML_KMEANS_FILTER must be f16 or bf16, got %r" % v)
    return v


def nearest_centroid_split(XP: torch.Tensor, m: int, C: torch.Tensor, xnorm: torch.Tensor,
                           cnorm: Optional[torch.Tensor] = None, approx: bool = False,
                           X: Optional[torch.Tensor] = None, mu: Optional[torch.Tensor] = None
                           ) -> Tuple[torch.Tensor, torch.Tensor]:
    """``nearest_centroid`` on pre-split X planes (``split_bf16x3``): the distance GEMM runs on
    the bf16 matrix cores as six cross products of the planes (fp32-accurate; see splitmm.hip).
    ``approx=True`` (tiled planes): only the three leading products (~2^-16 relative dot error,
    half the MFMAs) — for consumers of approximate distances (k-means|| sampling).
    ``X`` given (tiled planes, GPU): certified filter-and-refine search — the 3-product pass plus
    an exact 6-product re-search of the near-tie rows only; same labels as the exact search.
    ``mu``: XP holds planes of X - mu (``split_bf16x3(..., mu=mu)``) and ``xnorm`` = ||x - mu||^2;
    the centroids are centred the same way (distances are translation invariant)."""
    k = C.shape[0]
    Cf = C.float()
    if mu is not None:
        Cf = Cf - mu.float().view(1, -1).to(Cf.device)
        cnorm = None
    if cnorm is None:
        cnorm = (Cf * Cf).sum(1)
    tiled = XP.dim() == 5
    CP = split_bf16x3(_c(Cf).to(XP.device), 256 if (k > 256 or tiled) else 128, tiled=tiled)
    if not XP.is_cuda:
        Xh, Xm, Xl = (XP[p, :m].float() for p in range(3))
        Ch, Cm, Cl = (CP[p, :k].float() for p in range(3))
        dot = Xm @ Ch.T + Xh @ Cm.T + Xh @ Ch.T
        if not (approx and tiled):
            dot = Xl @ Ch.T + Xm @ Cm.T + Xh @ Cl.T + dot
        v, i = (cnorm.float().view(1, -1) - 2.0 * dot).min(1)
        return i.int(), (v + xnorm.float()).clamp_min(0)
    cn = _c(cnorm.to(torch.float32))
    st = native.stream(XP.device)
    if X is not None and tiled and not approx:
        return _nearest_centroid_certified(XP, X, m, k, CP, cn, xnorm, st, mu)
    best = torch.full((m,), -1, dtype=torch.int64, device=XP.device)
    if tiled:
        native.call("srml_nearest_centroid_split_tiled_np", XP.data_ptr(), m, XP.shape[1] * 256, XP.shape[2] * 16,
                    CP.data_ptr(), k, CP.shape[1] * 256, cn.data_ptr(), best.data_ptr(), 3 if approx else 6, st)
    else:
        native.call("srml_nearest_centroid_split", XP.data_ptr(), m, XP.shape[1], XP.shape[2], CP.data_ptr(), k,
                    CP.shape[1], cn.data_ptr(), best.data_ptr(), st)
    labels = torch.empty(m, dtype=torch.int32, device=XP.device)
    dist = torch.empty(m, dtype=torch.float32, device=XP.device)
    native.call("srml_nn_finalize", best.data_ptr(), m, _c(xnorm.float()).data_ptr(), labels.data_ptr(),
                dist.data_ptr(), st)
    return labels, dist


_M64 = (1 << 64) - 1


def _splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


def _uniform01(seed: int, ctr: int) -> float:
    return (_splitmix64((seed * 0x2545F4914F6CDD1D + ctr) & _M64) >> 11) * (1.0 / 9007199254740992.0)


KMEANSPP_MAX_CANDIDATES = 8192  # KPP_T * KPP_PER in csrc/kmeans.hip


KMEANSPP_MAX_TRIALS = 16


def kmeanspp_trials(k: int) -> int:
    """Greedy k-means++ candidates per centre (scikit-learn / cuML: 2 + floor(ln k))."""
    return int(min(KMEANSPP_MAX_TRIALS, 2 + int(math.log(max(k, 1)))))


def kmeanspp_gram(G: torch.Tensor, w: torch.Tensor, k: int, seed: int, trials: Optional[int] = None) -> torch.Tensor:
    """Greedy weighted k-means++ seeding (indices of k candidates) from the candidates' Gram matrix
    G = C C^T: pick 0 ~ w; every later pick draws ``trials`` candidates ~ w_i min_j ||c_i - c_j||^2
    and keeps the one with the lowest resulting potential. GPU: one block, no host round trip
    per pick; CPU: the same draws (same counter-based uniforms) in numpy."""
    nc = G.shape[0]
    seed = int(seed) & _M64
    L = int(trials) if trials is not None else kmeanspp_trials(k)
    L = max(1, min(L, KMEANSPP_MAX_TRIALS))
    if G.is_cuda and nc <= KMEANSPP_MAX_CANDIDATES:
        out = torch.empty(k, dtype=torch.int32, device=G.device)
        Gd = _c(G.double())
        ldg = nc
        if nc % 4 and nc <= 4096 and L <= 8:  # the register kernel reads 4-candidate groups from 32-B aligned rows
            ldg = nc + (-nc) % 4
            Gp = zeros((nc, ldg), dtype=torch.float64, device=G.device)
            Gp[:, :nc] = Gd
            Gd = Gp
        native.call("srml_kmeanspp_gram", Gd.data_ptr(), nc, ldg, _c(w.double()).data_ptr(), int(k), L, seed,
                    out.data_ptr(), native.stream(G.device))
        return out.long()
    Gh = G.double().cpu().numpy()
    wh = w.double().cpu().numpy()
    diag = np.diag(Gh).copy()
    d2 = np.full(nc, np.inf)

    def draw(p: np.ndarray, ctr: int) -> int:
        cs = np.cumsum(p)
        tot = cs[-1] if nc else 0.0
        if not tot > 0:
            return -1
        i = int(np.searchsorted(cs, _uniform01(seed, ctr) * tot, side="right"))
        return min(i, nc - 1)

    c = max(draw(wh, 0), 0)
    picks = [c]
    for t in range(1, k):
        d2 = np.minimum(d2, np.maximum(diag + Gh[c, c] - 2.0 * Gh[c], 0.0))
        p = wh * d2
        cands = [draw(p, t * KMEANSPP_MAX_TRIALS + j) for j in range(L)]
        if cands[0] < 0:
            c = int(_splitmix64((seed + 77 * t) & _M64) % nc)
        else:
            pots = [float((wh * np.minimum(d2, np.maximum(diag + Gh[x, x] - 2.0 * Gh[x], 0.0))).sum()) for x in cands]
            c = cands[int(np.argmin(pots))]
        picks.append(c)
    return torch.tensor(picks, dtype=torch.long, device=G.device)


def label_sort(labels: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Stable grouping of rows by label in [0, k): (perm int32 — row ids in (label, row) order,
    off int64 (k + 1) — start of every label's run, sorted labels int32). Device: counting sort
    (``srml_label_sort``: per-tile LDS histograms, one scan, ballot-ranked stable scatter; no
    library sort, no host sync). Rows with labels outside [0, k) trail after off[k]."""
    m = labels.shape[0]
    dev = labels.device
    lab = _c(labels.to(torch.int32))
    if not lab.is_cuda or k > int(native.lib().srml_label_sort_kmax()):
        slab, perm = torch.sort(lab, stable=True)
        off = torch.searchsorted(slab, torch.arange(k + 1, device=dev, dtype=slab.dtype)).long()
        return perm.to(torch.int32), off, slab
    perm = torch.empty(m, dtype=torch.int32, device=dev)
    slab = torch.empty(m, dtype=torch.int32, device=dev)
    off = torch.empty(k + 1, dtype=torch.int64, device=dev)
    ws = torch.empty(int(native.lib().srml_label_sort_ws(m, k)), dtype=torch.int64, device=dev)
    native.call("srml_label_sort", lab.data_ptr(), m, int(k), perm.data_ptr(), slab.data_ptr(), off.data_ptr(),
                ws.data_ptr(), native.stream(dev))
    return perm, off, slab


def label_counts(labels: torch.Tensor, k: int) -> torch.Tensor:
    """int64 counts of labels 0..k-1 (others ignored) without a host read-back (``torch.bincount``
    syncs on the maximum): per-block LDS histograms + one u64 atomic per (block, label)."""
    lab = _c(labels.to(torch.int32))
    if not lab.is_cuda or k > int(native.lib().srml_label_sort_kmax()) + 1:
        ok = lab[(lab >= 0) & (lab < k)].long()
        return torch.bincount(ok, minlength=k)[:k]
    counts = zeros(k, dtype=torch.int64, device=lab.device)
    native.call("srml_label_counts", lab.data_ptr(), lab.shape[0], int(k), counts.data_ptr(), native.stream(lab.device))
    return counts


def sorted_counts(sorted_labels: torch.Tensor, k: int) -> torch.Tensor:
    """int64 counts of labels 0..k-1 from an ascending label vector: segment boundaries by binary
    search (no atomics, no host synchronisation - torch.bincount reads the maximum back first)."""
    bounds = torch.searchsorted(sorted_labels.contiguous(),
                                torch.arange(k + 1, device=sorted_labels.device, dtype=sorted_labels.dtype))
    return (bounds[1:] - bounds[:-1]).long()


def lloyd_small_ok(X: torch.Tensor, k: int, search_only: bool = False) -> bool:
    """Whether ``kmeans_lloyd_small`` takes X (fp32 on the device, k <= 32, n <= 64, n % 4 == 0,
    16-B aligned rows); ``SRML_KMEANS_SMALL=0`` disables it."""
    del search_only  # the search alone has the same limits (k in (32, 64]: no faster than MFMA)
    if not (X.is_cuda and X.dtype == torch.float32 and X.dim() == 2 and 1 <= k <= 32):
        return False
    m, n = X.shape
    return (n <= 64 and n % 4 == 0 and X.stride(1) == 1 and X.stride(0) % 4 == 0 and X.data_ptr() % 16 == 0
            and os.environ.get("SRML_KMEANS_SMALL", "1") != "0")


def lloyd_kernel() -> str:
    """Small-k Lloyd kernel: ``mfma`` (default: bf16 matrix cores over an exact 3-way split,
    ``lloyd.hip``) or ``valu`` (``SRML_LLOYD_KERNEL=valu``: VALU distances + f32 one-hot MFMA)."""
    return "valu" if os.environ.get("SRML_LLOYD_KERNEL", "mfma") == "valu" else "mfma"


def kmeans_lloyd_small(X: torch.Tensor, C: torch.Tensor, cnorm: Optional[torch.Tensor] = None,
                       with_sums: bool = True, out: Optional[torch.Tensor] = None,
                       done: Optional[torch.Tensor] = None, labels: Optional[torch.Tensor] = None,
                       dist: Optional[torch.Tensor] = None, rows_out: bool = True,
                       mu: Optional[torch.Tensor] = None,
                       book: Optional[Tuple[torch.Tensor, ...]] = None) -> Tuple[torch.Tensor, ...]:
    """Fused small-k Lloyd step (ONE pass over X): (labels int32, squared distances fp32) and,
    with ``with_sums``, (cluster sums fp64 [k, n], counts int64 [k], inertia fp64 [1]) by those
    labels. ``out`` (fp64 [k n + k + 1], zeroed): the MFMA kernel accumulates [sums | counts |
    inertia] there (the all-reduce buffer of the device Lloyd loop; the returned sums / counts /
    inertia are views of it); ``done`` (int32 device flag): the step is a no-op once it is set;
    ``labels`` / ``dist``: preallocated outputs (a loop reuses them). ``rows_out=False`` (MFMA
    kernel, with ``out``): no per-row labels / distances are written (the Lloyd loop needs only
    the sums, counts and inertia); (None, None, sums, counts, inertia) is returned. ``mu`` (MFMA
    kernel): the rows are searched and summed as x - mu against ``C`` / ``cnorm`` given CENTRED
    (C - mu): the returned sums are of x - mu (labels and distances are unchanged). ``book`` (MFMA
    kernel, with ``out`` of k n + k + 2 doubles): the device Lloyd loop's label book (labels int32
    [m], mode int32 [1]): every row's label is kept and out[k n + k + 1] counts the rows whose
    label changed; when mode is set the step is a DELTA step — out gets the sums' and counts'
    change only, from the tiles holding a moved row (see ``lloyd.hip``)."""
    m, n = X.shape
    k = C.shape[0]
    dev = X.device
    C = _c(C.to(device=dev, dtype=torch.float32))
    cn = _c((C * C).sum(1) if cnorm is None else cnorm.to(device=dev, dtype=torch.float32))
    mfma = lloyd_kernel() == "mfma"
    if not rows_out and not (mfma and with_sums):
        rows_out = True  # only the MFMA kernel's summing step runs without per-row outputs
    if rows_out:
        labels = torch.empty(m, dtype=torch.int32, device=dev) if labels is None else labels
        dist = torch.empty(m, dtype=torch.float32, device=dev) if dist is None else dist
    else:
        labels = dist = None
    if mu is not None and not mfma:
        raise ValueError("kmeans_lloyd_small: mu needs the MFMA kernel")
    if mfma:
        if with_sums and out is None:
            out = zeros(k * n + k + 1, dtype=torch.float64, device=dev)
        muc = _c(mu.to(device=dev, dtype=torch.float32).view(-1)) if mu is not None else None
        bk = [t.data_ptr() for t in book] if book is not None else [None] * 2
        if book is not None and (out is None or out.numel() < k * n + k + 2 or book[0].numel() < m):
            raise ValueError("kmeans_lloyd_small: a label book needs out of k n + k + 2 and m labels")
        native.call("srml_kmeans_lloyd_mfma", X.data_ptr(), m, n, X.stride(0), C.data_ptr(), k, cn.data_ptr(),
                    labels.data_ptr() if rows_out else None, dist.data_ptr() if rows_out else None,
                    out.data_ptr() if with_sums else None,
                    done.data_ptr() if done is not None else None, muc.data_ptr() if muc is not None else None,
                    *bk, native.stream(dev))
        if not with_sums:
            return labels, dist
        return labels, dist, out[: k * n].view(k, n), out[k * n: k * n + k].long(), out[k * n + k:]
    sums = counts = inertia = None
    if with_sums:
        sums = zeros((k, n), dtype=torch.float64, device=dev)
        counts = zeros(k, dtype=torch.int32, device=dev)
        inertia = zeros(1, dtype=torch.float64, device=dev)
    native.call("srml_kmeans_lloyd_small", X.data_ptr(), m, n, X.stride(0), C.data_ptr(), k, cn.data_ptr(),
                labels.data_ptr(), dist.data_ptr(), sums.data_ptr() if with_sums else None,
                counts.data_ptr() if with_sums else None, inertia.data_ptr() if with_sums else None,
                native.stream(dev))
    if not with_sums:
        return labels, dist
    if out is not None:
        out[: k * n].copy_(sums.view(-1))
        out[k * n: k * n + k].copy_(counts)
        out[k * n + k:].copy_(inertia)
    return labels, dist, sums, counts.long(), inertia


class LloydBook:
    """Device bookkeeping of the large-k Lloyd loop (``lloyd_book.hip``), the loop's local buffer
    ``L`` = [sums (k n) | counts (k) | inertia] in fp64 being updated in place:

    * ``moved(labels, prev)``: number of rows whose label changed (one read-back);
    * ``delta_into(X, labels, prev, nm, L)``: L's sums / counts += the moved rows' change (rows
      entering their new cluster, ``~row`` leaving the old one, ONE label sort of both lists, the
      sorted-sum kernel reading X through the row list);
    * ``full_into(X, labels, L)``: L's sums / counts of all rows (label sort + sorted sums);
    * ``inertia_into(d2, L)``: L's inertia = sum of the squared distances (fp64, fixed order);
    * ``update(G, C)``: C (fp64, in place) = sums / counts of the all-reduced buffer G (empty
      clusters keep theirs) -> (max squared centre shift, inertia), one read-back.

    No torch library kernels run in an iteration (the torch bookkeeping was ~37 launches each)."""

    def __init__(self, X: torch.Tensor, k: int) -> None:
        self.m, self.n = X.shape
        self.k = k
        dev = X.device
        self.dev = dev
        lib = native.lib()
        self.blk = torch.empty(max(1, int(lib.srml_lloyd_moved_ws(max(1, self.m)))), dtype=torch.int64, device=dev)
        self.dtot = torch.empty(1, dtype=torch.int64, device=dev)
        self.sum_ws = torch.empty(int(lib.srml_sum_f32_ws()), dtype=torch.float64, device=dev)
        self.part = torch.empty(max(1, k), dtype=torch.float64, device=dev)
        self.out = torch.empty(2, dtype=torch.float64, device=dev)
        self.h_out = torch.empty(2, dtype=torch.float64, pin_memory=True)
        self.h_tot = torch.empty(1, dtype=torch.int64, pin_memory=True)
        self.sorted_ok = X.dtype == torch.float32 and k <= int(lib.srml_label_sort_kmax())

    def _read(self, host: torch.Tensor, dev_t: torch.Tensor) -> torch.Tensor:
        host.copy_(dev_t, non_blocking=True)
        torch.cuda.current_stream(self.dev).synchronize()
        return host

    def moved(self, labels: torch.Tensor, prev: torch.Tensor) -> int:
        native.call("srml_lloyd_moved_count", labels.data_ptr(), prev.data_ptr(), self.m, self.blk.data_ptr(),
                    self.dtot.data_ptr(), native.stream(self.dev))
        return int(self._read(self.h_tot, self.dtot)[0])

    def delta_into(self, X: torch.Tensor, labels: torch.Tensor, prev: torch.Tensor, nm: int,
                   L: torch.Tensor) -> None:
        k, n, st = self.k, self.n, native.stream(self.dev)
        rows2 = torch.empty(2 * nm, dtype=torch.int32, device=self.dev)
        lab2 = torch.empty(2 * nm, dtype=torch.int32, device=self.dev)
        native.call("srml_lloyd_moved_compact", labels.data_ptr(), prev.data_ptr(), self.m, self.blk.data_ptr(), nm,
                    rows2.data_ptr(), lab2.data_ptr(), L[k * n:].data_ptr(), st)
        perm, _, slab = label_sort(lab2, k)
        native.call("srml_kmeans_accumulate_sorted_rows_f32", X.data_ptr(), 2 * nm, n, X.stride(0), perm.data_ptr(),
                    rows2.data_ptr(), slab.data_ptr(), L.data_ptr(), st)

    def full_into(self, X: torch.Tensor, labels: torch.Tensor, L: torch.Tensor) -> None:
        k, n = self.k, self.n
        if not self.sorted_ok:
            sums, counts = cluster_sums(X, labels, k)
            L[: k * n].copy_(sums.view(-1))
            L[k * n: k * n + k].copy_(counts)
            return
        st = native.stream(self.dev)
        perm, off, slab = label_sort(labels, k)
        native.call("srml_memset_async", L.data_ptr(), 0, k * n * 8, st)
        native.call("srml_kmeans_accumulate_sorted_rows_f32", X.data_ptr(), self.m, n, X.stride(0), perm.data_ptr(),
                    None, slab.data_ptr(), L.data_ptr(), st)
        native.call("srml_counts_from_offsets", off.data_ptr(), k, L[k * n:].data_ptr(), st)

    def inertia_into(self, d2: torch.Tensor, L: torch.Tensor) -> None:
        native.call("srml_sum_f32_f64", d2.data_ptr(), d2.shape[0], self.sum_ws.data_ptr(), L[-1:].data_ptr(),
                    native.stream(self.dev))

    def update(self, G: torch.Tensor, C: torch.Tensor) -> Tuple[float, float]:
        native.call("srml_lloyd_centre_update", G.data_ptr(), self.k, self.n, C.data_ptr(), self.part.data_ptr(),
                    self.out.data_ptr(), native.stream(self.dev))
        h = self._read(self.h_out, self.out)
        return float(h[0]), float(h[1])


def kmeans_small_update(buf: torch.Tensor, k: int, n: int, C64: torch.Tensor, C32: torch.Tensor,
                        cnorm: torch.Tensor, tol2: float, flags: torch.Tensor, stat: torch.Tensor,
                        G: Optional[torch.Tensor] = None) -> None:
    """Device centre update of the small-k Lloyd loop (``srml_kmeans_small_update``): C = sums /
    counts from the reduced ``buf`` (empty clusters keep theirs), fp32 copy + norms, the max
    squared shift and the convergence flag (flags = [done, iterations, delta mode]) — no host
    sync. With a label book: ``G`` (k n + k fp64) keeps the running sums / counts (a full step
    sets them, a delta step adds its change) and the next step is a delta step when under 1/4 of
    the rows (all ranks) moved."""
    native.call("srml_kmeans_small_update", buf.data_ptr(), k, n, C64.data_ptr(), C32.data_ptr(), cnorm.data_ptr(),
                float(tol2), flags.data_ptr(), stat.data_ptr(), G.data_ptr() if G is not None else None,
                native.stream(buf.device))


def cluster_sums(X: torch.Tensor, labels: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """(sums fp64 [k, n], counts int64 [k]) of rows grouped by label."""
    m, n = X.shape
    if not X.is_cuda or X.dtype not in (torch.float32, torch.float64):
        sums = zeros((k, n), dtype=torch.float64, device=X.device)
        sums.index_add_(0, labels.long(), X.double())
        counts = torch.bincount(labels.long(), minlength=k)
        return sums, counts
    X = _c(X)
    lab = _c(labels.to(torch.int32))
    if X.dtype == torch.float64 or deterministic():
        # label-sorted segments, one block per (cluster, column chunk), fixed order, no atomics
        perm, off, _ = label_sort(lab, k)
        counts = off[1:] - off[:-1]
        sums = torch.empty((k, n), dtype=torch.float64, device=X.device)
        # split every segment so (clusters x column chunks x splits) covers the chip; the
        # partials are folded in split order (deterministic)
        cblocks = k * ((n + 255) // 256)
        splits = int(max(1, min(64, m // max(1, k * 256), (4096 + cblocks - 1) // cblocks)))
        ws = torch.empty(splits * k * n, dtype=torch.float64, device=X.device) if splits > 1 else None
        name = "srml_kmeans_segment_sums_f64" if X.dtype == torch.float64 else "srml_kmeans_segment_sums_f32"
        native.call(name, X.data_ptr(), m, n, X.stride(0), perm.data_ptr(), off.data_ptr(), k,
                    sums.data_ptr(), splits, ws.data_ptr() if ws is not None else None, native.stream(X.device))
        return sums, counts
    counts = zeros(k, dtype=torch.int32, device=X.device)
    st = native.stream(X.device)
    if k * n * 4 + k * 4 <= 64 * 1024:
        sums = zeros((k, n), dtype=torch.float64, device=X.device)
        native.call("srml_kmeans_accumulate_f32", X.data_ptr(), m, n, X.stride(0), lab.data_ptr(), k, sums.data_ptr(),
                    None, counts.data_ptr(), st)
        return sums, counts.long()
    # large k*n: visit rows in label-sorted order (segment sums, ~(m/256 + k) * n fp64 atomics)
    perm, off, slab = label_sort(lab, k)
    sums = zeros((k, n), dtype=torch.float64, device=X.device)
    native.call("srml_kmeans_accumulate_sorted_f32", X.data_ptr(), m, n, X.stride(0), perm.data_ptr(),
                slab.data_ptr(), sums.data_ptr(), st)
    return sums, off[1:] - off[:-1]


def cluster_sums_rows(X: torch.Tensor, rows: torch.Tensor, labels: torch.Tensor, k: int
                      ) -> Tuple[torch.Tensor, torch.Tensor]:
    """``cluster_sums(X[rows], labels, k)`` without the gathered copy: the rows are label-sorted and
    the sorted-segment kernel reads them from X through the index list (the Lloyd loop's delta
    update over the rows that changed cluster)."""
    n = X.shape[1]
    if not X.is_cuda or X.dtype != torch.float32 or deterministic():
        return cluster_sums(X.index_select(0, rows.long()), labels, k)
    X = _c(X)
    lab = _c(labels.to(torch.int32))
    perm, off, slab = label_sort(lab, k)
    prow = _c(rows.to(torch.int32).index_select(0, perm.long()))
    sums = zeros((k, n), dtype=torch.float64, device=X.device)
    native.call("srml_kmeans_accumulate_sorted_f32", X.data_ptr(), int(rows.shape[0]), n, X.stride(0),
                prow.data_ptr(), slab.data_ptr(), sums.data_ptr(), native.stream(X.device))
    return sums, off[1:] - off[:-1]


def cluster_delta_sums(X: torch.Tensor, rows: torch.Tensor, new_lab: torch.Tensor, old_lab: torch.Tensor, k: int
                       ) -> Tuple[torch.Tensor, torch.Tensor]:
    """Change of the cluster sums / counts when ``rows`` move from ``old_lab`` to ``new_lab``:
    (sums fp64 [k, n], counts int64 [k]) = those of X[rows] by new_lab minus by old_lab. Device:
    ONE label sort of both lists (a leaving row enters as ~row and is subtracted by the sorted-sum
    kernel) instead of two sorted sums and a difference."""
    if not X.is_cuda or X.dtype != torch.float32 or deterministic():
        s_new, c_new = cluster_sums_rows(X, rows, new_lab, k)
        s_old, c_old = cluster_sums_rows(X, rows, old_lab, k)
        return s_new - s_old, c_new - c_old
    n = X.shape[1]
    X = _c(X)
    r32 = rows.to(torch.int32)
    lab2 = torch.cat([new_lab.to(torch.int32), old_lab.to(torch.int32)])
    rows2 = torch.cat([r32, torch.bitwise_not(r32)])
    perm, off, slab = label_sort(lab2, k)
    prow = _c(rows2.index_select(0, perm.long()))
    sums = zeros((k, n), dtype=torch.float64, device=X.device)
    native.call("srml_kmeans_accumulate_sorted_f32", X.data_ptr(), int(prow.shape[0]), n, X.stride(0),
                prow.data_ptr(), slab.data_ptr(), sums.data_ptr(), native.stream(X.device))
    return sums, label_counts(new_lab, k) - label_counts(old_lab, k)


# ------------------------------------------------------------------------------------------
# Random forest primitives
# ------------------------------------------------------------------------------------------
def rf_quantize(X: torch.Tensor, edges: torch.Tensor, out: Optional[torch.Tensor] = None, col0: int = 0
                ) -> torch.Tensor:
    """Feature-major uint8 bins (n, m): bin(x) = #edges[f] strictly below x. edges: (n, B-1) fp32.
    ``out`` (n, M) with ``col0``: the rows of X are rows col0 .. col0 + m of a larger shard (a
    streamed-ingest chunk binned as it lands); returns ``out``."""
    m, n = X.shape
    ne = edges.shape[1]
    if out is None:
        out = torch.empty((n, m), dtype=torch.uint8, device=X.device)
        col0 = 0
    if out.shape[0] != n or out.stride(1) != 1 or col0 < 0 or col0 + m > out.shape[1]:
        raise ValueError("rf_quantize: out must be (n, >= col0 + m) with unit column stride")
    if not X.is_cuda or X.dtype != torch.float32:
        for f in range(n):
            out[f, col0: col0 + m] = torch.searchsorted(edges[f].contiguous().to(X.dtype), X[:, f].contiguous(),
                                                        right=False).to(torch.uint8)
        return out
    X = _c(X)
    e = _c(edges.to(torch.float32))
    native.call("srml_rf_quantize_u8_ld", X.data_ptr(), m, n, X.stride(0), e.data_ptr(), ne, out.data_ptr() + col0,
                out.stride(0), native.stream(X.device))
    return out


def rf_quantiles(S: torch.Tensor, nq: int) -> torch.Tensor:
    """(n, nq) fp32 order statistics floor(q_j k), q_j = (j + 1) / (nq + 1), of every column of the
    (k, n) sample S (NaN ranks as +inf). GPU: one LDS bitonic sort per feature (k <= 32768)."""
    k, n = S.shape
    if not S.is_cuda or k > 32768:
        Ss, _ = torch.sort(torch.nan_to_num(S.float(), nan=float("inf")), 0)
        q = torch.arange(1, nq + 1, device=S.device, dtype=torch.float64) / (nq + 1)
        pos = (q * k).long().clamp(0, k - 1)
        return Ss.index_select(0, pos).T.contiguous()
    ST = S.float().T.contiguous()  # feature-major: each block reads one contiguous column
    out = torch.empty((n, nq), dtype=torch.float32, device=S.device)
    native.call("srml_rf_quantiles_f32", ST.data_ptr(), k, n, nq, out.data_ptr(), native.stream(S.device))
    return out


RF_HIST_FB_MAX = 8  # FB in csrc/forest.hip (checked against srml_rf_hist_fb_max on load in tests)


def rf_yscale(y: torch.Tensor, total_weight: Optional[float] = None) -> float:
    """Fixed-point scale of the regression histograms' i64 w*y sums. Every sum the kernels form —
    a block's LDS cell and the global cross-chunk fold of one (node, feature, bin) cell — covers
    rows of ONE tree, so |sum| <= W * max|y| * yscale with W the largest per-tree bootstrap weight
    total (<= rows * 255); yscale = 2^62 / (W max|y|) keeps every such sum inside i64 whatever the
    row count (1M rows: 2^42 steps per max|y|; 50M: 2^36). Without ``total_weight`` the bound is
    the per-item one (65536 rows * 255)."""
    ymax = float(y.abs().max().item()) if y.numel() else 0.0
    if ymax <= 0:
        return 1.0
    W = float(total_weight) if total_weight is not None and total_weight > 0 else 65536.0 * 255.0
    return float(2.0 ** 62 / (max(W, 1.0) * ymax))


def rf_hist_fb(B: int, S: int, regression: bool) -> int:
    """Features per histogram work item for (B bins, S stats): the per-item LDS slab
    fb * B * S' * 4 bytes (S' = 3 for regression: count + 64-bit fixed-point sum) fits 64 KiB;
    mirrors ``srml_rf_hist_fb``. Raises for histograms that do not fit the 160 KiB LDS at all."""
    per = B * (3 if regression else S) * 4
    fb = min(RF_HIST_FB_MAX, (64 * 1024) // max(per, 1))
    if fb < 1:
        if per > 160 * 1024:
            raise ValueError(f"histogram of {B} bins x {S} classes ({per} bytes per feature) exceeds the 160 KiB LDS")
        fb = 1
    return int(fb)


def rf_hist_fb_wide(B: int, S: int, regression: bool, packed: bool = False) -> int:
    """Features per work item of the wide record-layout histogram (``srml_rf_hist_wide_fb``): the
    1024-thread block's LDS slab (fb * B * S' words + feature metadata) within 150 KiB; S' = 2 for
    the packed regression cells, 3 for count + fixed-point sum, S for class counts."""
    per = B * (2 if (regression and packed) else 3 if regression else S) * 4 + 4
    return int(min(512, (150 * 1024 - 64) // max(per, 1)))


RF_PACK_BITS = 22  # |rint(y * scale)| <= 2^22 (csrc/forest.hip RF_PACK_BIAS)
RF_PACK_MAX_WEIGHT = float(1 << 20)  # per work item: (sum w) << 44 must not overflow


def rf_pack_scale(y: torch.Tensor) -> float:
    """Fixed-point scale of the packed regression cells: 2^22 / max|y| (one host read)."""
    ymax = float(y.abs().max().item()) if y.numel() else 0.0
    return float(1 << RF_PACK_BITS) / ymax if ymax > 0 else 1.0


def rf_interleave(bins: torch.Tensor, rec_bytes: int = 32) -> torch.Tensor:
    """Record layout of a feature-major (n, m) uint8 bin matrix: record (g, r) holds the bins of
    features R g .. R g + R - 1 of row r, R = ``rec_bytes`` (32: the 8-feature item kernel; 32 or
    64: the wide kernel) (``srml_rf_interleave_u8``); flat uint8 tensor."""
    n, m = bins.shape
    # 64-B records are stored in line-sized pairs (groups 2h, 2h + 1 of a row share 128 B)
    span = 128 if rec_bytes == 64 else rec_bytes
    G = (n + span - 1) // span
    out = torch.empty(G * m * span, dtype=torch.uint8, device=bins.device)
    native.call("srml_rf_interleave_u8", _c(bins).data_ptr(), m, n, int(rec_bytes), out.data_ptr(),
                native.stream(bins.device))
    return out


def rf_row_major(bins: torch.Tensor) -> torch.Tensor:
    """Row-major (m, n) copy of a feature-major (n, m) uint8 bin matrix (``srml_rf_transpose_u8``
    on the device: LDS-tiled, one pass each way)."""
    n, m = bins.shape
    if not bins.is_cuda:
        return bins.t().contiguous()
    out = torch.empty((m, n), dtype=torch.uint8, device=bins.device)
    native.call("srml_rf_transpose_u8", _c(bins).data_ptr(), m, n, out.data_ptr(), native.stream(bins.device))
    return out


def rf_il_useful(n: int, nf: int, fb: int) -> bool:
    """Whether a node's chunk of ``fb`` ascending sampled features (nf of n) spans few enough
    32-feature records that the record layout halves the bin loads per row (at least)."""
    span = fb * n / max(nf, 1)
    return span / 32.0 + 1.0 <= fb / 2.0


def rf_hist_wy(idx: torch.Tensor, label: torch.Tensor, wcnt: Optional[torch.Tensor] = None,
               pos_weight: Optional[torch.Tensor] = None) -> torch.Tensor:
    """(weight, label) fp32 pairs in ``idx`` order: the histogram kernels' contiguous row stream
    (device: one ``srml_rf_pack_wy`` pass)."""
    if (idx.is_cuda and pos_weight is not None and wcnt is None and idx.dtype == torch.int32
            and pos_weight.dtype == torch.float32 and label.dtype == torch.float32):
        P = idx.shape[0]
        wy = torch.empty((P, 2), dtype=torch.float32, device=idx.device)
        native.call("srml_rf_pack_wy", _c(idx).data_ptr(), _c(pos_weight).data_ptr(), _c(label).data_ptr(), P,
                    wy.data_ptr(), native.stream(idx.device))
        return wy
    rows = idx.long()
    if pos_weight is not None:
        wv = pos_weight.float()
    else:
        wv = wcnt[rows].float() if wcnt is not None else torch.ones(rows.shape[0], dtype=torch.float32,
                                                                    device=idx.device)
    return torch.stack([wv, label[rows].float()], 1).contiguous()


def rf_hist(bins: torch.Tensor, idx: torch.Tensor, label: torch.Tensor, wcnt: Optional[torch.Tensor],
            items: torch.Tensor, node_feats: torch.Tensor, nodes: int, B: int, S: int,
            regression: bool, pos_weight: Optional[torch.Tensor] = None, fb: Optional[int] = None,
            yscale: Optional[float] = None, exclusive: Optional[Dict[str, torch.Tensor]] = None,
            bins_il: Optional[torch.Tensor] = None, wide: bool = False, rec_bytes: int = 32,
            bins_rm: Optional[torch.Tensor] = None,
            packed_scale: Optional[float] = None, out: Optional[torch.Tensor] = None,
            wy: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-(node, feature slot, bin) statistics: uint32 class counts or fp64 (count, sum[, sumsq]).
    Weights: per row (``wcnt``, indexed by row id) or per position of ``idx`` (``pos_weight``).
    ``items`` rows are (node, row_begin, row_end, feature_chunk) with chunks of ``fb`` features
    (default ``rf_hist_fb(B, S, regression)``). ``bins_il``: the record layout of ``bins``
    (``rf_interleave``) for the device kernel to gather from (same results); ``wide``: the
    1024-thread record-layout kernel with chunks of ``fb = rf_hist_fb_wide(...)`` features, on
    records of ``rec_bytes`` (the value ``bins_il`` was built with). ``packed_scale`` (wide
    regression, not deterministic): one u64 LDS cell per (feature, bin) holding the weighted count
    and the sum of w * rint(y * packed_scale), packed_scale = 2^22 / max|y| (``rf_pack_scale``);
    the caller keeps the weights of one item <= 2^20. ``out``: a zeroed / partly accumulated
    histogram the items ADD into (no single-chunk stores: ``exclusive`` must be None) — a histogram
    built over several launches, e.g. one per streamed row chunk; ``wy``: the (weight, label) pairs
    in ``idx`` order from an earlier call (``rf_hist_wy``)."""
    if out is not None and (exclusive is not None or (regression and deterministic())):
        raise ValueError("rf_hist(out=): accumulating launches need atomics (no exclusive / fixed-point mode)")
    if wide and fb is None:
        fb = rf_hist_fb_wide(B, S, regression)
    fb = rf_hist_fb(B, S, regression) if fb is None else int(fb)
    n, m = bins.shape
    nf = node_feats.shape[1]
    dev = bins.device
    hdt = torch.float64 if regression else torch.int32
    if out is not None:
        hist = out
        if items.shape[0] == 0:
            return hist
    elif not bins.is_cuda or items.shape[0] == 0:
        hist = zeros((nodes, nf, B, S), dtype=hdt, device=dev)
        if items.shape[0] == 0:
            return hist
    elif exclusive is not None:
        # nodes served by ONE row chunk are written with plain stores by their items (flag bit 30 of
        # item.w); only the multi-chunk nodes accumulate with atomics and need zeroing
        hist = torch.empty((nodes, nf, B, S), dtype=hdt, device=dev)
        if exclusive["multi_nodes"].numel():
            hist.index_fill_(0, exclusive["multi_nodes"], 0)
    else:
        hist = zeros((nodes, nf, B, S), dtype=hdt, device=dev)
    if not bins.is_cuda:
        it = items.cpu().numpy()
        for node, rb, re, fc in it:
            fc = int(fc) & 0x3FFFFFFF
            rows = idx[rb:re].long()
            if pos_weight is not None:
                w = pos_weight[rb:re].double()
            else:
                w = wcnt[rows].double() if wcnt is not None else torch.ones(len(rows), dtype=torch.float64)
            y = label[rows]
            for j in range(fc * fb, min(nf, (fc + 1) * fb)):
                f = int(node_feats[node, j])
                b = bins[f, rows].long()
                if regression:
                    hist[node, j, :, 0].index_add_(0, b, w)
                    hist[node, j, :, 1].index_add_(0, b, w * y.double())
                    if S > 2:
                        hist[node, j, :, 2].index_add_(0, b, w * y.double() ** 2)
                else:
                    flat = b * S + y.long()
                    hist[node, j].view(-1).index_add_(0, flat, w.to(torch.int32))
        return hist
    if wy is None:
        wy = rf_hist_wy(idx, label, wcnt, pos_weight)
    if regression:
        if S != 2:
            raise ValueError("device regression histograms carry (count, sum): S must be 2")
        if yscale is None:  # callers growing many levels pass rf_yscale(y) once per fit (no host sync here)
            yscale = rf_yscale(wy[:, 1], float(wy[:, 0].sum().item()))
    else:
        yscale = 1.0
    st = native.stream(dev)
    if wide:
        if bins_il is None:
            raise ValueError("the wide histogram kernel reads the record layout: pass bins_il")
        fixed = bool(regression and deterministic())
        mode = 1 if fixed else (2 if (regression and packed_scale is not None) else 0)
        ys = float(packed_scale) if mode == 2 else float(yscale)
        native.call("srml_rf_hist_wide", bins_il.data_ptr(), m, idx.data_ptr(), wy.data_ptr(), _c(items).data_ptr(),
                    int(items.shape[0]), _c(node_feats).data_ptr(), nf, B, S, int(regression), ys, fb,
                    mode, int(rec_bytes), hist.data_ptr() if not regression else None,
                    hist.data_ptr() if regression else None, st)
        if fixed:
            native.call("srml_rf_hist_fixed_finish", hist.data_ptr(), hist.numel(), float(yscale), st)
        return hist
    if regression and deterministic():
        # exact i64 fixed-point cross-chunk folds, converted in place: bit-reproducible histograms
        src = bins_il if bins_il is not None else bins
        native.call("srml_rf_hist_fixed", src.data_ptr(), m, idx.data_ptr(), wy.data_ptr(), _c(items).data_ptr(),
                    int(items.shape[0]), _c(node_feats).data_ptr(), nf, B, float(yscale), fb, hist.data_ptr(),
                    int(bins_il is not None), st)
        native.call("srml_rf_hist_fixed_finish", hist.data_ptr(), hist.numel(), float(yscale), st)
        return hist
    src = bins_il if bins_il is not None else (bins_rm if bins_rm is not None else bins)
    mode = 1 if bins_il is not None else (2 if bins_rm is not None else 0)
    native.call("srml_rf_hist", src.data_ptr(), m if mode != 2 else int(bins_rm.shape[1]), idx.data_ptr(),
                wy.data_ptr(), _c(items).data_ptr(), int(items.shape[0]), _c(node_feats).data_ptr(), nf, B, S,
                int(regression), float(yscale), fb, hist.data_ptr() if not regression else None,
                hist.data_ptr() if regression else None, mode, st)
    return hist


def rf_best_split(hist: torch.Tensor, B: int, S: int, regression: bool, crit: int, min_leaf: float,
                  min_gain: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per node: out (nodes, 6) = {gain, feature_slot, bin, n_left, n_right, impurity}; totals (nodes, S)."""
    nodes, nf = hist.shape[0], hist.shape[1]
    dev = hist.device
    if not hist.is_cuda:
        return _rf_best_split_ref(hist.double(), S, regression, crit, min_leaf, min_gain)
    out = torch.empty((nodes, 6), dtype=torch.float64, device=dev)
    tot = torch.empty((nodes, S), dtype=torch.float64, device=dev)
    native.call("srml_rf_best_split", hist.data_ptr() if not regression else None,
                hist.data_ptr() if regression else None, nodes, nf, B, S, int(regression), int(crit),
                float(min_leaf), float(min_gain), out.data_ptr(), tot.data_ptr(), native.stream(dev))
    return out, tot


def rf_node_split_ok(nf: int, B: int, S: int) -> bool:
    """Whether the fused small-node classification split (``rf_node_split``) takes nf sampled
    features x B bins x S classes (the whole node histogram within 150 KiB of LDS)."""
    return bool(int(native.lib().srml_rf_node_split_ok(int(nf), int(B), int(S))))


def rf_node_split(bins_rm: torch.Tensor, idx: torch.Tensor, wy: torch.Tensor, se: torch.Tensor,
                  node_feats: torch.Tensor, B: int, S: int, crit: int, min_leaf: float,
                  min_gain: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """Classification histogram + split search of small nodes in one kernel (``srml_rf_node_split``,
    the node's histogram never leaves LDS). ``bins_rm``: row-major (m, n) uint8 bins; ``idx`` /
    ``wy``: the level's row ids and (weight, class) pairs (``rf_hist_wy``); ``se``: (nodes, 2)
    int32 [begin, end) positions; ``node_feats``: (nodes, nf) ascending sampled feature ids.
    Returns the ``rf_best_split`` record (nodes, 6) and the winner's left-child class totals
    (nodes, S) (zeros without a split) — equal to ``rf_hist`` + ``rf_best_split`` + the
    left-prefix of the winning histogram."""
    nodes, nf = int(node_feats.shape[0]), int(node_feats.shape[1])
    dev = bins_rm.device
    if se.shape != (nodes, 2) or idx.dtype != torch.int32 or wy.dtype != torch.float32 or wy.shape[-1] != 2:
        raise ValueError("rf_node_split: se (nodes, 2) int32, idx int32, wy (P, 2) float32")
    if wy.shape[0] != idx.shape[0]:
        raise ValueError("rf_node_split: wy holds %d positions, idx %d" % (wy.shape[0], idx.shape[0]))
    if not rf_node_split_ok(nf, B, S):
        raise ValueError("rf_node_split: nf=%d B=%d S=%d exceeds the LDS histogram" % (nf, B, S))
    out = torch.empty((nodes, 6), dtype=torch.float64, device=dev)
    left = torch.empty((nodes, S), dtype=torch.float64, device=dev)
    rm = _c(bins_rm)
    native.call("srml_rf_node_split", rm.data_ptr(), int(rm.shape[1]), _c(idx).data_ptr(), _c(wy).data_ptr(),
                _c(se.to(torch.int32)).data_ptr(), nodes, _c(node_feats.to(torch.int32)).data_ptr(), nf, int(B),
                int(S), int(crit), float(min_leaf), float(min_gain), out.data_ptr(), left.data_ptr(),
                native.stream(dev))
    return out, left


def _impurity_ref(s: torch.Tensor, crit: int) -> torch.Tensor:
    if crit == 2:
        n = s[..., 0]
        mean = s[..., 1] / n.clamp_min(1e-300)
        return torch.where(n > 0, (s[..., 2] / n.clamp_min(1e-300) - mean * mean).clamp_min(0), torch.zeros_like(n))
    n = s.sum(-1)
    p = s / n.clamp_min(1e-300).unsqueeze(-1)
    if crit == 0:
        return torch.where(n > 0, 1 - (p * p).sum(-1), torch.zeros_like(n))
    ent = -(torch.where(p > 0, p * torch.log2(p.clamp_min(1e-300)), torch.zeros_like(p))).sum(-1)
    return torch.where(n > 0, ent, torch.zeros_like(n))


def _rf_best_split_ref(hist: torch.Tensor, S: int, regression: bool, crit: int, min_leaf: float,
                       min_gain: float) -> Tuple[torch.Tensor, torch.Tensor]:
    nodes, nf, B, _ = hist.shape
    tot = hist[:, 0].sum(1)  # (nodes, S)
    ntot = tot[:, 0] if regression else tot.sum(-1)
    pimp = _impurity_ref(tot, crit) if (not regression or S > 2) else torch.zeros_like(ntot)
    left = hist.cumsum(2)[:, :, : B - 1]  # (nodes, nf, B-1, S)
    right = tot[:, None, None, :] - left
    nl = left[..., 0] if regression else left.sum(-1)
    nr = ntot[:, None, None] - nl
    if regression:
        # variance reduction from (count, sum) only: (sL^2/nL + sR^2/nR - s^2/n) / n
        nt = ntot[:, None, None].clamp_min(1e-300)
        sl, sr = left[..., 1], right[..., 1]
        gain = (sl * sl / nl.clamp_min(1e-300) + sr * sr / nr.clamp_min(1e-300)
                - (tot[:, 1] ** 2)[:, None, None] / nt) / nt
        if S < 3:
            pimp = torch.zeros_like(ntot)
    else:
        gain = pimp[:, None, None] - nl / ntot[:, None, None].clamp_min(1e-300) * _impurity_ref(left, crit) \
            - nr / ntot[:, None, None].clamp_min(1e-300) * _impurity_ref(right, crit)
    valid = (nl >= min_leaf) & (nr >= min_leaf) & (nl > 0) & (nr > 0)
    gain = torch.where(valid, gain, torch.full_like(gain, -1.0))
    out = torch.empty((nodes, 6), dtype=torch.float64)
    flat = gain.reshape(nodes, -1)
    best, arg = flat.max(1)  # first max -> lowest (feature, bin)
    f = arg // (B - 1)
    b = arg % (B - 1)
    ok = (best > 1e-15) & ((best > min_gain) | (min_gain < 0))
    out[:, 0] = torch.where(ok, best, torch.full_like(best, -1.0))
    out[:, 1] = torch.where(ok, f.double(), torch.full_like(best, -1.0))
    out[:, 2] = torch.where(ok, b.double(), torch.full_like(best, -1.0))
    nlw = nl.reshape(nodes, -1).gather(1, arg.view(-1, 1)).view(-1)
    out[:, 3] = torch.where(ok, nlw, torch.zeros_like(nlw))
    out[:, 4] = torch.where(ok, ntot - nlw, torch.zeros_like(nlw))
    out[:, 5] = pimp
    return out, tot


def rf_route(bins: torch.Tensor, idx: torch.Tensor, seg_node: torch.Tensor, node_feature: torch.Tensor,
             node_bin: torch.Tensor, child_base: torch.Tensor) -> torch.Tensor:
    n, m = bins.shape
    total = idx.shape[0]
    if not bins.is_cuda:
        f = node_feature[seg_node.long()]
        leaf = f < 0
        fb = bins[f.clamp_min(0).long(), idx.long()].int()
        right = (fb > node_bin[seg_node.long()]).int()
        keys = child_base[seg_node.long()] + right
        return torch.where(leaf, torch.full_like(keys, 2**31 - 1), keys)
    keys = torch.empty(total, dtype=torch.int32, device=bins.device)
    native.call("srml_rf_route", bins.data_ptr(), m, idx.data_ptr(), seg_node.data_ptr(), total,
                node_feature.data_ptr(), node_bin.data_ptr(), child_base.data_ptr(), keys.data_ptr(),
                native.stream(bins.device))
    return keys


def rf_route_segments(bins: torch.Tensor, idx: torch.Tensor, bounds: torch.Tensor, node_feature: torch.Tensor,
                      node_bin: torch.Tensor, child_base: torch.Tensor) -> torch.Tensor:
    """Child key of every position: segment s = [bounds[s], bounds[s+1]) found by binary search."""
    n, m = bins.shape
    total = idx.shape[0]
    if not bins.is_cuda:
        pos = torch.arange(total, device=bins.device)
        seg = (torch.searchsorted(bounds.long(), pos, right=True) - 1).int()
        return rf_route(bins, idx, seg, node_feature, node_bin, child_base)
    keys = torch.empty(total, dtype=torch.int32, device=bins.device)
    if total:
        native.call("srml_rf_route_segments", bins.data_ptr(), m, idx.data_ptr(), total,
                    _c(bounds.long()).data_ptr(), int(bounds.shape[0] - 1), node_feature.data_ptr(),
                    node_bin.data_ptr(), child_base.data_ptr(), keys.data_ptr(), native.stream(bins.device))
    return keys


def rf_left_totals(hist: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """(C, S) fp64 class totals of every node's left child under its best split (zeros without
    one): the winning feature's histogram (C, nslot, B, S) summed up to the split bin
    (``srml_rf_left_totals``; torch on the host)."""
    C, nslot, B, S = hist.shape
    if hist.is_cuda and hist.dtype in (torch.int32, torch.float64) and hist.is_contiguous():
        left = torch.empty((C, S), dtype=torch.float64, device=hist.device)
        native.call("srml_rf_left_totals", hist.data_ptr(), int(hist.dtype == torch.float64), C, nslot, B, S,
                    _c(out.double()).data_ptr(), left.data_ptr(), native.stream(hist.device))
        return left
    ok = out[:, 1] >= 0
    slot = torch.where(ok, out[:, 1], torch.zeros_like(out[:, 1])).long()
    b = torch.where(ok, out[:, 2], torch.zeros_like(out[:, 2])).long()
    ar = torch.arange(C, device=hist.device)
    left = hist[ar, slot].double().cumsum(1)[ar, b]
    return torch.where(ok.view(-1, 1), left, torch.zeros_like(left))


def rf_gather_feature(feats: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """(C, 1) winning feature ids (``feats[c, out[c, 1]]``, slot clamped at 0) in out's dtype."""
    C = out.shape[0]
    if feats.is_cuda and feats.dtype == torch.int32 and out.dtype == torch.float64 and feats.stride(1) == 1:
        fsel = torch.empty((C, 1), dtype=torch.float64, device=out.device)
        native.call("srml_rf_gather_feature", feats.data_ptr(), feats.stride(0), _c(out).data_ptr(), C,
                    fsel.data_ptr(), native.stream(out.device))
        return fsel
    return feats[:C].gather(1, out[:, 1].clamp_min(0).long().view(-1, 1)).to(out.dtype)


def rf_decide(out: torch.Tensor, fsel: torch.Tensor, cand: torch.Tensor, L: int, left: Optional[torch.Tensor],
              tot: Optional[torch.Tensor]) -> Tuple[torch.Tensor, ...]:
    """One level's split decisions on the device (``srml_rf_decide``): candidate j (segment
    cand[j]) splits iff out[j, 1] >= 0, its children are segments 2 r, 2 r + 1 with r its rank among
    the splitting candidates. Returns (node_feature, node_bin, child_base) (L int32 each: -1 / 0 / 0
    off the splits) and, with ``left`` / ``tot`` (classification), the children's totals (2C, S)
    (left = prefix, right = parent - left; rows past the real children zero)."""
    dev = out.device
    C = out.shape[0]
    st = native.stream(dev)
    node = torch.empty((3, L), dtype=torch.int32, device=dev)
    native.call("srml_memset_async", node[0].data_ptr(), 0xFF, L * 4, st)
    native.call("srml_memset_async", node[1].data_ptr(), 0, 2 * L * 4, st)
    pos = torch.empty(max(C, 1), dtype=torch.int32, device=dev)
    k_d = torch.empty(1, dtype=torch.int64, device=dev)
    tot_n = None
    if left is not None:
        S = int(left.shape[1])
        tot_n = torch.empty((2 * C, S), dtype=torch.float64, device=dev)
    native.call("srml_rf_decide", _c(out).data_ptr(), _c(fsel).data_ptr(), _c(cand).data_ptr(), C, pos.data_ptr(),
                k_d.data_ptr(), node[0].data_ptr(), node[1].data_ptr(), node[2].data_ptr(),
                _c(left).data_ptr() if left is not None else None,
                _c(tot.double()).data_ptr() if left is not None else None,
                int(left.shape[1]) if left is not None else 0, tot_n.data_ptr() if tot_n is not None else None, st)
    return node[0], node[1], node[2], tot_n


def rf_level_pack(bounds: torch.Tensor, tot_n: torch.Tensor, regression: bool, crit: int, out: torch.Tensor,
                  fsel: torch.Tensor) -> torch.Tensor:
    """The level's read-back buffer (``srml_rf_level_pack``, fp64, on the device): [child bounds
    (2C + 1) | per child [leaf value(s) | weight | impurity] (forest._seg_stats) | out (6C) | fsel]."""
    C = out.shape[0]
    S = int(tot_n.shape[1])
    V2 = 3 if regression else S + 2
    hb = torch.empty(2 * C + 1 + 2 * C * V2 + 7 * C, dtype=torch.float64, device=out.device)
    native.call("srml_rf_level_pack", _c(bounds).data_ptr(), C, _c(tot_n).data_ptr(), S, int(bool(regression)),
                int(crit), _c(out).data_ptr(), _c(fsel).data_ptr(), hb.data_ptr(), native.stream(out.device))
    return hb


def seg_lower_bound(idx: torch.Tensor, start: np.ndarray, count: np.ndarray, vals: torch.Tensor) -> np.ndarray:
    """(nseg, nv) int64 host array: for every segment idx[start[j] : start[j] + count[j]] (ascending)
    the global position of the first entry >= vals[c] (one device launch for all segments)."""
    nseg, nv = len(start), int(vals.numel())
    if not idx.is_cuda or idx.dtype != torch.int32:
        return np.stack([torch.searchsorted(idx[int(s0): int(s0) + int(cn)], vals.to(idx.device)).cpu().numpy()
                         + int(s0) for s0, cn in zip(start, count)]).astype(np.int64)
    dev = idx.device
    se = torch.from_numpy(np.stack([np.asarray(start, np.int64), np.asarray(count, np.int64)])).pin_memory().to(
        dev, non_blocking=True)
    out = torch.empty((nseg, nv), dtype=torch.int64, device=dev)
    native.call("srml_seg_lower_bound", idx.data_ptr(), se[0].data_ptr(), se[1].data_ptr(), nseg,
                _c(vals.to(device=dev, dtype=torch.int32)).data_ptr(), nv, out.data_ptr(), native.stream(dev))
    return out.cpu().numpy()


def rf_sample_features(C: int, n: int, nf: int, seed: int, device: torch.device) -> torch.Tensor:
    """(C, nf) int32: per node a uniform random subset of nf of n features, ascending
    (``srml_rf_sample_features``: Floyd's algorithm for sparse subsets, nf <= n / 8, else
    selection sampling; CPU: numpy's own uniform subsets)."""
    seed &= (1 << 64) - 1
    if device.type != "cuda":
        rng = np.random.default_rng(seed)
        return torch.from_numpy(np.sort(np.stack([rng.choice(n, nf, replace=False) for _ in range(C)]), 1)
                                .astype(np.int32)) if C else zeros((0, nf), dtype=torch.int32)
    out = torch.empty((C, nf), dtype=torch.int32, device=device)
    native.call("srml_rf_sample_features", C, n, nf, seed, out.data_ptr(), native.stream(device))
    return out


def _mix64_np(x: np.ndarray) -> np.ndarray:
    x = x + np.uint64(0x9E3779B97F4A7C15)
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def rf_bootstrap(T: int, m: int, rate: float, seed: int, device: torch.device
                 ) -> Tuple[torch.Tensor, torch.Tensor, np.ndarray]:
    """Poisson(rate) bagging of T trees over m rows (Spark's bagging, cuML's bootstrap): (in-bag row
    ids int32, their multiplicities float32 — tree-major, ascending inside a tree —, tree bounds
    int64 [T + 1] on the host). Element i = t m + r draws by inversion from the counter-based
    uniform (splitmix64(seed ^ splitmix64(i + 1)) >> 11) 2^-53, clamped to 255: one count pass, one
    scan, one scatter (``srml_rf_bootstrap``); the CPU path is the same draw in numpy."""
    seed &= (1 << 64) - 1
    N = int(T) * int(m)
    if device.type != "cuda":
        i = np.arange(N, dtype=np.uint64)
        with np.errstate(over="ignore"):
            u = (_mix64_np(np.uint64(seed) ^ _mix64_np(i + np.uint64(1))) >> np.uint64(11)).astype(np.float64) \
                * 2.0 ** -53
        k = np.zeros(N, dtype=np.int64)
        p = np.full(N, math.exp(-rate))
        F = p.copy()
        live = u > F
        while live.any():
            k[live] += 1
            p[live] *= rate / k[live]
            F[live] += p[live]
            live &= (u > F) & (k < 255)
        nz = np.nonzero(k)[0]
        bounds = np.searchsorted(nz, np.arange(T + 1, dtype=np.int64) * m).astype(np.int64)
        return (torch.from_numpy((nz % m).astype(np.int32)), torch.from_numpy(k[nz].astype(np.float32)), bounds)
    idx = torch.empty(N, dtype=torch.int32, device=device)
    w = torch.empty(N, dtype=torch.float32, device=device)
    tb = torch.empty(T + 1, dtype=torch.int64, device=device)
    ws = torch.empty(int(native.lib().srml_rf_bootstrap_ws(T, m)) + 1, dtype=torch.int64, device=device)
    native.call("srml_rf_bootstrap", T, m, float(rate), seed, idx.data_ptr(), w.data_ptr(), tb.data_ptr(),
                ws.data_ptr(), native.stream(device))
    bounds = tb.cpu().numpy()
    tot = int(bounds[-1])
    return idx[:tot], w[:tot], bounds


def rf_partition(keys: torch.Tensor, bounds: torch.Tensor, node_feature: torch.Tensor, child_base: torch.Tensor,
                 k: int, idx: torch.Tensor, wpos: torch.Tensor, kept: Optional[int] = None, trim: bool = True
                 ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Stable re-partition of (idx, wpos) into the 2k child segments of the k split parents
    (child keys from ``rf_route_segments``; other positions leave the tree): (idx, wpos, bounds
    of the 2k children). Device: prefix-count kernels + one scatter (``srml_rf_partition``).
    ``kept``: the caller's count of positions in split parents (their rows all stay), which
    spares reading it back from the device. ``trim=False`` (device): the position arrays keep their
    full length (the kept prefix is ``bounds[-1]``; the caller slices after its own read of bounds).
    ``k`` may be an upper bound on the splits: children past the real ones are empty segments."""
    total = int(keys.shape[0])
    if not keys.is_cuda:
        keys_sorted, perm = torch.sort(keys, stable=True)
        nb = torch.searchsorted(keys_sorted.contiguous(), torch.arange(2 * k + 1, dtype=keys_sorted.dtype))
        kept = int(nb[-1].item())
        perm = perm[:kept]
        return idx[perm].contiguous(), wpos[perm].contiguous(), nb.to(torch.int64)
    dev = keys.device
    nseg = int(bounds.shape[0]) - 1
    ws = torch.empty(int(native.lib().srml_rf_partition_ws(total, k)), dtype=torch.int64, device=dev)
    idx_out = torch.empty(max(total, 1), dtype=torch.int32, device=dev)
    w_out = torch.empty(max(total, 1), dtype=torch.float32, device=dev)
    nb = torch.empty(2 * k + 1, dtype=torch.int64, device=dev)
    native.call("srml_rf_partition", keys.data_ptr(), total, _c(bounds.long()).data_ptr(), nseg,
                _c(node_feature.int()).data_ptr(), _c(child_base.int()).data_ptr(), int(k), _c(idx).data_ptr(),
                _c(wpos.float()).data_ptr(), idx_out.data_ptr(), w_out.data_ptr(), nb.data_ptr(), ws.data_ptr(),
                native.stream(dev))
    if not trim:
        return idx_out, w_out, nb
    if kept is None:
        kept = int(nb[-1].item())
    return idx_out[:kept], w_out[:kept], nb


def rf_node_stats(idx: torch.Tensor, wpos: torch.Tensor, label: torch.Tensor, bounds: torch.Tensor, S: int,
                  regression: bool) -> torch.Tensor:
    """Per segment [bounds[s], bounds[s+1]): regression (sum w, sum w y, sum w y^2) or per-class sum w
    (nseg, 3 | S) fp64."""
    nseg = bounds.shape[0] - 1
    K = 3 if regression else S
    dev = idx.device
    if not idx.is_cuda:
        wr = wpos.double()
        yr = label[idx.long()].double()
        if regression:
            vals = torch.stack([wr, wr * yr, wr * yr * yr], 0)
        else:
            vals = torch.stack([wr * (yr.long() == c) for c in range(S)], 0)
        cs = torch.cat([zeros((K, 1), dtype=torch.float64), vals.cumsum(1)], 1)
        b = bounds.long()
        return (cs[:, b[1:]] - cs[:, b[:-1]]).T.contiguous()
    if deterministic():  # one block per segment, fixed-order reduction, no atomics
        out = torch.empty((nseg, K), dtype=torch.float64, device=dev)
        native.call("srml_rf_node_stats_det", idx.data_ptr(), _c(wpos.float()).data_ptr(),
                    _c(label.float()).data_ptr(), _c(bounds.long()).data_ptr(), nseg, int(S), int(regression),
                    out.data_ptr(), native.stream(dev))
        return out
    out = zeros((nseg, K), dtype=torch.float64, device=dev)
    native.call("srml_rf_node_stats", idx.data_ptr(), _c(wpos.float()).data_ptr(), _c(label.float()).data_ptr(),
                int(idx.shape[0]), _c(bounds.long()).data_ptr(), nseg, int(S), int(regression), out.data_ptr(),
                native.stream(dev))
    return out


def rf_predict(X: torch.Tensor, roots: torch.Tensor, feature: torch.Tensor, threshold: torch.Tensor,
               left: torch.Tensor, right: torch.Tensor, value_off: torch.Tensor, values: torch.Tensor, S: int,
               want_leaves: bool = False, nodes: Optional[torch.Tensor] = None
               ) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Sum over trees of leaf value vectors (rows, S) (+ per-tree leaf ids). Device with packed
    16-B ``nodes`` (``pack_forest``): wave-per-row kernel, trees over the lanes."""
    m = X.shape[0]
    T = roots.shape[0]
    if not X.is_cuda or X.dtype != torch.float32 or S > 32:
        Xf = X.float()
        out = zeros((m, S), dtype=torch.float32, device=X.device)
        leaves = torch.empty((m, T), dtype=torch.int32, device=X.device) if want_leaves else None
        rows = torch.arange(m, device=X.device)
        for t in range(T):
            node = torch.full((m,), int(roots[t]), dtype=torch.long, device=X.device)
            while True:
                f = feature[node]
                active = f >= 0
                if not bool(active.any()):
                    break
                xv = Xf[rows, f.clamp_min(0).long()]
                go_left = xv <= threshold[node]
                nxt = torch.where(go_left, left[node].long(), right[node].long())
                node = torch.where(active, nxt, node)
            if leaves is not None:
                leaves[:, t] = (node - int(roots[t])).int()
            off = value_off[node].long()
            out += values[off.view(-1, 1) + torch.arange(S, device=X.device).view(1, -1)]
        return out, leaves
    X = X if X.stride(1) == 1 else X.contiguous()
    out = torch.empty((m, S), dtype=torch.float32, device=X.device)
    leaves = torch.empty((m, T), dtype=torch.int32, device=X.device) if want_leaves else None
    if nodes is not None and nodes.is_cuda:
        native.call("srml_rf_predict_nodes2", X.data_ptr(), m, X.stride(0), X.shape[1], _c(nodes).data_ptr(),
                    roots.data_ptr(), T,
                    values.data_ptr(), S, out.data_ptr(), leaves.data_ptr() if leaves is not None else None,
                    native.stream(X.device))
        return out, leaves
    native.call("srml_rf_predict", X.data_ptr(), m, X.stride(0), roots.data_ptr(), T, feature.data_ptr(),
                threshold.data_ptr(), left.data_ptr(), right.data_ptr(), value_off.data_ptr(), values.data_ptr(), S,
                out.data_ptr(), leaves.data_ptr() if leaves is not None else None, native.stream(X.device))
    return out, leaves


# ------------------------------------------------------------------------------------------
# Nearest-neighbour search
# ------------------------------------------------------------------------------------------
# all-points IVF kNN candidates on fp16 MFMAs with query-list centring (ops.knn_lists centroids=)
KNN_LISTS_F16 = os.environ.get("SRML_KNN_LISTS_F16", "1") != "0"
KNN_KMAX = 64          # register/LDS insertion-list kernel (srml_knn_f32)
TOPK_KMAX = 16384      # distance-chunk + radix-select path (srml_knn_dist_f32 + srml_topk_rows_f32)
_TOPK_SLICE = 65536    # columns per select block
_KNN_DIST_BYTES = 1 << 30  # distance chunk budget


def topk_rows(vals: torch.Tensor, k: int, ids: Optional[torch.Tensor] = None, id_base: int = 0,
              slice_len: Optional[int] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """k smallest values of every row (ascending, ties -> lower column) and their ids
    (``ids[r, c]``, or ``id_base + c``). Rows longer than ``slice_len`` are selected per slice and
    merged. Device: ``srml_topk_rows_f32``; host: torch.topk."""
    rows, L = vals.shape
    if not vals.is_cuda:
        kk = min(k, L)
        v, j = torch.sort(vals.float(), dim=1, stable=True)  # ties keep the lower column
        v, j = v[:, :kk], j[:, :kk]
        outv = torch.full((rows, k), float("inf"), dtype=torch.float32, device=vals.device)
        outi = torch.full((rows, k), -1, dtype=torch.int64, device=vals.device)
        outv[:, :kk] = v
        outi[:, :kk] = ids.gather(1, j) if ids is not None else j + id_base
        return outv, outi
    if k > TOPK_KMAX:
        raise ValueError("topk_rows: k=%d > %d" % (k, TOPK_KMAX))
    if vals.dtype != torch.float32 or vals.stride(1) != 1:
        vals = vals.float().contiguous()
    S = int(slice_len or _TOPK_SLICE)
    S = max(S, k)
    nsl = (L + S - 1) // S
    ids_c = _c(ids.long()) if ids is not None else None
    st = native.stream(vals.device)
    if nsl == 1:
        outv = torch.empty((rows, k), dtype=torch.float32, device=vals.device)
        outi = torch.empty((rows, k), dtype=torch.int64, device=vals.device)
        native.call("srml_topk_rows_f32", vals.data_ptr(), rows, vals.stride(0), S, L,
                    ids_c.data_ptr() if ids_c is not None else None, ids_c.stride(0) if ids_c is not None else 0,
                    int(id_base), k, outv.data_ptr(), outi.data_ptr(), k, 0, st)
        return outv, outi
    pv = torch.empty((rows, nsl * k), dtype=torch.float32, device=vals.device)
    pi = torch.empty((rows, nsl * k), dtype=torch.int64, device=vals.device)
    native.call("srml_topk_rows_f32", vals.data_ptr(), rows, vals.stride(0), S, L,
                ids_c.data_ptr() if ids_c is not None else None, ids_c.stride(0) if ids_c is not None else 0,
                int(id_base), k, pv.data_ptr(), pi.data_ptr(), nsl * k, k, st)
    return topk_rows(pv, k, ids=pi, slice_len=nsl * k)  # one merge block per row


def knn(Q: torch.Tensor, I: torch.Tensor, k: int, inorm: Optional[torch.Tensor] = None,
        qnorm: Optional[torch.Tensor] = None, id_offset: int = 0) -> Tuple[torch.Tensor, torch.Tensor]:
    """Exact k nearest items of every query: (squared L2 distances fp32 [mq, k], item ids int64 [mq, k]).
    Device: k <= 64 -> fused MFMA tiles + LDS insertion lists (``srml_knn_f32``); 64 < k <= 1024 ->
    bounded distance chunks on the MFMA tile + radix select (``_knn_large_k``)."""
    mq, n = Q.shape
    mi = I.shape[0]
    kk = min(k, mi)
    if Q.is_cuda and Q.dtype == torch.float32 and k > TOPK_KMAX:
        raise ValueError("knn: k=%d > %d" % (k, TOPK_KMAX))
    if Q.is_cuda and Q.dtype == torch.float32 and KNN_KMAX < k:
        return _knn_large_k(Q, I, kk, inorm, qnorm, id_offset)
    if inorm is None:
        inorm = row_sqnorm(I)
    if qnorm is None:
        qnorm = row_sqnorm(Q)
    if not Q.is_cuda or Q.dtype != torch.float32 or k > KNN_KMAX:
        Qf, If = Q.float(), I.float()
        outs_d, outs_i = [], []
        bs = max(1, (1 << 25) // max(mi, 1))
        for s in range(0, mq, bs):
            d = (qnorm[s: s + bs].float().view(-1, 1) + inorm.float().view(1, -1) - 2.0 * (Qf[s: s + bs] @ If.T))
            v, i = torch.topk(d, kk, dim=1, largest=False)
            outs_d.append(v.clamp_min(0))
            outs_i.append(i + id_offset)
        return torch.cat(outs_d), torch.cat(outs_i)
    Q = _c(Q)
    I = _c(I.to(torch.float32))
    inorm = _c(inorm.float())
    # enough item slices that the grid covers the chip for small query sets
    qblocks = (mq + 127) // 128
    slices = max(1, min((mi + 4095) // 4096, (1024 + qblocks - 1) // qblocks))
    od = torch.empty((mq, slices, kk), dtype=torch.float32, device=Q.device)
    oi = torch.empty((mq, slices, kk), dtype=torch.int64, device=Q.device)
    native.call("srml_knn_f32", Q.data_ptr(), mq, n, Q.stride(0), I.data_ptr(), mi, I.stride(0), inorm.data_ptr(), kk,
                slices, od.data_ptr(), oi.data_ptr(), int(id_offset), native.stream(Q.device))
    od = od.view(mq, slices * kk)
    oi = oi.view(mq, slices * kk)
    if slices > 1:
        od, oi = topk_rows(od, kk, ids=oi)
    return (od + qnorm.float().view(-1, 1)).clamp_min(0), oi


def _knn_large_k(Q: torch.Tensor, I: torch.Tensor, k: int, inorm: Optional[torch.Tensor],
                 qnorm: Optional[torch.Tensor], id_offset: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """64 < k <= 1024: per (query chunk, item chunk) the partial distances ||i||^2 - 2 q.i are
    materialised (<= 1 GB) by the MFMA tile kernel, selected per 64k-column slice by the radix-
    select kernel, and the per-chunk lists merged by the same kernel with ids."""
    mq, n = Q.shape
    mi = I.shape[0]
    Q = _c(Q)
    I = _c(I.to(torch.float32))
    inorm = _c(row_sqnorm(I) if inorm is None else inorm.float())
    qnorm = row_sqnorm(Q) if qnorm is None else qnorm.float()
    st = native.stream(Q.device)
    Lc = min(mi, 16 * _TOPK_SLICE)
    R = max(128, min(4096, (_KNN_DIST_BYTES // (Lc * 4)) // 128 * 128))
    nchunks = (mi + Lc - 1) // Lc
    outv = torch.empty((mq, k), dtype=torch.float32, device=Q.device)
    outi = torch.empty((mq, k), dtype=torch.int64, device=Q.device)
    D = torch.empty((min(R, mq), Lc), dtype=torch.float32, device=Q.device)
    for q0 in range(0, mq, R):
        r = min(R, mq - q0)
        parts_v, parts_i = [], []
        for c in range(nchunks):
            i0 = c * Lc
            L = min(Lc, mi - i0)
            native.call("srml_knn_dist_f32", Q[q0:].data_ptr(), r, n, Q.stride(0), I[i0:].data_ptr(), L, I.stride(0),
                        inorm[i0:].data_ptr(), D.data_ptr(), Lc, st)
            v, i = topk_rows(D[:r, :L], k, id_base=i0 + int(id_offset))
            parts_v.append(v)
            parts_i.append(i)
        if nchunks > 1:
            v, i = topk_rows(torch.cat(parts_v, 1), k, ids=torch.cat(parts_i, 1))
        else:
            v, i = parts_v[0], parts_i[0]
        outv[q0: q0 + r] = (v + qnorm[q0: q0 + r].view(-1, 1)).clamp_min(0)
        outi[q0: q0 + r] = i
    return outv, outi


_IVF_CAND_BYTES = 1 << 30  # candidate matrix budget of the large-k IVF paths (distances + ids)


def _ivf_large_k(Q: torch.Tensor, nq: int, probes: torch.Tensor, list_off: torch.Tensor, items: torch.Tensor,
                 inorm: torch.Tensor, ids: Optional[torch.Tensor], k: int, qlist: Optional[torch.Tensor] = None
                 ) -> Tuple[torch.Tensor, torch.Tensor]:
    """64 < k <= 1024 over IVF lists on the device: every (query, probe) writes its list's partial
    distances ||i||^2 - 2 q.i (+ ids / list positions) into the query's candidate row
    (``srml_ivf_candidates_f32``), then the radix-select kernel keeps k per row (ids carried).
    Query chunks bound the candidate matrix to ``_IVF_CAND_BYTES``. Padding: +inf / -1."""
    dev = Q.device
    n = Q.shape[1]
    st = native.stream(dev)
    pr = _c(probes.int())
    lo = _c(list_off.long())
    ql = _c(qlist.int()) if qlist is not None else None
    nprobe = int(pr.shape[1])
    cmax = zeros(1, dtype=torch.int64, device=dev)
    native.call("srml_ivf_candidate_max", pr.data_ptr(), nprobe, ql.data_ptr() if ql is not None else None, nq,
                lo.data_ptr(), cmax.data_ptr(), st)
    L = int(cmax.item())
    od = torch.full((nq, k), float("inf"), dtype=torch.float32, device=dev)
    oi = torch.full((nq, k), -1, dtype=torch.int64, device=dev)
    if L == 0 or nq == 0:
        return od, oi
    kk = min(k, L)
    R = max(1, min(nq, _IVF_CAND_BYTES // (L * 12)))
    D = torch.empty((R, L), dtype=torch.float32, device=dev)
    DI = torch.empty((R, L), dtype=torch.int64, device=dev)
    Qc, Ic = _c(Q.float()), _c(items.float())
    idc = _c(ids.long()) if ids is not None else None
    inc = _c(inorm.float())
    for q0 in range(0, nq, R):
        r = min(R, nq - q0)
        native.call("srml_ivf_candidates_f32", Qc.data_ptr(), q0, r, n, Qc.stride(0), pr.data_ptr(), nprobe,
                    ql.data_ptr() if ql is not None else None, lo.data_ptr(), Ic.data_ptr(), Ic.stride(0),
                    inc.data_ptr(), idc.data_ptr() if idc is not None else None, D.data_ptr(), DI.data_ptr(), L, st)
        v, i = topk_rows(D[:r], kk, ids=DI[:r])
        od[q0: q0 + r, :kk] = v
        oi[q0: q0 + r, :kk] = i
    return od, oi


def ivf_search(Q: torch.Tensor, probes: torch.Tensor, list_off: torch.Tensor, items: torch.Tensor,
               inorm: torch.Tensor, ids: torch.Tensor, k: int, qnorm: Optional[torch.Tensor] = None
               ) -> Tuple[torch.Tensor, torch.Tensor]:
    """IVF-Flat scan of each query's probed lists: (squared L2 [nq, k], ids int64 [nq, k])."""
    nq, n = Q.shape
    if qnorm is None:
        qnorm = row_sqnorm(Q)
    if Q.is_cuda and Q.dtype == torch.float32 and k > TOPK_KMAX:
        raise ValueError("ivf_search: k=%d > %d" % (k, TOPK_KMAX))
    if Q.is_cuda and Q.dtype == torch.float32 and KNN_KMAX < k:
        od, oi = _ivf_large_k(Q, nq, probes, list_off, items, inorm, ids, k)
        return (od + qnorm.float().view(-1, 1)).clamp_min(0), oi
    if not Q.is_cuda or Q.dtype != torch.float32 or k > KNN_KMAX:
        od = torch.full((nq, k), float("inf"), dtype=torch.float32, device=Q.device)
        oi = torch.full((nq, k), -1, dtype=torch.int64, device=Q.device)
        lo = list_off.cpu().numpy()
        pr = probes.cpu().numpy()
        for q in range(nq):
            rows = [torch.arange(int(lo[l]), int(lo[l + 1]), device=Q.device) for l in pr[q] if l >= 0]
            if not rows:
                continue
            r = torch.cat(rows)
            d = inorm[r].float() - 2.0 * (items[r].float() @ Q[q].float())
            kk = min(k, d.shape[0])
            v, j = torch.topk(d, kk, largest=False)
            od[q, :kk] = v
            oi[q, :kk] = ids[r[j]]
        return (od + qnorm.float().view(-1, 1)).clamp_min(0), oi
    Q = _c(Q)
    od = torch.empty((nq, k), dtype=torch.float32, device=Q.device)
    oi = torch.empty((nq, k), dtype=torch.int64, device=Q.device)
    native.call("srml_ivf_search_f32", Q.data_ptr(), nq, n, Q.stride(0), _c(probes.int()).data_ptr(),
                int(probes.shape[1]), _c(list_off.long()).data_ptr(), _c(items).data_ptr(), items.stride(0),
                _c(inorm.float()).data_ptr(), _c(ids.long()).data_ptr(), k, od.data_ptr(), oi.data_ptr(),
                native.stream(Q.device))
    return (od + qnorm.float().view(-1, 1)).clamp_min(0), oi


def knn_lists_f16_ok(X: torch.Tensor, k: int, centroids: Optional[torch.Tensor]) -> bool:
    """The centred fp16 candidate kernel applies (n <= 128, n % 4 == 0, k <= 32, fp32 rows)."""
    return (KNN_LISTS_F16 and centroids is not None and X.is_cuda and X.dtype == torch.float32
            and centroids.dtype == torch.float32 and X.dim() == 2 and 1 <= X.shape[1] <= 128
            and X.shape[1] % 4 == 0 and 1 <= k <= 32 and X.stride(1) == 1 and X.stride(0) % 4 == 0
            and X.data_ptr() % 16 == 0 and centroids.shape[0] >= 1)


def knn_lists(X: torch.Tensor, xnorm: torch.Tensor, list_off: torch.Tensor, probes: torch.Tensor,
              tile_q0: torch.Tensor, tile_list: torch.Tensor, k: int,
              centroids: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-points kNN over IVF lists (rows of ``X`` sorted by list, ``list_off`` nlist+1 offsets).

    Every query tile (``tile_q0[i]``: first row of <= 128 rows of list ``tile_list[i]``) is
    compared with the items of the lists ``probes[tile_list[i]]``. Returns (N x k partial
    distances ||i||^2 - 2 q.i fp32, N x k item positions int32, ascending); rows outside the
    given tiles are +inf / -1.

    With ``centroids`` (nlist x n, the lists' centres) and ``knn_lists_f16_ok``, the search runs
    on fp16 MFMAs with rows centred on the query's list centre (knn_graph.hip): the returned
    distances are then centred fp16 ranking keys, and the caller re-ranks the candidates exactly.
    """
    N, n = X.shape
    nprobe = int(probes.shape[1])
    ntiles = int(tile_q0.shape[0])
    od = torch.full((N, k), float("inf"), dtype=torch.float32, device=X.device)
    oi = torch.full((N, k), -1, dtype=torch.int32, device=X.device)
    if ntiles == 0:
        return od, oi
    if tile_list.shape[0] != ntiles or list_off.shape[0] != probes.shape[0] + 1:
        raise ValueError("knn_lists: inconsistent tile / list descriptors")
    if X.is_cuda and X.dtype == torch.float32 and k > TOPK_KMAX:
        raise ValueError("knn_lists: k=%d > %d" % (k, TOPK_KMAX))
    if X.is_cuda and X.dtype == torch.float32 and KNN_KMAX < k:
        # the given tiles cover one contiguous row range (a rank's slice of the tile list); each of
        # those rows probes its own list's probe set
        lo = _c(list_off.long())
        last = int(tile_list[-1].item())
        r0 = int(tile_q0[0].item())
        r1 = min(int(tile_q0[-1].item()) + 128, int(lo[last + 1].item()))
        qlist = torch.empty(N, dtype=torch.int32, device=X.device)
        native.call("srml_row_list", lo.data_ptr(), int(probes.shape[0]), N, qlist.data_ptr(), native.stream(X.device))
        d, pos = _ivf_large_k(X[r0:r1], r1 - r0, probes, lo, X, xnorm, None, k, qlist=qlist[r0:r1])
        od[r0:r1] = d
        oi[r0:r1] = pos.int()
        return od, oi
    if not X.is_cuda or X.dtype != torch.float32 or k > KNN_KMAX:
        lo = list_off.cpu().numpy()
        pr = probes.cpu().numpy()
        tq = tile_q0.cpu().numpy()
        tl = tile_list.cpu().numpy()
        for q0, c in zip(tq, tl):
            q1 = min(int(q0) + 128, int(lo[c + 1]))
            cand = [torch.arange(int(lo[l]), int(lo[l + 1]), device=X.device) for l in pr[c] if l >= 0]
            if not cand:
                continue
            r = torch.cat(cand)
            d = xnorm[r].float().view(1, -1) - 2.0 * (X[int(q0):q1].float() @ X[r].float().T)
            kk = min(k, d.shape[1])
            v, j = torch.topk(d, kk, dim=1, largest=False)
            od[int(q0):q1, :kk] = v
            oi[int(q0):q1, :kk] = r[j].int()
        return od, oi
    if int(list_off[-1]) != N:
        raise ValueError("knn_lists: list offsets do not cover the %d rows" % N)
    if knn_lists_f16_ok(X, k, centroids) and nprobe <= 128:
        Cc = _c(centroids)
        if Cc.shape != (probes.shape[0], n):
            raise ValueError("knn_lists: centroids must be nlist x n")
        native.call("srml_knn_lists_f16c", X.data_ptr(), n, X.stride(0), Cc.data_ptr(), _c(list_off.long()).data_ptr(),
                    _c(probes.int()).data_ptr(), nprobe, _c(tile_q0.long()).data_ptr(), _c(tile_list.int()).data_ptr(),
                    ntiles, int(k), od.data_ptr(), oi.data_ptr(), native.stream(X.device))
        return od, oi
    X = _c(X)
    native.call("srml_knn_lists_f32", X.data_ptr(), n, X.stride(0), _c(xnorm.float()).data_ptr(),
                _c(list_off.long()).data_ptr(), _c(probes.int()).data_ptr(), nprobe, _c(tile_q0.long()).data_ptr(),
                _c(tile_list.int()).data_ptr(), ntiles, int(k), od.data_ptr(), oi.data_ptr(), native.stream(X.device))
    return od, oi


def knn_pool_probes(X: torch.Tensor, list_off: torch.Tensor, C: torch.Tensor, pool: torch.Tensor,
                    tile_q0: torch.Tensor, tile_list: torch.Tensor, p: int, r0: int, r1: int,
                    pool_rows: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Per-query IVF probes: the ``p`` lists whose centres are nearest to each row of the given
    query tiles (rows ``r0 .. r1`` of ``X``, sorted by list), chosen among the ``P`` lists of the
    row's own list's pool (``pool``: nlist x P list ids nearest to each list's centre, all valid).
    Returns (r1 - r0, p) int32 list ids, nearest first.

    Device (``knn_lists_f16_ok``): the pool centres are laid out as P-row virtual lists after X's
    rows (``pool_rows``: a (N + nlist P, n) buffer whose first N rows are X, or None to build one)
    and the fp16 centred list kernel ranks them, so the rows need no gathered copy. Host: exact
    fp32 distances."""
    N, n = X.shape
    nlist, P = int(pool.shape[0]), int(pool.shape[1])
    p = min(int(p), P)
    out = torch.full((r1 - r0, p), -1, dtype=torch.int32, device=X.device)
    if r1 <= r0 or tile_q0.shape[0] == 0:
        return out
    if not knn_lists_f16_ok(X, p, C):
        lo = list_off.cpu().numpy()
        for q0, c in zip(tile_q0.cpu().tolist(), tile_list.cpu().tolist()):
            q1 = min(q0 + 128, int(lo[c + 1]))
            cand = pool[c].long()
            d = torch.cdist(X[q0:q1].float(), C[cand].float())
            j = torch.topk(d, p, dim=1, largest=False).indices
            out[q0 - r0: q1 - r0] = cand[j].int()
        return out
    if pool_rows is None or pool_rows.shape[0] < N + nlist * P:
        pool_rows = torch.empty((N + nlist * P, n), dtype=torch.float32, device=X.device)
        pool_rows[:N] = X
    torch.index_select(C, 0, pool.reshape(-1).long(), out=pool_rows[N: N + nlist * P])
    off_e = torch.cat([list_off.long(), N + P * torch.arange(1, nlist + 1, device=X.device, dtype=torch.int64)])
    probes_e = torch.cat([torch.arange(nlist, 2 * nlist, device=X.device, dtype=torch.int32),
                          torch.full((nlist,), -1, device=X.device, dtype=torch.int32)]).view(-1, 1)
    # the kernel writes row q of the tiles at q * p: the outputs hold rows r0 .. r1 only, so their
    # base pointers are shifted back by r0 rows (no row outside r0 .. r1 is written)
    od = torch.empty((r1 - r0, p), dtype=torch.float32, device=X.device)
    oi = torch.empty((r1 - r0, p), dtype=torch.int32, device=X.device)
    native.call("srml_knn_lists_f16c", pool_rows.data_ptr(), n, pool_rows.stride(0), _c(C).data_ptr(),
                _c(off_e).data_ptr(), _c(probes_e).data_ptr(), 1, _c(tile_q0.long()).data_ptr(),
                _c(tile_list.int()).data_ptr(), int(tile_q0.shape[0]), p, od.data_ptr() - 4 * r0 * p,
                oi.data_ptr() - 4 * r0 * p, native.stream(X.device))
    flat = pool.reshape(-1)
    pos = oi.long() - N
    return torch.where(pos >= 0, flat[pos.clamp_min(0)], torch.full_like(pos, -1)).int()


def center_rows_f16(X: torch.Tensor, C: torch.Tensor, list_off: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """The pair search's pre-centred items (device, ``knn_lists_f16_ok`` rows): (Xh (N, 128) fp16 =
    X[r] - C[list of r], zero padded; ||Xh[r]||^2 fp32 of the rounded values)."""
    N, n = X.shape
    Xh = torch.empty((N, 128), dtype=torch.float16, device=X.device)
    nr = torch.empty(N, dtype=torch.float32, device=X.device)
    native.call("srml_center_rows_f16", X.data_ptr(), n, X.stride(0), _c(C).data_ptr(), _c(list_off.long()).data_ptr(),
                int(list_off.shape[0]) - 1, N, Xh.data_ptr(), nr.data_ptr(), native.stream(X.device))
    return Xh, nr


def knn_pairs(X: torch.Tensor, list_off: torch.Tensor, C: torch.Tensor, pair_off: torch.Tensor,
              qrows: torch.Tensor, qslot: torch.Tensor, tile_q0: torch.Tensor, tile_list: torch.Tensor, k: int,
              nslots: int, thr_row: Optional[torch.Tensor] = None,
              items_f16: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-query probing, inverted: the (row, probed list) pairs sorted by list (``pair_off``:
    nlist + 1 offsets; ``qrows``: the X row of each sorted pair; ``qslot``: its output slot);
    every pair's k nearest items of its list. Returns slot-major (nslots, k) squared distances
    (device: fp16-rounded ranking keys, comparable across one row's lists; re-rank exactly) and
    item rows int32, ascending (+inf / -1 padding). ``thr_row`` (N floats, indexed by X row): keep
    only items whose squared distance is below the row's threshold (its k-th best so far).
    ``items_f16``: ``center_rows_f16(X, C, list_off)``, computed once per graph: the kernel then
    copies pre-centred fp16 item tiles (half the bytes, no per-tile conversion)."""
    N, n = X.shape
    nlist = int(list_off.shape[0]) - 1
    od = torch.full((nslots, k), float("inf"), dtype=torch.float32, device=X.device)
    oi = torch.full((nslots, k), -1, dtype=torch.int32, device=X.device)
    ntiles = int(tile_q0.shape[0])
    if ntiles == 0:
        return od, oi
    if not knn_lists_f16_ok(X, k, C):
        lo = list_off.cpu().numpy()
        po = pair_off.cpu().numpy()
        for q0, c in zip(tile_q0.cpu().tolist(), tile_list.cpu().tolist()):
            q1 = min(q0 + 128, int(po[c + 1]))
            rows = qrows[q0:q1].long()
            items = torch.arange(int(lo[c]), int(lo[c + 1]), device=X.device)
            if items.numel() == 0:
                continue
            d = torch.cdist(X[rows].float(), X[items].float()) ** 2
            if thr_row is not None:
                d = torch.where(d < thr_row[rows].view(-1, 1), d, torch.full_like(d, float("inf")))
            kk = min(k, items.numel())
            v, j = torch.topk(d, kk, dim=1, largest=False)
            j = torch.where(torch.isfinite(v), j, torch.full_like(j, -1))
            sl = qslot[q0:q1].long()
            od[sl, :kk] = v
            oi[sl, :kk] = torch.where(j >= 0, items[j.clamp_min(0)], torch.full_like(j, -1)).int()
        return od, oi
    if C.shape != (nlist, n):
        raise ValueError("knn_pairs: centroids must be nlist x n")
    self_probe = torch.arange(nlist, device=X.device, dtype=torch.int32)
    native.call("srml_knn_pairs_f16c", X.data_ptr(), n, X.stride(0), _c(C).data_ptr(), _c(list_off.long()).data_ptr(),
                _c(pair_off.long()).data_ptr(), _c(qrows.int()).data_ptr(), _c(qslot.int()).data_ptr(),
                _c(tile_q0.long()).data_ptr(), _c(tile_list.int()).data_ptr(), ntiles, int(k), od.data_ptr(),
                oi.data_ptr(), self_probe.data_ptr(), _c(thr_row.float()).data_ptr() if thr_row is not None else None,
                items_f16[0].data_ptr() if items_f16 is not None else None,
                items_f16[1].data_ptr() if items_f16 is not None else None, native.stream(X.device))
    return od, oi


# ------------------------------------------------------------------------------------------
# DBSCAN: eps-degree / core-core union-find over lower-triangle 128x128 tile pairs
# ------------------------------------------------------------------------------------------
DB_TILE = 128


def dbscan_num_tiles(N: int) -> int:
    nt = (N + DB_TILE - 1) // DB_TILE
    return nt * (nt + 1) // 2


def _tri_decode(t: int) -> Tuple[int, int]:
    i = int((np.sqrt(8.0 * t + 1.0) - 1.0) * 0.5)
    while i > 0 and i * (i + 1) // 2 > t:
        i -= 1
    while (i + 1) * (i + 2) // 2 <= t:
        i += 1
    return i, t - i * (i + 1) // 2


def _db_tiles(X: torch.Tensor, xnorm: torch.Tensor, eps2: float, t0: int, t1: int) -> Iterator[Any]:
    """CPU reference: yields (r0, c0, masked squared distances) per tile pair of the range."""
    N = X.shape[0]
    for t in range(t0, t1):
        bi, bj = _tri_decode(t)
        r0, c0 = bi * DB_TILE, bj * DB_TILE
        A, B = X[r0: r0 + DB_TILE].float(), X[c0: c0 + DB_TILE].float()
        d = (xnorm[r0: r0 + DB_TILE].float().view(-1, 1) + xnorm[c0: c0 + DB_TILE].float().view(1, -1)
             - 2.0 * (A @ B.T)).clamp_min(0)
        yield bi == bj, r0, c0, torch.where(d <= eps2, d, torch.full_like(d, float("inf")))


def dbscan_degree(X: torch.Tensor, xnorm: torch.Tensor, eps2: float, t0: int, t1: int,
                  counts: Optional[torch.Tensor] = None) -> torch.Tensor:
    """eps-neighbourhood sizes (self included) accumulated over tile pairs [t0, t1) into int32 counts."""
    N = X.shape[0]
    if counts is None:
        counts = zeros(N, dtype=torch.int32, device=X.device)
    if not X.is_cuda or X.dtype != torch.float32:
        for diag, r0, c0, d in _db_tiles(X, xnorm, eps2, t0, t1):
            adj = torch.isfinite(d)
            counts[r0: r0 + d.shape[0]] += adj.sum(1).int()
            if not diag:
                counts[c0: c0 + d.shape[1]] += adj.sum(0).int()
        return counts
    X = _c(X)
    native.call("srml_dbscan_degree_f32", X.data_ptr(), N, X.shape[1], X.stride(0), _c(xnorm.float()).data_ptr(),
                float(eps2), int(t0), int(t1), counts.data_ptr(), native.stream(X.device))
    return counts


def _orderable_key(d: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """int64 view of the kernel's packed u64 key (orderable(d) << 32 | idx) for d >= 0."""
    bits = d.float().contiguous().view(torch.int32).long() & 0xFFFFFFFF
    return (((bits | 0x80000000) - (1 << 32)) << 32) | (idx.long() & 0xFFFFFFFF)


def _uf_cpu_merge(parent: torch.Tensor, src: np.ndarray, dst: np.ndarray) -> None:
    from scipy.sparse import coo_matrix
    from scipy.sparse.csgraph import connected_components

    N = parent.shape[0]
    p = parent.cpu().numpy().astype(np.int64)
    s = np.concatenate([np.arange(N), src])
    d = np.concatenate([p, dst])
    g = coo_matrix((np.ones(len(s), dtype=np.int8), (s, d)), shape=(N, N))
    _, comp = connected_components(g, directed=False)
    mins = np.full(comp.max() + 1, N, dtype=np.int64)
    np.minimum.at(mins, comp, np.arange(N))
    parent.copy_(torch.from_numpy(mins[comp].astype(np.int32)))


def dbscan_link(X: torch.Tensor, xnorm: torch.Tensor, eps2: float, t0: int, t1: int, core: torch.Tensor,
                parent: torch.Tensor, best: torch.Tensor) -> None:
    """Unite core-core eps edges of tile pairs [t0, t1) into ``parent`` (int32 union-find) and keep,
    for every non-core point, the packed key of its nearest core neighbour in ``best`` (int64 MIN)."""
    N = X.shape[0]
    if not X.is_cuda or X.dtype != torch.float32:
        corb = core.bool()
        srcs, dsts = [], []
        for diag, r0, c0, d in _db_tiles(X, xnorm, eps2, t0, t1):
            adj = torch.isfinite(d)
            rc = corb[r0: r0 + d.shape[0]].view(-1, 1)
            cc = corb[c0: c0 + d.shape[1]].view(1, -1)
            e = torch.nonzero(adj & rc & cc)
            srcs.append((e[:, 0] + r0).numpy())
            dsts.append((e[:, 1] + c0).numpy())
            ridx = torch.arange(c0, c0 + d.shape[1]).view(1, -1).expand_as(d)
            cidx = torch.arange(r0, r0 + d.shape[0]).view(-1, 1).expand_as(d)
            inf = torch.full_like(d, float("inf"))
            # border row <- core column
            dr = torch.where(adj & ~rc & cc, d, inf)
            kr = torch.where(torch.isfinite(dr), _orderable_key(dr, ridx), torch.full_like(ridx, -1))
            best[r0: r0 + d.shape[0]] = torch.minimum(best[r0: r0 + d.shape[0]], _min_valid(kr, 1))
            dc = torch.where(adj & rc & ~cc, d, inf)
            kc = torch.where(torch.isfinite(dc), _orderable_key(dc, cidx), torch.full_like(cidx, -1))
            best[c0: c0 + d.shape[1]] = torch.minimum(best[c0: c0 + d.shape[1]], _min_valid(kc, 0))
        if srcs:
            _uf_cpu_merge(parent, np.concatenate(srcs), np.concatenate(dsts))
        return
    X = _c(X)
    native.call("srml_dbscan_link_f32", X.data_ptr(), N, X.shape[1], X.stride(0), _c(xnorm.float()).data_ptr(),
                float(eps2), int(t0), int(t1), _c(core.to(torch.uint8)).data_ptr(), parent.data_ptr(), best.data_ptr(),
                native.stream(X.device))


def _min_valid(k: torch.Tensor, dim: int) -> torch.Tensor:
    # keys of real candidates are negative int64 (top bit set); -1 means "none" and is the largest
    return k.min(dim).values


def uf_unite_pairs(parent: torch.Tensor, other: torch.Tensor) -> None:
    """Merge another union-find forest (edges i -> other[i]) into ``parent``."""
    if not parent.is_cuda:
        N = parent.shape[0]
        o = other.cpu().numpy().astype(np.int64)
        _uf_cpu_merge(parent, np.arange(N), o)
        return
    native.call("srml_uf_unite_pairs", parent.data_ptr(), parent.shape[0], _c(other.int()).data_ptr(),
                native.stream(parent.device))


def dbscan_labels(parent: torch.Tensor, core: torch.Tensor, best: torch.Tensor) -> torch.Tensor:
    """int64 cluster labels from the compressed forest (roots = each component's smallest core
    index), the core flags (uint8) and ``best`` (nearest core neighbour in the low 32 bits, -1 =
    none): clusters numbered by ascending root, border points take their core neighbour's cluster,
    noise is -1. Device: ``srml_dbscan_labels`` (root-flag prefix scan; no unique / sort)."""
    N = parent.shape[0]
    if not parent.is_cuda:
        corb = core.bool()
        root = parent.long()
        nb = (best & 0xFFFFFFFF).clamp(0, max(N - 1, 0))
        lab_root = torch.where(corb, root, torch.where(best != -1, root[nb], torch.full_like(root, -1)))
        is_root = corb & (root == torch.arange(N, device=parent.device))
        cid = torch.cumsum(is_root.long(), 0) - is_root.long()
        return torch.where(lab_root >= 0, cid[lab_root.clamp_min(0)], torch.full_like(lab_root, -1))
    out = torch.empty(N, dtype=torch.int64, device=parent.device)
    ws = torch.empty(int(native.lib().srml_dbscan_labels_ws(N)), dtype=torch.int32, device=parent.device)
    native.call("srml_dbscan_labels", _c(parent.int()).data_ptr(), _c(core.to(torch.uint8)).data_ptr(),
                _c(best.long()).data_ptr(), N, out.data_ptr(), ws.data_ptr(), native.stream(parent.device))
    return out


def uf_compress(parent: torch.Tensor) -> None:
    """Point every node directly at its root (the smallest index of its component)."""
    if not parent.is_cuda:
        _uf_cpu_merge(parent, np.zeros(0, np.int64), np.zeros(0, np.int64))
        return
    native.call("srml_uf_compress", parent.data_ptr(), parent.shape[0], native.stream(parent.device))


# ------------------------------------------------------------------------------------------
# UMAP: one SGD epoch over the fuzzy-graph edges
# ------------------------------------------------------------------------------------------
def umap_smooth_knn(dist: torch.Tensor, idx: torch.Tensor, k: float, local_connectivity: float = 1.0,
                    bandwidth: float = 1.0, self_rows: bool = True, n_iter: int = 64
                    ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Device smooth_knn_dist + membership strengths of a kNN graph (dist fp32, idx int64, [m, kk]):
    (sigma fp64 [m], rho fp64 [m], w fp32 [m, kk]); ``self_rows``: neighbour == row -> weight 0."""
    m, kk = dist.shape
    d = _c(dist.float())
    ix = _c(idx.long())
    sigma = torch.empty(m, dtype=torch.float64, device=d.device)
    rho = torch.empty(m, dtype=torch.float64, device=d.device)
    w = torch.empty((m, kk), dtype=torch.float32, device=d.device)
    mean_all = d.double().mean().view(1)
    native.call("srml_umap_smooth_knn", d.data_ptr(), ix.data_ptr(), m, kk, kk, float(math.log2(k) * bandwidth),
                float(local_connectivity), int(n_iter), mean_all.data_ptr(), int(bool(self_rows)), sigma.data_ptr(),
                rho.data_ptr(), w.data_ptr(), native.stream(d.device))
    return sigma, rho, w


def knn_refine_sort(Q: torch.Tensor, X: torch.Tensor, pos: torch.Tensor, inner_product: bool = False
                    ) -> Optional[Tuple[torch.Tensor, torch.Tensor]]:
    """Exact distances of each query's selected candidate rows ``pos`` (int64, -1 = none) of X —
    squared euclidean, or -2 q.x for ``inner_product`` — sorted ascending per row (ties keep the
    candidate order; missing candidates last at +inf): (d fp32, pos int64), both (mq, k).
    ``srml_knn_refine_sort_f32`` (one wave per query, no gathered copy of the rows) for fp32
    device data (n <= 1024 from registers, wider rows stream the tail): k <= 64 in one launch;
    larger k in 64-candidate column panels,
    each re-scored and sorted by the kernel, merged by the radix-select kernel (``topk_rows``,
    ties keep the candidate order). None otherwise (the caller keeps its torch path)."""
    mq, k = pos.shape
    n = Q.shape[1]
    if (not Q.is_cuda or Q.dtype != torch.float32 or X.dtype != torch.float32 or k < 1 or k > TOPK_KMAX
            or n < 1 or Q.stride(1) != 1 or X.stride(1) != 1):
        return None
    if k > 64:
        parts = [knn_refine_sort(Q, X, pos[:, c0: c0 + 64], inner_product) for c0 in range(0, k, 64)]
        return topk_rows(torch.cat([a for a, _ in parts], 1), k, ids=torch.cat([b for _, b in parts], 1))
    p = _c(pos.to(torch.int64))
    d = torch.empty((mq, k), dtype=torch.float32, device=Q.device)
    po = torch.empty((mq, k), dtype=torch.int64, device=Q.device)
    native.call("srml_knn_refine_sort_f32", Q.data_ptr(), mq, n, Q.stride(0), X.data_ptr(), X.stride(0), p.data_ptr(),
                k, p.stride(0), int(bool(inner_product)), d.data_ptr(), po.data_ptr(), native.stream(Q.device))
    return d, po


def radix_sort_pairs(keys: torch.Tensor, vals: torch.Tensor, key_bits: int = 64) -> None:
    """In-place stable ascending sort of (int64 key, 32-bit value) pairs by the low ``key_bits``
    bits of the keys (non-negative, < 2^key_bits): ``srml_radix_sort_u64``, 8-bit LSD passes
    (tile histograms, one scan, ballot-multisplit stable scatter); torch.sort on the CPU."""
    n = keys.shape[0]
    assert keys.dtype == torch.int64 and vals.element_size() == 4 and vals.shape[0] == n
    assert keys.is_contiguous() and vals.is_contiguous(), "sorted in place: contiguous tensors"
    if n <= 1:
        return
    if not keys.is_cuda:
        k2, order = torch.sort(keys, stable=True)
        keys.copy_(k2)
        vals.copy_(vals[order])
        return
    dev = keys.device
    ka = torch.empty_like(keys)
    va = torch.empty_like(vals)
    ws = torch.empty(int(native.lib().srml_radix_sort_ws(n)), dtype=torch.int64, device=dev)
    native.call("srml_radix_sort_u64", keys.data_ptr(), vals.data_ptr(), ka.data_ptr(), va.data_ptr(), n,
                int(key_bits), ws.data_ptr(), native.stream(dev))


def umap_fuzzy_union_knn(idx: torch.Tensor, w: torch.Tensor, mix: float = 1.0
                         ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Fuzzy union of the kNN membership matrix A (row i: neighbours idx[i], weights w[i]):
    mix·(A + Aᵀ - A∘Aᵀ) + (1 - mix)·A∘Aᵀ as (rows, cols, vals) sorted by (row, col)."""
    m, kk = idx.shape
    ix = _c(idx.long())
    wv = _c(w.float())
    dev = ix.device
    keys = torch.empty(2 * m * kk, dtype=torch.int64, device=dev)
    vals = torch.empty(2 * m * kk, dtype=torch.float32, device=dev)
    kept = zeros(1, dtype=torch.int64, device=dev)
    native.call("srml_umap_fuzzy_union_knn", ix.data_ptr(), wv.data_ptr(), m, kk, kk, float(mix), keys.data_ptr(),
                vals.data_ptr(), kept.data_ptr(), native.stream(dev))
    # absent entries carry key m*m: after the (row, col) sort they trail the kept ones
    radix_sort_pairs(keys, vals, max(1, int(m * m).bit_length()))
    nk = int(kept.item())
    keys = keys[:nk]
    return keys // m, keys % m, vals[:nk]


def umap_categorical(rows: torch.Tensor, cols: torch.Tensor, vals: torch.Tensor, y: torch.Tensor, n: int,
                     unknown_dist: float = 1.0, far_dist: float = 5.0, mix: float = 1.0) -> torch.Tensor:
    """New values of the (row, col)-sorted, pattern-symmetric fuzzy union after the categorical
    intersection with labels ``y`` (-1 = unknown) and the re-normalised fuzzy union
    (``srml_umap_categorical``: binary-searched transposes, no sort); same pattern and order."""
    nnz = rows.shape[0]
    dev = vals.device
    out = torch.empty(nnz, dtype=torch.float32, device=dev)
    ws = torch.empty(int(native.lib().srml_umap_categorical_ws(n, nnz)), dtype=torch.float64, device=dev)
    native.call("srml_umap_categorical", _c(rows.long()).data_ptr(), _c(cols.long()).data_ptr(),
                _c(vals.float()).data_ptr(), nnz, _c(y.long()).data_ptr(), n, float(unknown_dist), float(far_dist),
                float(mix), out.data_ptr(), ws.data_ptr(), native.stream(dev))
    return out


def umap_epoch(head: torch.Tensor, tail: torch.Tensor, eps: torch.Tensor, next_sample: torch.Tensor,
               next_neg: torch.Tensor, eps_neg: torch.Tensor, emb_head: torch.Tensor, emb_tail: torch.Tensor,
               a: float, b: float, gamma: float, alpha: float, epoch: int, move_other: bool, seed: int,
               pull: bool = False, neg_table: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> None:
    """In-place epoch ``epoch`` of umap-learn's optimize_layout_euclidean (edge-parallel).

    ``pull=True`` (symmetric edge lists only: every (j, k) has its (k, j) of equal weight) moves
    heads only and applies each edge's attraction twice — the same expected update as moving
    both ends, without scattered tail writes (see umap.hip).

    ``neg_table=(tab, ids)`` (device only; ``umap_neg_table``): negative samples are drawn from
    ``tab`` — a snapshot of ``emb_tail`` in the random vertex order ``ids`` (rows a multiple of 8)
    — eight consecutive edges sharing one random 8-row line."""
    n_tail = emb_tail.shape[0]
    dim = emb_head.shape[1]
    if emb_head.is_cuda:
        native.call("srml_umap_epoch", head.data_ptr(), tail.data_ptr(), head.shape[0], eps.data_ptr(),
                    next_sample.data_ptr(), next_neg.data_ptr(), eps_neg.data_ptr(), emb_head.data_ptr(),
                    emb_tail.data_ptr(), n_tail, dim, float(a), float(b), float(gamma), float(alpha), float(epoch),
                    int(bool(move_other)), int(bool(pull)), int(seed) & 0xFFFFFFFF,
                    neg_table[0].data_ptr() if neg_table is not None else None,
                    neg_table[1].data_ptr() if neg_table is not None else None,
                    int(neg_table[0].shape[0] // 8) if neg_table is not None else 0, native.stream(emb_head.device))
        return
    # CPU reference: all due edges of the epoch update from one snapshot (synchronous Hogwild)
    ep = float(epoch)
    idx = torch.nonzero((eps > 0) & (next_sample <= ep)).view(-1)
    if idx.numel() == 0:
        return
    j, k = head[idx].long(), tail[idx].long()
    cur = emb_head[j]
    diff = cur - emb_tail[k]
    d2 = (diff * diff).sum(1, keepdim=True)
    pb = d2.clamp_min(1e-30) ** b
    coef = torch.where(d2 > 0, (-2.0 * a * b * pb / d2.clamp_min(1e-30)) / (a * pb + 1.0), torch.zeros_like(d2))
    g = (coef * diff).clamp(-4, 4) * alpha
    cur = cur + (2.0 * g if pull else g)
    next_sample[idx] += eps[idx]
    en = eps_neg[idx]
    n_neg = torch.where(en > 0, torch.floor((ep - next_neg[idx]) / en.clamp_min(1e-30)), torch.zeros_like(en))
    n_neg = n_neg.clamp_min(0).long()
    rep = torch.repeat_interleave(torch.arange(idx.numel()), n_neg)
    delta = 2.0 * g if pull else g
    if rep.numel():
        gen = torch.Generator().manual_seed((int(seed) * 1000003 + int(epoch)) & 0x7FFFFFFF)
        kk = torch.randint(0, n_tail, (rep.numel(),), generator=gen)
        dn = cur[rep] - emb_tail[kk]
        d2n = (dn * dn).sum(1, keepdim=True)
        c = torch.where(d2n > 0, 2.0 * gamma * b / ((0.001 + d2n) * (a * d2n.clamp_min(1e-30) ** b + 1.0)),
                        torch.zeros_like(d2n))
        gn = torch.where(c > 0, (c * dn).clamp(-4, 4), torch.full_like(dn, 4.0))
        skip = ((d2n <= 0) & (j[rep] == kk).view(-1, 1)).expand_as(gn)
        gn = torch.where(skip, torch.zeros_like(gn), gn) * alpha
        delta = delta + torch.zeros_like(g).index_add_(0, rep, gn)
    next_neg[idx] += n_neg.float() * en
    if move_other and not pull:
        emb_tail.index_add_(0, k, -g)
    emb_head.index_add_(0, j, delta)


def umap_neg_table(emb: torch.Tensor, ids: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """out[r] = emb[ids[r]] (device): the epoch's snapshot for line-shared negative draws."""
    if ids.shape[0] != out.shape[0] or out.shape[1] != emb.shape[1]:
        raise ValueError("umap_neg_table: shape mismatch")
    if not emb.is_cuda:
        return torch.index_select(emb, 0, ids.long(), out=out)
    native.call("srml_umap_neg_table", _c(emb).data_ptr(), _c(ids).data_ptr(), ids.shape[0], emb.shape[1],
                out.data_ptr(), native.stream(emb.device))
    return out


# ------------------------------------------------------------------------------------------
# Symmetric eigensolver (parallel Jacobi, fp64)
# ------------------------------------------------------------------------------------------
def syevj(A: torch.Tensor, max_sweeps: int = 30, tol: float = 1e-15) -> Tuple[torch.Tensor, torch.Tensor]:
    """All eigenpairs of a symmetric matrix: (eigenvalues descending, eigenvectors as columns)."""
    n = A.shape[0]
    if not A.is_cuda:
        w, V = torch.linalg.eigh(A.double())
        return w.flip(0), V.flip(1)
    A = _c(A.double())
    W = torch.empty(n, dtype=torch.float64, device=A.device)
    V = torch.empty((n, n), dtype=torch.float64, device=A.device)
    fn = getattr(native.lib(), "srml_syevj_f64")
    rc = fn(A.data_ptr(), n, W.data_ptr(), V.data_ptr(), int(max_sweeps), float(tol), native.stream(A.device))
    if rc < 0:
        raise RuntimeError("srml_syevj_f64 failed with status %d" % rc)
    return W, V


# ------------------------------------------------------------------------------------------
# SPD solve and Gram-matrix coordinate descent (linear models)
# ------------------------------------------------------------------------------------------
def spd_solve(A: torch.Tensor, b: torch.Tensor) -> Tuple[torch.Tensor, bool]:
    """x = A^-1 b for symmetric positive definite A (fp64) by Cholesky; returns (x, ok).
    ok=False when a non-positive pivot shows A is (numerically) singular."""
    n = A.shape[0]
    if not A.is_cuda:
        L, info = torch.linalg.cholesky_ex(A.double())
        if int(info) != 0:
            return zeros(n, dtype=torch.float64), False
        return torch.cholesky_solve(b.double().view(-1, 1), L).view(-1), True
    st = native.stream(A.device)
    info = zeros(1, dtype=torch.int32, device=A.device)
    if n * 8 <= 110 * 1024:
        # augmented factorisation of [A b; b^T 1]: the trailing updates carry b along, so the last
        # row of the factor is z^T = (L^-1 b)^T and only the backward sweep L^T x = z remains. A
        # non-positive LAST pivot only reflects the arbitrary corner value: info > n is ignored.
        aug = torch.empty((n + 1, n + 1), dtype=torch.float64, device=A.device)
        aug[:n, :n] = A
        aug[n, :n] = b
        aug[n, n] = 1.0
        native.call("srml_potrf_f64", aug.data_ptr(), n + 1, aug.stride(0), info.data_ptr(), st)
        x = aug[n, :n].contiguous()
        native.call("srml_potrs_backward_f64", aug.data_ptr(), n, aug.stride(0), x.data_ptr(), st)
        iv = int(info.item())
        return x, iv == 0 or iv > n
    L = A.double().contiguous().clone()
    native.call("srml_potrf_f64", L.data_ptr(), n, L.stride(0), info.data_ptr(), st)
    x = b.double().contiguous().clone()
    native.call("srml_potrs_f64", L.data_ptr(), n, L.stride(0), x.data_ptr(), st)
    return x, int(info.item()) == 0


def spd_factor(A: torch.Tensor) -> Tuple[torch.Tensor, bool]:
    """Cholesky factor of a symmetric positive definite fp64 matrix (``srml_potrf_f64`` on the
    device), for repeated ``spd_factor_solve`` calls; returns (L, ok)."""
    if not A.is_cuda:
        L, info = torch.linalg.cholesky_ex(A.double())
        return L, int(info) == 0
    L = A.double().contiguous().clone()
    info = zeros(1, dtype=torch.int32, device=A.device)
    native.call("srml_potrf_f64", L.data_ptr(), L.shape[0], L.stride(0), info.data_ptr(), native.stream(A.device))
    return L, int(info.item()) == 0


def spd_factor_solve(L: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """x = (L L^T)^-1 b for a ``spd_factor`` factor (``srml_potrs_f64``: two triangular sweeps)."""
    if not L.is_cuda:
        return torch.cholesky_solve(b.double().view(-1, 1), L).view(-1)
    x = b.double().contiguous().clone()
    native.call("srml_potrs_f64", L.data_ptr(), L.shape[0], L.stride(0), x.data_ptr(), native.stream(L.device))
    return x


def cd_gram(A: torch.Tensor, b: torch.Tensor, l1: torch.Tensor, l2: torch.Tensor, max_iter: int, tol: float,
            w0: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, int]:
    """Cyclic coordinate descent: argmin 1/2 w'Aw - b'w + sum l1|w| + 1/2 sum l2 w^2 (fp64)."""
    n = A.shape[0]
    w = (zeros(n, dtype=torch.float64, device=A.device) if w0 is None else w0.double().clone()).contiguous()
    if A.is_cuda and 2 * n * 8 > 150 * 1024:
        # wider than the LDS-resident kernels: global-memory block-cyclic sweeps, one launch
        # sequence per sweep, the convergence word read once per sweep
        A = A.double().contiguous()
        g = zeros(n, dtype=torch.float64, device=A.device)
        dv = zeros(64, dtype=torch.float64, device=A.device)
        stats = zeros(2, dtype=torch.float64, device=A.device)
        bb, l1c, l2c = _c(b.double()), _c(l1.double()), _c(l2.double())
        st = native.stream(A.device)
        it = 0
        for it in range(1, max(1, max_iter) + 1):
            stats.zero_()
            native.call("srml_cd_sweep_global_f64", A.data_ptr(), n, A.stride(0), bb.data_ptr(), l1c.data_ptr(),
                        l2c.data_ptr(), w.data_ptr(), g.data_ptr(), dv.data_ptr(), stats.data_ptr(),
                        int(it == 1 and w0 is not None), st)
            md, mw = stats.tolist()
            if md <= tol * max(mw, 1e-300):
                break
        return w, it
    if not A.is_cuda:
        Ah, bh, l1h, l2h = (t.double().cpu().numpy() for t in (A, b, l1, l2))
        wh = w.cpu().numpy()
        g = Ah @ wh
        diag = np.diag(Ah) + l2h
        it = 0
        for it in range(1, max(1, max_iter) + 1):
            max_delta = max_w = 0.0
            for j in range(n):
                if diag[j] <= 0:
                    continue
                rho = bh[j] - g[j] + Ah[j, j] * wh[j]
                nw = (rho - l1h[j]) / diag[j] if rho > l1h[j] else ((rho + l1h[j]) / diag[j] if rho < -l1h[j] else 0.0)
                d = nw - wh[j]
                if d != 0.0:
                    g += d * Ah[:, j]
                    wh[j] = nw
                    max_delta = max(max_delta, abs(d))
                max_w = max(max_w, abs(nw))
            if max_delta <= tol * max(max_w, 1e-300):
                break
        return torch.from_numpy(wh).to(A.device), it
    A = A.double().contiguous()
    iters = zeros(1, dtype=torch.int32, device=A.device)
    native.call("srml_cd_gram_f64", A.data_ptr(), n, A.stride(0), _c(b.double()).data_ptr(), _c(l1.double()).data_ptr(),
                _c(l2.double()).data_ptr(), w.data_ptr(), int(max_iter), float(tol), iters.data_ptr(),
                native.stream(A.device))
    return w, int(iters.item())


# ------------------------------------------------------------------------------------------
# CSR (sparse features): ``A`` is any object with indptr (int64), indices (int32), data, shape
def _csr_torch(A) -> torch.Tensor:
    return torch.sparse_csr_tensor(A.indptr, A.indices.long(), A.data, tuple(A.shape))


def _csr_check(A) -> None:
    if A.indptr.dtype != torch.int64 or A.indices.dtype != torch.int32:
        raise TypeError("CSR kernels need int64 row offsets and int32 column indices")
    if A.data.dtype not in (torch.float32, torch.float64):
        raise TypeError("CSR kernels support fp32/fp64 values")
    if A.indptr.numel() != A.shape[0] + 1 or A.indices.numel() != A.data.numel():
        raise ValueError("inconsistent CSR arrays")
    if getattr(A, "_srml_checked", False):
        return
    # one-time host check (the kernels index through indptr/indices without bounds checks)
    ip = A.indptr.cpu()
    if ip.numel() and (int(ip[0]) != 0 or int(ip[-1]) != A.indices.numel() or bool((ip[1:] < ip[:-1]).any())):
        raise ValueError("CSR row offsets are not a monotone 0..nnz sequence")
    if A.indices.numel():
        lo, hi = int(A.indices.min().item()), int(A.indices.max().item())
        if lo < 0 or hi >= A.shape[1]:
            raise ValueError(f"CSR column index out of range [0, {A.shape[1]})")
    try:
        A._srml_checked = True
    except AttributeError:
        pass


def _sfx(A) -> str:
    return "f32" if A.data.dtype == torch.float32 else "f64"


def csr_logreg_binary_loss_grad(A, y: torch.Tensor, w: torch.Tensor, b: float,
                                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp64 [grad_w (n), grad_b, loss_sum] for CSR features: one pass over the non-zeros.
    ``out`` (device, n + 2 fp64): reused result buffer (zeroed here)."""
    m, n = A.shape
    if not A.data.is_cuda:
        Xs = _csr_torch(A).to(torch.float64) if A.data.dtype != torch.float64 else _csr_torch(A)
        z = (Xs @ w.double().view(-1, 1)).view(-1) + b
        yd = y.double()
        r = torch.sigmoid(z) - yd
        loss = torch.nn.functional.softplus(z).sum() - (yd * z).sum()
        g = (Xs.t() @ r.view(-1, 1)).view(-1)
        return torch.cat([g, r.sum().view(1), loss.view(1)])
    _csr_check(A)
    out = zeros(n + 2, dtype=torch.float64, device=A.data.device) if out is None else zero_(out)
    wf = _c(w.to(device=A.data.device, dtype=torch.float64))
    yf = _c(y.to(torch.float32))
    native.call("srml_csr_logreg_binary_" + _sfx(A), A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(),
                m, n, A.data.numel(), yf.data_ptr(), wf.data_ptr(), float(b), None, None, out.data_ptr(),
                native.stream(A.data.device))
    return out


def csr_spmm(A, W: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 Z (m, K) = A W + bias for W (n, K) (multinomial margins). Device: ``srml_csr_spmm_ld``
    over 16-column panels of W / Z (strided, no copies)."""
    m, n = A.shape
    K = W.shape[1]
    if not A.data.is_cuda:
        Z = (_csr_torch(A) @ W.to(A.data.dtype)).float()
        return Z + bias.float() if bias is not None else Z
    _csr_check(A)
    Wf = _c(W.to(torch.float32))
    bf = _c(bias.to(torch.float32)) if bias is not None else None
    Z = torch.empty(m, K, dtype=torch.float32, device=A.data.device)
    st = native.stream(A.data.device)
    for c0 in range(0, K, 16):
        kk = min(16, K - c0)
        native.call("srml_csr_spmm_ld_" + _sfx(A), A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(), m,
                    A.data.numel(), Wf[:, c0:].data_ptr(), kk, K, bf[c0:].data_ptr() if bf is not None else None,
                    Z[:, c0:].data_ptr(), K, st)
    return Z


def csr_spmtm(A, R: torch.Tensor) -> torch.Tensor:
    """fp64 (n, K) = A^T R for R (m, K) (multinomial gradient). Device: ``srml_csr_spmtm_ld`` over
    16-column panels."""
    m, n = A.shape
    K = R.shape[1]
    if not A.data.is_cuda:
        return (_csr_torch(A).t() @ R.to(A.data.dtype)).double()
    _csr_check(A)
    Rf = _c(R.to(torch.float32))
    out = zeros(n, K, dtype=torch.float64, device=A.data.device)
    st = native.stream(A.data.device)
    for c0 in range(0, K, 16):
        kk = min(16, K - c0)
        native.call("srml_csr_spmtm_ld_" + _sfx(A), A.indptr.data_ptr(), A.indices.data_ptr(), A.data.data_ptr(), m,
                    A.data.numel(), Rf[:, c0:].data_ptr(), kk, K, out[:, c0:].data_ptr(), K, st)
    return out


def csr_row_sums(A) -> torch.Tensor:
    """fp64 row sums of a CSR matrix (fp32 values; one thread per row, no atomics)."""
    m = A.shape[0]
    if not A.data.is_cuda:
        rows = torch.repeat_interleave(torch.arange(m), (A.indptr[1:] - A.indptr[:-1]).cpu())
        return zeros(m, dtype=torch.float64).index_add_(0, rows, A.data.double().cpu())
    out = torch.empty(m, dtype=torch.float64, device=A.data.device)
    native.call("srml_csr_row_sums_f32", A.indptr.data_ptr(), _c(A.data.float()).data_ptr(), m, out.data_ptr(),
                native.stream(A.data.device))
    return out


def csr_col_moments(A) -> Tuple[torch.Tensor, torch.Tensor]:
    """Per-column fp64 (sum, sum of squares) over the non-zeros of a CSR matrix."""
    n = A.shape[1]
    dev = A.data.device
    if not A.data.is_cuda:
        d = A.data.double()
        cols = A.indices.long()
        s = zeros(n, dtype=torch.float64).index_add_(0, cols, d)
        q = zeros(n, dtype=torch.float64).index_add_(0, cols, d * d)
        return s, q
    _csr_check(A)
    s = zeros(n, dtype=torch.float64, device=dev)
    q = zeros(n, dtype=torch.float64, device=dev)
    native.call("srml_csr_col_moments_" + _sfx(A), A.indices.data_ptr(), A.data.data_ptr(), A.data.numel(),
                s.data_ptr(), q.data_ptr(), native.stream(dev))
    return s, q


# ------------------------------------------------------------------------------------------
# Logistic loss + gradient accumulation for the on-device quasi-Newton driver (models/qn.py)
def _is_csr(X) -> bool:
    return hasattr(X, "indptr") and hasattr(X, "indices")


def logistic_path(X, K: int) -> str:
    """Which device pass ``logistic_loss_grad`` uses for X (reported by the fit / asserted in tests).
    Every device input runs on the srml kernels (dense fp64 multinomial: margins and X^T R on the
    fp64 MFMA GEMM around the fp64 softmax residual kernel)."""
    if _is_csr(X):
        if not X.data.is_cuda:
            return "torch-cpu"
        return "csr_binary" if K == 1 else ("csr_spmm" if K <= 16 else "csr_wide")
    if not X.is_cuda:
        return "torch-cpu"
    m, n = X.shape
    if deterministic() and X.dtype == torch.float32 and K <= 16:
        return "two_pass_deterministic_f32"
    if K == 1:
        if X.dtype == torch.float32 and n <= 4096:
            return "fused_binary_f32"
        if X.dtype in (torch.float32, torch.float64) and n <= 16384:
            return "lds_binary_" + ("f32" if X.dtype == torch.float32 else "f64")
        return "two_pass_binary_f32" if X.dtype == torch.float32 else "two_pass_binary_f64"
    if X.dtype == torch.float32 and K <= 16:
        fused = os.environ.get("SRML_LOGREG_FUSED", "0") == "1" and int(native.lib().srml_mlogit_supported(n, K))
        return "fused_multinomial_f32" if fused else "two_pass_multinomial_f32"
    if X.dtype == torch.float32:
        return "two_pass_wide_f32"
    return "two_pass_multinomial_f64"


def _glm_wide(X, y32: torch.Tensor, W: torch.Tensor, b: torch.Tensor, out: torch.Tensor,
              flag: Optional[torch.Tensor]) -> None:
    """Softmax data term for K > 16 classes (dense fp32 or CSR): margins in 32-class (dense,
    ``srml_xw_t_f32``) / 16-class (CSR SpMM) column panels of one Z, the wide residual kernel
    (``srml_logit_residual_wide_f32``: R and the loss), the bias gradient as the column sums of R
    (``srml_col_moments_f32``) and the X^T R panels (``srml_xtv_mfma_f32`` / CSR SpMTM)."""
    csr = _is_csr(X)
    m, n = X.shape
    K = W.shape[0]
    dev = X.data.device if csr else X.device
    st = native.stream(dev)
    fp = flag.data_ptr() if flag is not None else None
    Wf = W.to(torch.float32)
    if csr:
        Z = csr_spmm(X, Wf.t())  # 16-class panels inside
    else:
        Z = torch.empty((m, K), dtype=torch.float32, device=dev)
        for c0 in range(0, K, 32):
            xw_t(X, _c(Wf[c0: c0 + 32]), out=Z[:, c0: c0 + 32])
    R = zeros((m, K), dtype=torch.float32, device=dev)  # stays 0 if the done flag skips the residual
    Kn = K * n
    native.call("srml_logit_residual_wide_f32", Z.data_ptr(), m, K, K, _c(y32).data_ptr(), _c(b).data_ptr(), 1,
                R.data_ptr(), K, out[Kn + K:].data_ptr(), fp, st)
    del Z
    gb, _ = col_moments(R, need_sq=False)
    out[Kn: Kn + K] += gb
    if csr:
        out[: K * n] += csr_spmtm(X, R).t().reshape(-1)
        return
    for c0 in range(0, K, 16):
        kk = min(16, K - c0)
        native.call("srml_xtv_mfma_f32", X.data_ptr(), m, n, X.stride(0), R[:, c0:].data_ptr(), kk, K,
                    out[c0 * n:].data_ptr(), 1, n, fp, st)


def mbin_supported(X, M: int) -> bool:
    """Whether ``logistic_loss_grad_multi`` runs on the device kernels for this input (any M: models
    beyond 16 run in 16-model panels)."""
    return (not _is_csr(X)) and X.is_cuda and X.dtype == torch.float32 and M >= 1


def _glm_two_pass(X: torch.Tensor, y32: torch.Tensor, W: torch.Tensor, b: torch.Tensor, sb: int, mode: int,
                  grad: torch.Tensor, so_c: int, so_k: int, gb: torch.Tensor, sgb: int, loss: torch.Tensor, sl: int,
                  flag: Optional[torch.Tensor], zc: Optional[tuple] = None) -> None:
    """Two passes over X for K margins: Z = X W^T (``srml_xw_f32``, one bandwidth-bound pass for
    K <= 32), the residual stage on the device (``srml_logit_residual_f32``: softmax (mode 0) or K
    independent sigmoids (mode 1), bias gradients and losses block-reduced into fp64), then
    grad += R^T X (``srml_xtv2_f32``, one pass for K <= 16). ``W`` (K, n) rows (any row stride),
    output locations given by base tensors + element strides."""
    m, n = X.shape
    K = W.shape[0]
    st = native.stream(X.device)
    fp = flag.data_ptr() if flag is not None else None
    yp = _c(y32).data_ptr()
    if zc is not None:
        # the optimiser's line-search margin cache (K in [XW_MFMA_MIN_K, 16], softmax): the margin
        # and X^T R passes skip on the device while the step asks for a margins-only evaluation
        zfl, zb, zsc = zc
        skip = zfl[13:14]
        Wt = W.to(torch.float32).contiguous()
        Z = torch.empty((m, K), dtype=torch.float32, device=X.device)
        X = _c(X)
        native.call("srml_xw_t_f32_skip", X.data_ptr(), m, n, X.stride(0), Wt.data_ptr(), K, Wt.stride(0), None,
                    Z.data_ptr(), Z.stride(0), skip.data_ptr(), st)
        R = torch.empty((m, K), dtype=torch.float32, device=X.device)
        native.call("srml_logit_residual_zc_f32", Z.data_ptr(), m, K, Z.stride(0), yp, b.data_ptr(), sb, mode,
                    R.data_ptr(), K, gb.data_ptr(), sgb, loss.data_ptr(), sl, fp, zfl.data_ptr(), zb.data_ptr(),
                    zsc.data_ptr(), st)
        fn = "srml_xtv_mfma_f32" if K >= XTV_MFMA_MIN_K else "srml_xtv2_f32"
        native.call(fn, X.data_ptr(), m, n, X.stride(0), R.data_ptr(), K, K, grad.data_ptr(), so_c, so_k,
                    skip.data_ptr(), st)
        return
    Z = xw_t(X, W.to(torch.float32).contiguous()) if K >= XW_MFMA_MIN_K else xw(X, W.t().float().contiguous())
    R = torch.empty((m, K), dtype=torch.float32, device=X.device)
    if deterministic():
        # no atomics: per-block partials into workspaces, folded in block order (bit-reproducible);
        # the margin pass has none to begin with
        L = native.lib()
        ws = torch.empty(max(int(L.srml_logit_residual_ws(m, K)), int(L.srml_xtv_mfma_ws(m, n, K)), 1),
                         dtype=torch.float64, device=X.device)
        native.call("srml_logit_residual_det_f32", Z.data_ptr(), m, K, Z.stride(0), yp, b.data_ptr(), sb, mode,
                    R.data_ptr(), K, gb.data_ptr(), sgb, loss.data_ptr(), sl, fp, ws.data_ptr(), st)
        native.call("srml_xtv_mfma_det_f32", X.data_ptr(), m, n, X.stride(0), R.data_ptr(), K, K, grad.data_ptr(),
                    so_c, so_k, fp, ws.data_ptr(), st)
        return
    native.call("srml_logit_residual_f32", Z.data_ptr(), m, K, Z.stride(0), yp, b.data_ptr(), sb,
                mode, R.data_ptr(), K, gb.data_ptr(), sgb, loss.data_ptr(), sl, fp, st)
    fn = "srml_xtv_mfma_f32" if K >= XTV_MFMA_MIN_K else "srml_xtv2_f32"
    native.call(fn, X.data_ptr(), m, n, X.stride(0), R.data_ptr(), K, K, grad.data_ptr(), so_c, so_k, fp, st)


def logistic_loss_grad_multi(X: torch.Tensor, y32: torch.Tensor, WB: torch.Tensor, out: torch.Tensor) -> torch.Tensor:
    """ADD the data terms of M independent binary models into ``out`` (M, n + 2) rows
    [grad w_j | grad b_j | loss_j], model j at WB[j] = [w_j (n) | b_j] — ONE pass over X for all
    M models (hyper-parameter batching). Device: ``srml_mbin_f32``; otherwise per-model torch."""
    m, n = X.shape
    M = WB.shape[0]
    if mbin_supported(X, M) and WB.stride(1) == 1 and out.stride(1) == 1 and M > 16:
        for j0 in range(0, M, 16):  # 16-model panels: one pass over X each
            logistic_loss_grad_multi(X, y32, WB[j0: j0 + 16], out[j0: j0 + 16])
        return out
    if mbin_supported(X, M) and WB.stride(1) == 1 and out.stride(1) == 1:
        X = _c(X)
        if (os.environ.get("SRML_LOGREG_FUSED", "0") == "1" and not deterministic()
                and int(native.lib().srml_mlogit_supported(n, max(2, M)))):
            native.call("srml_mbin_f32", X.data_ptr(), m, n, X.stride(0), _c(y32).data_ptr(), WB.data_ptr(),
                        WB.stride(0), M, out.data_ptr(), out.stride(0), native.stream(X.device))
            return out
        ld = out.stride(0)
        _glm_two_pass(X, y32, WB[:, :n], WB[:, n:], WB.stride(0), 1, out, 1, ld, out[:, n:], ld, out[:, n + 1:], ld,
                      None)
        return out
    Xd = X.double()
    yd = y32.double()
    Z = Xd @ WB[:, :n].double().t() + WB[:, n].double().view(1, M)
    R = torch.sigmoid(Z) - yd.view(-1, 1)
    out[:, :n] += (R.t() @ Xd)
    out[:, n] += R.sum(0)
    out[:, n + 1] += (torch.nn.functional.softplus(Z) - yd.view(-1, 1) * Z).sum(0)
    return out


def logistic_loss_grad(X, y32: torch.Tensor, w: torch.Tensor, b: torch.Tensor, K: int, out: torch.Tensor,
                       flag: Optional[torch.Tensor] = None, ws: Optional[torch.Tensor] = None,
                       leave_partials: bool = False, zcache: Optional[tuple] = None) -> torch.Tensor:
    """ADD the summed logistic data term at (W, b) into ``out`` = [grad W (K*n, class-major) |
    grad b (K) | loss sum] (fp64). K == 1: binary (labels 0/1, sigmoid); K >= 2: softmax over K
    classes (labels 0..K-1). ``w`` (K*n) and ``b`` (K) are fp64 device tensors read by the kernel
    (no host round trip); ``flag`` (device int32, optional): the kernels skip once it is non-zero.
    ``zcache`` = (QN flags, 2 m K fp64 margin buffers, QN scalars): the optimiser's line-search
    margin cache — binary: the narrow / prefetching kernels (``srml_logreg_binary4_f32``; the
    caller checked ``logreg_zcache_ok``); multinomial (``two_pass_multinomial_f32``): the margin /
    residual / X^T R passes. X: dense (m, n) or CSR."""
    path = logistic_path(X, K)
    if _is_csr(X):
        m, n = X.shape
        dev = X.data.device
    else:
        X = _c(X)
        m, n = X.shape
        dev = X.device
    if path.startswith("torch"):
        if _is_csr(X):
            Xs = _csr_torch(X)
            Xs = Xs.to(torch.float64) if Xs.dtype != torch.float64 else Xs
            W = w.double().view(K, n)
            Z = (Xs @ W.t()) + b.double().view(1, K)
        else:
            Xd = X.double()
            W = w.double().view(K, n)
            Z = Xd @ W.t() + b.double().view(1, K)
        yd = y32.double()
        if K == 1:
            z = Z.view(-1)
            r = (torch.sigmoid(z) - yd).view(-1, 1)
            loss = (torch.nn.functional.softplus(z) - yd * z).sum()
        else:
            lse = torch.logsumexp(Z, 1)
            Y = torch.nn.functional.one_hot(yd.long(), K).double()
            r = torch.exp(Z - lse.view(-1, 1)) - Y
            loss = (lse - (Z * Y).sum(1)).sum()
        if _is_csr(X):
            G = (Xs.t() @ r).t()
        else:
            G = r.t() @ Xd
        out[: K * n] += G.reshape(-1)
        out[K * n: K * n + K] += r.sum(0)
        out[K * n + K] += loss
        return out
    st = native.stream(dev)
    fp = flag.data_ptr() if flag is not None else None
    assert w.dtype == torch.float64 and b.dtype == torch.float64 and out.dtype == torch.float64
    assert w.numel() == K * n and b.numel() == K and out.numel() == K * n + K + 1
    if path == "csr_binary":
        _csr_check(X)
        native.call("srml_csr_logreg_binary_" + _sfx(X), X.indptr.data_ptr(), X.indices.data_ptr(), X.data.data_ptr(),
                    m, n, X.data.numel(), y32.data_ptr(), w.data_ptr(), 0.0, b.data_ptr(), fp, out.data_ptr(), st)
    elif path == "csr_spmm":
        # margins (one SpMM pass, all classes) -> the softmax residual kernel (R, bias gradient,
        # loss) -> the X^T R SpMTM pass
        Z = csr_spmm(X, w.view(K, n).t())
        R = zeros((m, K), dtype=torch.float32, device=dev)  # stays 0 if the done flag skips the residual
        native.call("srml_logit_residual_f32", Z.data_ptr(), m, K, K, _c(y32).data_ptr(), b.data_ptr(), 1, 0,
                    R.data_ptr(), K, out[K * n:].data_ptr(), 1, out[K * n + K:].data_ptr(), 0, fp, st)
        out[: K * n] += csr_spmtm(X, R).t().reshape(-1)
    elif path in ("csr_wide", "two_pass_wide_f32"):
        _glm_wide(X, y32, w.view(K, n), b, out, flag)
    elif path == "two_pass_binary_f32":  # wider than the LDS-resident binary kernels
        _glm_two_pass(X, y32, w.view(1, n), b, 1, 1, out, 1, n, out[n:], 1, out[n + 1:], 1, flag)
    elif path == "two_pass_binary_f64":
        # fp64 inputs wider than the LDS kernels: margins and X^T r on the fp64 MFMA GEMM (split-K
        # over rows), the residual / loss / bias gradient in one fp64 pass (srml_logit_residual_f64)
        z = dgemm(X, w.view(n, 1))
        r = zeros((m, 1), dtype=torch.float64, device=dev)  # stays 0 if the done flag skips it
        native.call("srml_logit_residual_f64", z.data_ptr(), m, 1, 1, _c(y32).data_ptr(), b.data_ptr(), 1, 1,
                    r.data_ptr(), 1, out[n:].data_ptr(), 1, out[n + 1:].data_ptr(), 1, fp, st)
        dgemm(X, r, ta=True, beta=1.0, out=out[:n].view(n, 1))
    elif path == "two_pass_multinomial_f64":
        # fp64 softmax: margins Z = X W^T and the gradient R^T X on the fp64 MFMA GEMM, the
        # residual / bias gradient / loss in one fp64 pass (srml_logit_residual_f64, mode 0; K > 16:
        # the wave-per-row srml_logit_residual_wide_f64 and the bias gradient as R's column sums)
        Z = dgemm(X, w.view(K, n), tb=True)
        R = zeros((m, K), dtype=torch.float64, device=dev)  # stays 0 if the done flag skips it
        if K <= 16:
            native.call("srml_logit_residual_f64", Z.data_ptr(), m, K, K, _c(y32).data_ptr(), b.data_ptr(), 1, 0,
                        R.data_ptr(), K, out[K * n:].data_ptr(), 1, out[K * n + K:].data_ptr(), 0, fp, st)
        else:
            native.call("srml_logit_residual_wide_f64", Z.data_ptr(), m, K, K, _c(y32).data_ptr(), b.data_ptr(), 1,
                        R.data_ptr(), K, out[K * n + K:].data_ptr(), fp, st)
            del Z
            out[K * n: K * n + K] += col_moments(R, need_sq=False)[0]
        dgemm(R, X, ta=True, beta=1.0, out=out[: K * n].view(K, n))
    elif path == "fused_binary_f32":
        # ws: the fit's partial-row workspace (ops.logreg_workspace), None = per-block atomic flush;
        # leave_partials: the rows stay unfolded for the fused optimiser step (srml_qn_step_fused)
        if zcache is not None:
            zfl, zb, zsc = zcache
            native.call("srml_logreg_binary4_f32", X.data_ptr(), m, n, X.stride(0), y32.data_ptr(), w.data_ptr(),
                        0.0, b.data_ptr(), fp, out.data_ptr(), ws.data_ptr() if ws is not None else None,
                        int(bool(leave_partials and ws is not None)), zfl.data_ptr(), zb.data_ptr(), zsc.data_ptr(),
                        st)
        else:
            native.call("srml_logreg_binary3_f32", X.data_ptr(), m, n, X.stride(0), y32.data_ptr(), w.data_ptr(),
                        0.0, b.data_ptr(), fp, out.data_ptr(), ws.data_ptr() if ws is not None else None,
                        int(bool(leave_partials and ws is not None)), st)
    elif path.startswith("lds_binary"):
        native.call("srml_logreg_binary_lds_" + path[-3:], X.data_ptr(), m, n, X.stride(0), y32.data_ptr(),
                    w.data_ptr(), 0.0, b.data_ptr(), fp, out.data_ptr(), st)
    elif path == "fused_multinomial_f32":
        native.call("srml_mlogit_f32", X.data_ptr(), m, n, X.stride(0), y32.data_ptr(), w.data_ptr(), b.data_ptr(),
                    fp, K, out.data_ptr(), st)
    elif path == "two_pass_multinomial_f32" or (path == "two_pass_deterministic_f32" and K > 1):
        _glm_two_pass(X, y32, w.view(K, n), b, 1, 0, out, 1, n, out[K * n:], 1, out[K * n + K:], 0, flag,
                      zc=zcache if path == "two_pass_multinomial_f32" else None)
    elif path == "two_pass_deterministic_f32":  # binary: one sigmoid model
        _glm_two_pass(X, y32, w.view(1, n), b, 1, 1, out, 1, n, out[n:], 1, out[n + 1:], 1, flag)
    else:  # pragma: no cover
        raise AssertionError(path)
    return out


# ------------------------------------------------------------------------------------------
# Small transfers for host-driven solver loops (see csrc/xfer.hip)
def h2d_async(dst: torch.Tensor, src: torch.Tensor) -> None:
    """Enqueue a copy of a page-locked host tensor into a device tensor on the current stream.
    ``src`` must stay untouched until a later synchronising transfer on that stream."""
    if not dst.is_cuda:
        dst.copy_(src)
        return
    assert src.is_pinned() and dst.is_contiguous() and src.is_contiguous() and dst.nbytes == src.nbytes
    native.call("srml_memcpy_h2d_async", dst.data_ptr(), src.data_ptr(), dst.nbytes, native.stream(dst.device))


def d2h_sync(dst: torch.Tensor, src: torch.Tensor) -> None:
    """Copy a device tensor into a page-locked host tensor and wait for the current stream."""
    if not src.is_cuda:
        dst.copy_(src)
        return
    assert dst.is_pinned() and dst.is_contiguous() and src.is_contiguous() and dst.nbytes == src.nbytes
    native.call("srml_memcpy_d2h_sync", dst.data_ptr(), src.data_ptr(), src.nbytes, native.stream(src.device))


def zero_(t: torch.Tensor) -> torch.Tensor:
    """Stream-ordered memset of a contiguous tensor (no fill kernel launch through the dispatcher)."""
    if not t.is_cuda:
        return t.zero_()
    assert t.is_contiguous()
    if t.numel():
        native.call("srml_memset_async", t.data_ptr(), 0, t.nbytes, native.stream(t.device))
    return t


def zeros(*size: Any, **kw: Any) -> torch.Tensor:
    """``torch.zeros`` whose device fill is a stream-ordered DMA memset (``srml_memset_async``)
    instead of a dispatcher fill kernel: the fits allocate zeroed accumulators in their level /
    iteration loops, and each torch fill was one more library launch of serial host work."""
    return zero_(torch.empty(*size, **kw))


# ------------------------------------------------------------------------------------------
# Evaluation partials on the device (csrc/metrics.hip): the CrossValidator transform-evaluate pass
_KIND = {torch.float64: 0, torch.float32: 1, torch.int64: 2, torch.int32: 3}


def _kind(t: torch.Tensor) -> Tuple[torch.Tensor, int]:
    t = _c(t)
    if t.dtype not in _KIND:
        t = t.double()
    return t, _KIND[t.dtype]


CONFUSION_MAX_CLASSES = 4096  # srml_confusion_counts rejects larger C (status -2)


def confusion_counts(y: torch.Tensor, pred: torch.Tensor, C: int) -> Optional[np.ndarray]:
    """(C, C) int64 counts of (label, prediction) pairs, or None when a label / prediction is not
    an integer in [0, C) or C > CONFUSION_MAX_CLASSES (the caller falls back to the host summary).
    Device: LDS-privatised histogram (``srml_confusion_counts``); only the C x C counts come to
    the host."""
    if C > CONFUSION_MAX_CLASSES:
        return None
    m = int(y.shape[0])
    if not y.is_cuda:
        yy, pp = y.double().cpu().numpy(), pred.double().cpu().numpy()
        ok = (yy >= 0) & (yy < C) & (yy == np.floor(yy)) & (pp >= 0) & (pp < C) & (pp == np.floor(pp))
        if not ok.all():
            return None
        out = np.zeros((C, C), np.int64)
        np.add.at(out, (yy.astype(np.int64), pp.astype(np.int64)), 1)
        return out
    yk, yi = _kind(y)
    pk, pi = _kind(pred)
    cnt = torch.zeros(C * C + 1, dtype=torch.int64, device=y.device)
    native.call("srml_confusion_counts", yk.data_ptr(), yi, pk.data_ptr(), pi, m, int(C), cnt.data_ptr(),
                native.stream(y.device))
    h = cnt.cpu().numpy()
    if h[-1] != 0:
        return None
    return h[:-1].reshape(C, C)


def logloss_sum(prob: torch.Tensor, y: torch.Tensor, eps: float) -> float:
    """sum_r -log(max(prob[r, y_r], eps)) (labels clipped to [0, C - 1]); one double to the host."""
    m, C = prob.shape
    if not prob.is_cuda:
        idx = np.clip(y.cpu().numpy().astype(np.int64), 0, C - 1)
        pl = prob.double().cpu().numpy()[np.arange(m), idx]
        return float(-np.log(np.maximum(pl, eps)).sum())
    pk, pi = _kind(prob)
    yk, yi = _kind(y)
    out = torch.zeros(1, dtype=torch.float64, device=prob.device)
    native.call("srml_logloss_sum", pk.data_ptr(), pi, m, C, pk.stride(0), yk.data_ptr(), yi, float(eps),
                out.data_ptr(), native.stream(prob.device))
    return float(out.item())


def reg_moments(y: torch.Tensor, pred: torch.Tensor) -> np.ndarray:
    """(4, 3) fp64 [sum, sum of squares, sum |x|, sum of squared deviations] of the columns
    (label, label - prediction, prediction); 12 doubles to the host."""
    if not y.is_cuda:
        yy, pp = y.double().cpu().numpy(), pred.double().cpu().numpy()
        M = np.stack([yy, yy - pp, pp])
        mu = M.mean(1) if M.shape[1] else np.zeros(3)
        return np.stack([M.sum(1), (M * M).sum(1), np.abs(M).sum(1), ((M - mu[:, None]) ** 2).sum(1)])
    yk, yi = _kind(y)
    pk, pi = _kind(pred)
    out = torch.zeros(12, dtype=torch.float64, device=y.device)
    native.call("srml_reg_moments", yk.data_ptr(), yi, pk.data_ptr(), pi, int(y.shape[0]), out.data_ptr(),
                native.stream(y.device))
    return out.cpu().numpy().reshape(4, 3)
