"""Device primitives. GPU tensors -> hand-written gfx950 HIP kernels (``libsrml_ops.so``);
CPU tensors -> PyTorch reference implementations of the same math (used by GPU-less CI and as
the numerics oracle in the kernel tests).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import native

__all__ = ["col_moments", "gram", "xw", "dgemm", "sign_flip", "is_native"]


def is_native(t: torch.Tensor) -> bool:
    return t.is_cuda


def _c(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------------------------------
def col_moments(X: torch.Tensor, need_sq: bool = True) -> Tuple[torch.Tensor, Optional[torch.Tensor]]:
    """Per-column fp64 (sum, sum of squares) of a row-major (m, n) matrix."""
    m, n = X.shape
    if not X.is_cuda:
        Xd = X.double()
        return Xd.sum(0), (Xd * Xd).sum(0) if need_sq else None
    X = _c(X)
    s = torch.zeros(n, dtype=torch.float64, device=X.device)
    q = torch.zeros(n, dtype=torch.float64, device=X.device) if need_sq else None
    name = "srml_col_moments_f32" if X.dtype == torch.float32 else "srml_col_moments_f64"
    if X.dtype not in (torch.float32, torch.float64):
        raise TypeError("col_moments supports fp32/fp64")
    native.call(name, X.data_ptr(), m, n, X.stride(0), s.data_ptr(), q.data_ptr() if q is not None else None,
                native.stream(X.device))
    return s, q


def gram(X: torch.Tensor, mean: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out (fp64 n x n) += (X - mean)^T (X - mean); returns out (full symmetric matrix)."""
    m, n = X.shape
    if out is None:
        out = torch.zeros((n, n), dtype=torch.float64, device=X.device)
    if not X.is_cuda:
        Xc = X.double() - (mean.double() if mean is not None else 0.0)
        out += Xc.T @ Xc
        return out
    if X.dtype != torch.float32:
        # fp64 inputs: f64 path on the f64 MFMA dgemm (A^T A)
        Xc = X - mean.to(X.dtype) if mean is not None else X
        Xc = _c(Xc)
        dgemm(Xc, Xc, ta=True, tb=False, alpha=1.0, beta=1.0, out=out)
        return out
    X = _c(X)
    mu = _c(mean.to(torch.float32)) if mean is not None else None
    tmp = out
    if mu is not None or True:
        # kernel accumulates only the upper triangle; mirror afterwards
        up = torch.zeros_like(out)
        native.call("srml_gram_f32", X.data_ptr(), m, n, X.stride(0), mu.data_ptr() if mu is not None else None,
                    up.data_ptr(), native.stream(X.device))
        native.call("srml_mirror_upper_f64", up.data_ptr(), n, native.stream(X.device))
        tmp += up
    return tmp


_XW_WIDTHS = (1, 2, 3, 4, 8, 16, 32)


def xw(X: torch.Tensor, W: torch.Tensor, bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out = X @ W (+ bias): X (m, n) fp32, W (n, k). One bandwidth-bound pass over X."""
    m, n = X.shape
    k = W.shape[1]
    if not X.is_cuda:
        out = X.to(W.dtype) @ W
        return out + bias if bias is not None else out
    if X.dtype != torch.float32 or k > 32:
        out = X @ W.to(X.dtype)
        return out + bias.to(X.dtype) if bias is not None else out
    X = _c(X)
    kk = next(w for w in _XW_WIDTHS if w >= k)
    Wp = torch.zeros((n, kk), dtype=torch.float32, device=X.device)
    Wp[:, :k] = W.to(torch.float32)
    bp = None
    if bias is not None:
        bp = torch.zeros(kk, dtype=torch.float32, device=X.device)
        bp[:k] = bias.to(torch.float32)
    out = torch.empty((m, kk), dtype=torch.float32, device=X.device)
    native.call("srml_xw_f32", X.data_ptr(), m, n, X.stride(0), Wp.data_ptr(), kk,
                bp.data_ptr() if bp is not None else None, out.data_ptr(), kk, native.stream(X.device))
    return out[:, :k] if kk != k else out


def dgemm(A: torch.Tensor, B: torch.Tensor, ta: bool = False, tb: bool = False, alpha: float = 1.0,
          beta: float = 0.0, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp64 out = alpha op(A) op(B) + beta out (row-major)."""
    M = A.shape[1] if ta else A.shape[0]
    K = A.shape[0] if ta else A.shape[1]
    N = B.shape[0] if tb else B.shape[1]
    if out is None:
        out = torch.zeros((M, N), dtype=torch.float64, device=A.device)
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
    native.call("srml_dgemm", int(ta), int(tb), M, N, K, float(alpha), A.data_ptr(), A.stride(0), B.data_ptr(),
                B.stride(0), float(beta), out.data_ptr(), out.stride(0), native.stream(A.device))
    return out


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
