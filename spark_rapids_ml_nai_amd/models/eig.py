"""Top-k symmetric eigensolver for covariance / Gram matrices resident in HBM.

Replaces the reference's dense cuSOLVER ``syevd`` path (``raft::linalg::eigDC`` +
``colReverse``/``rowReverse``/``seqRoot``/``signFlip``, ``jvm/native/src/rapidsml_jni.cu:215-269``;
cuML PCAMG internally). PCA needs only the top-k eigenpairs with k << n, so the MI355X design
is a restarted block-Krylov Rayleigh–Ritz iteration:

* the n x n fp64 matrix stays on the device; every Krylov product ``C @ Q`` and the skinny basis
  products run on our f64-MFMA GEMM (``ops.dgemm`` -> ``srml_dgemm_splitk``: K split over
  grid.z so a 3000 x 3000 x 19 product launches ~1000 blocks instead of 47 output tiles, the
  splits folded in index order) — the only O(n^2) work;
* the (n x b·q) basis stays on the device too: block Gram–Schmidt and CholeskyQR2 are device
  GEMMs; only the tiny (b·q)^2 Gram / projected matrices go to host LAPACK (Cholesky, eigh);
* convergence is checked with true residuals ``||C u - θ u|| <= tol · θ_max`` and the basis is
  restarted from the best Ritz vectors;
* the epilogue orders eigenpairs descending and fixes signs on the device (``srml_sign_flip``,
  the reference N1 ``signFlip``).

Small matrices (n <= DENSE_N) or k close to n use a dense fp64 ``eigh`` directly.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import torch

from .. import ops

DENSE_N = 512


def _orth(V: np.ndarray) -> np.ndarray:
    q, _ = np.linalg.qr(V)
    return q


def _dorth(V: torch.Tensor) -> torch.Tensor:
    """Orthonormal basis of the columns of a device (n x b) fp64 block: CholeskyQR2 (two passes
    of G = V^T V on a device GEMM, a b x b Cholesky on the host, V <- V R^-1 on the device).
    Falls back to a host Householder QR when the Gram matrix is numerically singular."""
    W = V
    for _ in range(2):
        G = ops.dgemm(W, W, ta=True).cpu().numpy()
        G = (G + G.T) * 0.5
        try:
            L = np.linalg.cholesky(G)
        except np.linalg.LinAlgError:
            return torch.from_numpy(_orth(V.cpu().numpy())).to(V.device)
        d = np.diag(L)
        if d.min() <= 1e-7 * d.max():  # nearly rank-deficient: CholQR loses orthogonality
            return torch.from_numpy(_orth(V.cpu().numpy())).to(V.device)
        Rinv = np.linalg.solve(L, np.eye(L.shape[0])).T  # (L^T)^-1 = R^-1
        W = ops.dgemm(W, torch.from_numpy(np.ascontiguousarray(Rinv)).to(V.device))
    return W


def topk_eigh(C: torch.Tensor, k: int, tol: float = 1e-10, max_restarts: int = 60,
              seed: int = 0) -> Tuple[np.ndarray, np.ndarray]:
    """Largest-k eigenpairs of the symmetric fp64 matrix C (device or host).

    Returns (eigenvalues desc [k], eigenvectors [n, k]) as host fp64 arrays with the max-|x|
    entry of every eigenvector positive.
    """
    n = C.shape[0]
    k = min(k, n)
    if n <= DENSE_N or k > n // 4:
        A = C.detach().cpu().double().numpy()
        w, V = np.linalg.eigh((A + A.T) * 0.5)
        w = w[::-1][:k].copy()
        V = np.ascontiguousarray(V[:, ::-1][:, :k])
        Vt = torch.from_numpy(V)
        ops.sign_flip(Vt)
        return w, Vt.numpy()

    dev = C.device
    b = min(n, max(2 * k, k + 16))          # block width
    q = 4                                   # Krylov depth per restart
    rng = np.random.default_rng(seed)
    Q0 = _dorth(torch.from_numpy(rng.standard_normal((n, b))).to(dev))
    theta = None
    U = None
    scale = None
    for _ in range(max_restarts):
        blocks = [Q0]
        Qprev = Q0
        for _j in range(q):
            W = ops.dgemm(C, Qprev)
            # block Gram–Schmidt against the basis so far (twice for stability), then orthonormalise
            Vb = torch.cat(blocks, 1)
            for _r in range(2):
                W = ops.dgemm(Vb, ops.dgemm(Vb, W, ta=True), alpha=-1.0, beta=1.0, out=W.clone())
            Qn = _dorth(W)
            blocks.append(Qn)
            Qprev = Qn
        V = _dorth(torch.cat(blocks, 1))
        CV = ops.dgemm(C, V)
        T = ops.dgemm(V, CV, ta=True).cpu().numpy()
        w, S = np.linalg.eigh((T + T.T) * 0.5)
        order = np.argsort(w)[::-1]
        w, S = w[order], S[:, order]
        Sd = torch.from_numpy(np.ascontiguousarray(S[:, :b])).to(dev)
        U = ops.dgemm(V, Sd)
        CU = ops.dgemm(CV, Sd)
        theta = w[:b]
        if scale is None:
            scale = max(abs(theta[0]), 1e-300)
        th = torch.from_numpy(theta[:k].copy()).to(dev)
        res = torch.linalg.vector_norm(CU[:, :k] - U[:, :k] * th, dim=0).cpu().numpy()
        if np.all(res <= tol * max(abs(theta[0]), 1e-300) * 10 + 1e-300) or np.all(res <= 1e-12 * scale):
            break
        Q0 = _dorth(U[:, :b].contiguous())
    assert theta is not None and U is not None
    vals = theta[:k].copy()
    Vt = U[:, :k].contiguous()
    ops.sign_flip(Vt)
    return vals, Vt.cpu().numpy()
