"""Top-k symmetric eigensolver for covariance / Gram matrices resident in HBM.

Replaces the reference's dense cuSOLVER ``syevd`` path (``raft::linalg::eigDC`` +
``colReverse``/``rowReverse``/``seqRoot``/``signFlip``, ``jvm/native/src/rapidsml_jni.cu:215-269``;
cuML PCAMG internally). PCA needs only the top-k eigenpairs with k << n, so the MI355X design
is a restarted block-Krylov Rayleigh–Ritz iteration:

* the n x n fp64 matrix stays on the device; every Krylov product ``C @ Q`` runs on the f64
  MFMA GEMM (``srml_dgemm``) — the only O(n^2) work;
* orthogonalisation / Rayleigh–Ritz on the tiny (n x b·q) basis and (b·q)^2 projected matrix
  run in fp64 LAPACK on the host (microseconds to a few ms at n = 3000);
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
    Q0 = _orth(rng.standard_normal((n, b)))
    theta = None
    U = None
    scale = None
    for _ in range(max_restarts):
        blocks = [Q0]
        Qprev = Q0
        for _j in range(q):
            W = ops.dgemm(C, torch.from_numpy(np.ascontiguousarray(Qprev)).to(dev)).cpu().numpy()
            # block Gram–Schmidt against the basis so far (twice for stability), then QR
            Vb = np.hstack(blocks)
            for _r in range(2):
                W -= Vb @ (Vb.T @ W)
            Qn = _orth(W)
            blocks.append(Qn)
            Qprev = Qn
        V = np.hstack(blocks)
        V = _orth(V)
        CV = ops.dgemm(C, torch.from_numpy(np.ascontiguousarray(V)).to(dev)).cpu().numpy()
        T = V.T @ CV
        w, S = np.linalg.eigh((T + T.T) * 0.5)
        order = np.argsort(w)[::-1]
        w, S = w[order], S[:, order]
        U = V @ S[:, :b]
        CU = CV @ S[:, :b]
        theta = w[:b]
        if scale is None:
            scale = max(abs(theta[0]), 1e-300)
        res = np.linalg.norm(CU[:, :k] - U[:, :k] * theta[:k], axis=0)
        if np.all(res <= tol * max(abs(theta[0]), 1e-300) * 10 + 1e-300) or np.all(res <= 1e-12 * scale):
            break
        Q0 = _orth(U[:, :b])
    assert theta is not None and U is not None
    vals = theta[:k].copy()
    vecs = np.ascontiguousarray(U[:, :k])
    Vt = torch.from_numpy(vecs).to(dev)
    ops.sign_flip(Vt)
    return vals, Vt.cpu().numpy()
