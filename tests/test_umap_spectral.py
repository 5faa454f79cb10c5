"""UMAP spectral initialisation: the device subspace iteration (in-tree CSR SpMM + CholeskyQR2)
spans the same leading eigenvector space as the host Lanczos/eigh path (umap-learn's
spectral_layout semantics), and CholeskyQR2 returns an orthonormal basis of the input span."""
import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd.models import umap as U


def _graph(n=1500, seed=0):
    """Connected symmetric kNN graph on a 3:1 rectangle: the leading non-trivial eigenvectors
    (cos(pi x/3), cos(2 pi x/3)) are separated from the next (cos(pi y)) by a clear gap."""
    rng = np.random.default_rng(seed)
    X = rng.uniform(size=(n, 2)) * np.array([3.0, 1.0])
    D = ((X[:, None, :] - X[None, :, :]) ** 2).sum(-1)
    k = 12
    nbr = np.argsort(D, 1)[:, 1: k + 1]
    rows = np.repeat(np.arange(n), k)
    cols = nbr.reshape(-1)
    vals = np.exp(-D[rows, cols] / D[rows, cols].mean())
    A = np.zeros((n, n))
    A[rows, cols] = vals
    A = np.maximum(A, A.T)
    r, c = np.nonzero(A)
    return r.astype(np.int32), c.astype(np.int32), A[r, c].astype(np.float32), n


def _projector(V):
    Q, _ = np.linalg.qr(V)
    return Q @ Q.T


def test_cholqr2_orthonormal_same_span():
    g = torch.Generator().manual_seed(0)
    Y = torch.randn(5000, 11, generator=g) @ torch.diag(torch.logspace(0, 3, 11))
    Q = U._cholqr2(Y)
    torch.testing.assert_close(Q.double().T @ Q.double(), torch.eye(11, dtype=torch.float64), atol=1e-5, rtol=0)
    P1, P2 = _projector(Y.double().numpy()), _projector(Q.double().numpy())
    assert np.abs(P1 - P2).max() < 1e-4


def _exact_top(r, c, v, n, dim):
    """Eigenvectors 2 .. dim + 1 of D^-1/2 A D^-1/2 by a dense fp64 eigensolver (numpy)."""
    deg = np.zeros(n)
    np.add.at(deg, r, v.astype(np.float64))
    dinv = 1.0 / np.sqrt(np.maximum(deg, 1e-30))
    M = np.zeros((n, n))
    M[r, c] = dinv[r] * v * dinv[c]
    w, V = np.linalg.eigh(0.5 * (M + M.T))
    return V[:, np.argsort(w)[::-1][1: dim + 1]]


@pytest.mark.gpu
def test_spectral_device_chebyshev_matches_exact(gpu_device, monkeypatch):
    """Chebyshev-filtered iteration (opt-in) against the exact eigenvectors: this graph's top
    eigenvalues are 0.9994, 0.9977, 0.9946, 0.9944 — gaps of ~2e-3 that 300 plain subspace steps
    do not resolve (a plain fp64 iteration is still 0.28 away in projector norm)."""
    monkeypatch.setattr(U, "CHEB_DEGREE", 8)
    r, c, v, n = _graph()
    ref = _exact_top(r, c, v, n, 2)
    dev = U._spectral_device(torch.from_numpy(r).to(gpu_device), torch.from_numpy(c).to(gpu_device),
                             torch.from_numpy(v).to(gpu_device), n, 2, 0).cpu().double().numpy()
    assert np.abs(_projector(ref) - _projector(dev)).max() < 1e-2 * np.abs(_projector(ref)).max()


@pytest.mark.gpu
def test_spectral_device_plain_spans_top_cluster(gpu_device):
    """Default plain iteration: the two returned vectors lie in the span of the top eigenvectors
    (their near-degenerate cluster), orthogonal to the trivial one."""
    r, c, v, n = _graph()
    top = _exact_top(r, c, v, n, 12)
    dev = U._spectral_device(torch.from_numpy(r).to(gpu_device), torch.from_numpy(c).to(gpu_device),
                             torch.from_numpy(v).to(gpu_device), n, 2, 0).cpu().double().numpy()
    dev = dev / np.linalg.norm(dev, axis=0, keepdims=True)
    resid = dev - top @ (top.T @ dev)
    assert np.linalg.norm(resid, axis=0).max() < 0.2
