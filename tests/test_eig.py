"""Top-k symmetric eigensolver (PCA): device-resident block-Krylov Rayleigh-Ritz with CholeskyQR2
vs numpy's dense fp64 eigh (reference N5 ``calSVD`` semantics: descending order, sign-fixed)."""
import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd.models.eig import topk_eigh


def _mat(n, kind, seed=0):
    rng = np.random.default_rng(seed)
    if kind == "rand":
        M = rng.standard_normal((3 * n, n))
        return M.T @ M / (3 * n)
    U = np.linalg.qr(rng.standard_normal((n, 20)))[0]
    s = np.exp(-np.arange(20) / 3.0) * 100
    return (U * s) @ U.T + 1e-6 * np.eye(n)


def _check(dev, n, kind, k):
    A = _mat(n, kind)
    w, V = topk_eigh(torch.from_numpy(A).to(dev), k)
    wr, Vr = np.linalg.eigh(A)
    wr, Vr = wr[::-1][:k], Vr[:, ::-1][:, :k]
    np.testing.assert_allclose(w, wr, rtol=1e-10)
    np.testing.assert_allclose(np.abs(V.T @ Vr), np.eye(k), atol=1e-8)
    idx = np.abs(V).argmax(0)
    assert (V[idx, np.arange(k)] > 0).all()  # sign convention: max-|x| entry positive


@pytest.mark.parametrize("n,kind,k", [(700, "rand", 3), (1100, "lowrank", 5)])
def test_topk_eigh_cpu(n, kind, k):
    _check(torch.device("cpu"), n, kind, k)


@pytest.mark.gpu
@pytest.mark.parametrize("n,kind,k", [(700, "rand", 3), (3000, "lowrank", 3), (2000, "rand", 10)])
def test_topk_eigh_gpu(gpu_device, n, kind, k):
    _check(gpu_device, n, kind, k)


@pytest.mark.gpu
def test_topk_eigh_gpu_rank_deficient_falls_back(gpu_device):
    """Exactly rank-2 matrix, k=3: the Krylov blocks lose rank, the device CholeskyQR breaks down
    and the solver must redo the restart with the host-checked orthonormalisation."""
    rng = np.random.default_rng(3)
    n = 1200
    U = np.linalg.qr(rng.standard_normal((n, 2)))[0]
    A = (U * np.array([5.0, 2.0])) @ U.T
    w, V = topk_eigh(torch.from_numpy(A).to(gpu_device), 3)
    assert np.isfinite(w).all() and np.isfinite(V).all()
    np.testing.assert_allclose(w[:2], [5.0, 2.0], rtol=1e-9)
    np.testing.assert_allclose(np.abs(V[:, :2].T @ U), np.eye(2), atol=1e-8)
