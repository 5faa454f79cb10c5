"""Sparse (CSR) feature path: the CSR kernels vs a dense fp64 PyTorch reference of the same op, and
LogisticRegression fit on sparse VectorUDT input vs the same data dense.

Reference behaviour: ``enable_sparse_data_optim`` keeps sparse vectors as CSR for cuML's QN solver
(classification.py:957-1151; tests/test_logistic_regression.py:1453-1723 compare sparse against
dense fits)."""
import numpy as np
import pytest
import scipy.sparse as sp
import torch

from spark_rapids_ml_nai_amd import DataFrame, ops
from spark_rapids_ml_nai_amd.core.base import CSR


def _csr(m, n, density, dtype, dev, seed=0, empty_rows=True, heavy_row=0):
    rng = np.random.default_rng(seed)
    A = sp.random(m, n, density=density, format="csr", random_state=rng, dtype=np.float64)
    A.data = rng.standard_normal(A.nnz)
    A = A.tolil()
    if empty_rows and m > 3:
        A[1, :] = 0
        A[m - 1, :] = 0
    if heavy_row:  # one long row exercises the non-cached tail of the row loop
        cols = rng.choice(n, size=min(n, heavy_row), replace=False)
        A[0, cols] = rng.standard_normal(len(cols))
    A = A.tocsr()
    A.sort_indices()
    t = CSR(indptr=torch.from_numpy(A.indptr.astype(np.int64)).to(dev),
            indices=torch.from_numpy(A.indices.astype(np.int32)).to(dev),
            data=torch.from_numpy(A.data).to(dtype).to(dev), shape=A.shape)
    return A, t


def _dense(A):
    return torch.from_numpy(A.toarray())


CASES = [(2000, 300, 0.01, 0), (5000, 1000, 0.05, 700), (3000, 64, 0.5, 0), (777, 4000, 0.002, 3000)]


def _check_kernels(dev, m, n, density, heavy, dtype):
    A, t = _csr(m, n, density, dtype, dev, seed=m, heavy_row=heavy)
    D = _dense(A).to(torch.float64)
    if dtype == torch.float32:
        D = D.float().double()
    rng = np.random.default_rng(1)
    y = torch.from_numpy((rng.random(m) > 0.5).astype(np.float32))
    w = torch.from_numpy(rng.standard_normal(n) * 0.3)
    b = 0.25
    out = ops.csr_logreg_binary_loss_grad(t, y.to(dev), w.to(dev), b).cpu()
    z = D @ w + b
    r = torch.sigmoid(z) - y.double()
    ref = torch.cat([D.T @ r, r.sum().view(1), (torch.nn.functional.softplus(z) - y.double() * z).sum().view(1)])
    torch.testing.assert_close(out, ref, rtol=2e-5, atol=2e-4)

    for K in (1, 3, 5, 16):
        W = torch.from_numpy(rng.standard_normal((n, K))).float()
        bias = torch.from_numpy(rng.standard_normal(K)).float()
        Z = ops.csr_spmm(t, W.to(dev), bias.to(dev)).cpu()
        torch.testing.assert_close(Z.double(), D @ W.double() + bias.double(), rtol=1e-4, atol=1e-4)
        R = torch.from_numpy(rng.standard_normal((m, K))).float()
        G = ops.csr_spmtm(t, R.to(dev)).cpu()
        torch.testing.assert_close(G, D.T @ R.double(), rtol=1e-5, atol=1e-4)

    s, q = ops.csr_col_moments(t)
    torch.testing.assert_close(s.cpu(), D.sum(0), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(q.cpu(), (D * D).sum(0), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("m,n,density,heavy", CASES[:2])
def test_csr_ops_cpu_reference(m, n, density, heavy):
    _check_kernels(torch.device("cpu"), m, n, density, heavy, torch.float64)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
@pytest.mark.parametrize("m,n,density,heavy", CASES)
def test_csr_kernels(gpu_device, m, n, density, heavy, dtype):
    _check_kernels(gpu_device, m, n, density, heavy, dtype)


@pytest.mark.gpu
def test_csr_rejects_bad_indices(gpu_device):
    A, t = _csr(100, 50, 0.1, torch.float32, gpu_device)
    bad = CSR(indptr=t.indptr, indices=t.indices.clone(), data=t.data, shape=t.shape)
    bad.indices[0] = 50
    with pytest.raises(ValueError):
        ops.csr_spmm(bad, torch.ones(50, 2, device=gpu_device))


def _fit_pair(multiclass: bool):
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    rng = np.random.default_rng(7)
    m, n = 3000, 200
    A = sp.random(m, n, density=0.05, format="csr", random_state=rng)
    wt = rng.standard_normal((n, 3 if multiclass else 1))
    Z = A @ wt
    y = (Z.argmax(1) if multiclass else (Z[:, 0] > np.median(Z[:, 0]))).astype(np.float64)
    kw = dict(maxIter=60, regParam=0.01, tol=1e-10, float32_inputs=False)
    ms = LogisticRegression(enable_sparse_data_optim=True, **kw).fit(DataFrame.from_numpy(A, y, num_partitions=2))
    md = LogisticRegression(**kw).fit(DataFrame.from_numpy(A.toarray(), y, num_partitions=2))
    return ms, md


@pytest.mark.parametrize("multiclass", [False, True])
def test_sparse_logreg_matches_dense_cpu(multiclass):
    ms, md = _fit_pair(multiclass)
    # same optimum: objectives agree tightly, coefficients up to the objective's flat directions
    assert abs(ms.objective - md.objective) <= 1e-7 * abs(md.objective)
    np.testing.assert_allclose(ms.coefficientMatrix.toArray(), md.coefficientMatrix.toArray(), rtol=1e-3, atol=3e-3)
    np.testing.assert_allclose(ms.interceptVector.toArray(), md.interceptVector.toArray(), rtol=1e-3, atol=3e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("multiclass", [False, True])
def test_sparse_logreg_matches_dense_gpu(gpu_device, multiclass):
    ms, md = _fit_pair(multiclass)
    assert abs(ms.objective - md.objective) <= 1e-6 * abs(md.objective)
    np.testing.assert_allclose(ms.coefficientMatrix.toArray(), md.coefficientMatrix.toArray(), rtol=1e-3, atol=5e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [4, 16, 23])
def test_csr_multinomial_loss_grad_native(gpu_device, K):
    """CSR softmax data term on the srml kernels (SpMM margins, residual kernel, SpMTM) for K <= 16
    (``csr_spmm``) and K > 16 (``csr_wide``) vs the dense fp64 reference."""
    m, n = 3000, 400
    A, t = _csr(m, n, 0.02, torch.float32, gpu_device, seed=K)
    D = _dense(A).float().double()
    rng = np.random.default_rng(K)
    y = torch.from_numpy(rng.integers(0, K, m).astype(np.float32))
    W = torch.from_numpy(rng.standard_normal(K * n) * 0.2)
    b = torch.from_numpy(rng.standard_normal(K) * 0.3)
    assert ops.logistic_path(t, K) == ("csr_spmm" if K <= 16 else "csr_wide")
    out = torch.zeros(K * n + K + 1, dtype=torch.float64, device=gpu_device)
    ops.logistic_loss_grad(t, y.to(gpu_device), W.to(gpu_device), b.to(gpu_device), K, out)
    Z = D @ W.view(K, n).T + b.view(1, K)
    lse = torch.logsumexp(Z, 1)
    Y = torch.nn.functional.one_hot(y.long(), K).double()
    R = torch.exp(Z - lse.view(-1, 1)) - Y
    ref = torch.cat([(R.T @ D).reshape(-1), R.sum(0), (lse - (Z * Y).sum(1)).sum().view(1)])
    got = out.cpu()
    scale = ref[:-1].abs().max().item()
    assert (got[:-1] - ref[:-1]).abs().max().item() <= 2e-5 * scale + 1e-6
    assert abs(got[-1].item() - ref[-1].item()) <= 1e-5 * abs(ref[-1].item())
    flag = torch.ones(1, dtype=torch.int32, device=gpu_device)
    out2 = torch.zeros_like(out)
    ops.logistic_loss_grad(t, y.to(gpu_device), W.to(gpu_device), b.to(gpu_device), K, out2, flag)
    assert out2.abs().max().item() == 0.0
