"""Device paths that used to fall back to host loops / library ops, each against
an fp64 torch oracle: IVF candidates for wide rows (n = 784, k = 100), exact kNN with k = 2000
(radix select beyond 1024), the refine-sort for k > 64, 20 batched binary LogReg models (16-model
panels), fp64 binary LogReg with n = 20000 (fp64 MFMA GEMM + fp64 residual) and CSR SpMM /
SpMTM with K = 20 classes (strided 16-column panels)."""
import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import ops

pytestmark = pytest.mark.gpu


def _g(seed):
    return torch.Generator().manual_seed(seed)


def test_knn_k2000(gpu_device):
    Q = torch.randn(300, 48, generator=_g(1)).to(gpu_device)
    I = torch.randn(20000, 48, generator=_g(2)).to(gpu_device)
    d, i = ops.knn(Q, I, 2000)
    D = torch.cdist(Q.double().cpu(), I.double().cpu()) ** 2
    ref_d, _ = torch.topk(D, 2000, dim=1, largest=False)
    torch.testing.assert_close(d.double().cpu(), ref_d, rtol=1e-3, atol=1e-3)
    # the returned ids are at the returned distances
    got = D.gather(1, i.cpu())
    torch.testing.assert_close(got, ref_d, rtol=1e-3, atol=1e-3)


def test_topk_rows_k5000(gpu_device):
    V = torch.randn(40, 70000, generator=_g(3)).to(gpu_device)
    v, j = ops.topk_rows(V, 5000)
    rv, rj = torch.sort(V.cpu(), dim=1, stable=True)
    torch.testing.assert_close(v.cpu(), rv[:, :5000])
    assert torch.equal(j.cpu(), rj[:, :5000])


def test_ivf_wide_rows_k100(gpu_device):
    nlist, n, k = 16, 784, 100
    items = torch.randn(6000, n, generator=_g(4)).to(gpu_device)
    lab = torch.randint(0, nlist, (6000,), generator=_g(5))
    order = torch.argsort(lab, stable=True)
    items = items[order.to(gpu_device)].contiguous()
    counts = torch.bincount(lab, minlength=nlist)
    off = torch.zeros(nlist + 1, dtype=torch.int64)
    off[1:] = torch.cumsum(counts, 0)
    ids = order.to(gpu_device) + 7  # original row ids of the list-sorted items
    Q = torch.randn(50, n, generator=_g(6)).to(gpu_device)
    probes = torch.stack([torch.randperm(nlist, generator=_g(100 + q))[:4] for q in range(50)]).int()
    inorm = (items.double() ** 2).sum(1).float()
    d, i = ops.ivf_search(Q, probes.to(gpu_device), off.to(gpu_device), items, inorm, ids, k)
    Ih, Qh = items.double().cpu(), Q.double().cpu()
    for q in range(50):
        rows = torch.cat([torch.arange(int(off[l]), int(off[l + 1])) for l in probes[q].tolist()])
        dd = ((Ih[rows] - Qh[q]) ** 2).sum(1)
        kk = min(k, rows.numel())
        ref, j = torch.topk(dd, kk, largest=False)
        torch.testing.assert_close(d[q, :kk].double().cpu(), ref, rtol=2e-3, atol=2e-2)
        assert (i[q, :kk].cpu() - 7 == order[rows[j]]).float().mean() > 0.97


def test_refine_sort_k100(gpu_device):
    Q = torch.randn(64, 40, generator=_g(8)).to(gpu_device)
    X = torch.randn(5000, 40, generator=_g(9)).to(gpu_device)
    pos = torch.randint(0, 5000, (64, 100), generator=_g(10)).to(gpu_device)
    d, p = ops.knn_refine_sort(Q, X, pos)
    ref = ((X.double()[pos] - Q.double()[:, None, :]) ** 2).sum(-1)
    rs, _ = torch.sort(ref.cpu(), dim=1)
    torch.testing.assert_close(d.double().cpu(), rs, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(((X.double()[p] - Q.double()[:, None, :]) ** 2).sum(-1).cpu(), rs, rtol=1e-5, atol=1e-4)


def test_logreg_multi_m20(gpu_device):
    m, n, M = 3000, 70, 20
    X = torch.randn(m, n, generator=_g(11)).to(gpu_device)
    y = (torch.rand(m, generator=_g(12)) > 0.5).float().to(gpu_device)
    WB = (torch.randn(M, n + 1, generator=_g(13), dtype=torch.float64) * 0.1).to(gpu_device)
    out = torch.zeros(M, n + 2, dtype=torch.float64, device=gpu_device)
    ops.logistic_loss_grad_multi(X, y, WB, out)
    Xd, yd = X.double().cpu(), y.double().cpu()
    Z = Xd @ WB[:, :n].cpu().T + WB[:, n].cpu()
    R = torch.sigmoid(Z) - yd[:, None]
    torch.testing.assert_close(out[:, :n].cpu(), R.T @ Xd, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(out[:, n].cpu(), R.sum(0), rtol=1e-5, atol=1e-4)
    loss = (torch.nn.functional.softplus(Z) - yd[:, None] * Z).sum(0)
    torch.testing.assert_close(out[:, n + 1].cpu(), loss, rtol=1e-6, atol=1e-5)


def test_logreg_fp64_wide(gpu_device):
    m, n = 400, 20000
    X = (torch.randn(m, n, generator=_g(14), dtype=torch.float64) * 0.05).to(gpu_device)
    y = (torch.rand(m, generator=_g(15)) > 0.5).float().to(gpu_device)
    w = (torch.randn(n, generator=_g(16), dtype=torch.float64) * 0.1).to(gpu_device)
    b = torch.tensor([0.3], dtype=torch.float64, device=gpu_device)
    assert ops.logistic_path(X, 1) == "two_pass_binary_f64"
    out = torch.zeros(n + 2, dtype=torch.float64, device=gpu_device)
    ops.logistic_loss_grad(X, y, w, b, 1, out)
    Xd, yd = X.cpu(), y.double().cpu()
    z = Xd @ w.cpu() + 0.3
    r = torch.sigmoid(z) - yd
    # the residual's sigmoid uses the fp32 hardware exp (common.h logistic_terms): ~1e-7 per row
    torch.testing.assert_close(out[:n].cpu(), Xd.T @ r, rtol=1e-5, atol=2e-6)
    torch.testing.assert_close(out[n].cpu(), r.sum(), rtol=1e-6, atol=1e-5)
    torch.testing.assert_close(out[n + 1].cpu(), (torch.nn.functional.softplus(z) - yd * z).sum(), rtol=1e-7,
                               atol=1e-5)


def test_csr_spmm_spmtm_k20(gpu_device):
    import scipy.sparse as sp

    from spark_rapids_ml_nai_amd.core.base import CSR

    A = sp.random(2000, 300, density=0.05, random_state=3, format="csr", dtype=np.float32)
    Ad = CSR(indptr=torch.from_numpy(A.indptr.astype(np.int64)).to(gpu_device),
             indices=torch.from_numpy(A.indices.astype(np.int32)).to(gpu_device),
             data=torch.from_numpy(A.data).to(gpu_device), shape=A.shape)
    W = torch.randn(300, 20, generator=_g(17)).to(gpu_device)
    bias = torch.randn(20, generator=_g(18)).to(gpu_device)
    Z = ops.csr_spmm(Ad, W, bias)
    dense = torch.from_numpy(A.toarray()).double()
    torch.testing.assert_close(Z.double().cpu(), dense @ W.double().cpu() + bias.double().cpu(), rtol=1e-4, atol=1e-4)
    R = torch.randn(2000, 20, generator=_g(19)).to(gpu_device)
    G = ops.csr_spmtm(Ad, R)
    torch.testing.assert_close(G.cpu(), dense.T @ R.double().cpu(), rtol=1e-6, atol=1e-6)
    rs = ops.csr_row_sums(Ad)
    torch.testing.assert_close(rs.cpu(), dense.sum(1), rtol=1e-12, atol=1e-9)
