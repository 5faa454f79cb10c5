"""UMAP device kernels (fuzzy simplicial set, spectral init) vs the torch reference of the same
math on the CPU, and device fits under the reference's trustworthiness gate."""
import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import ops
from spark_rapids_ml_nai_amd.models import umap as U

pytestmark = pytest.mark.gpu


def _graph(n=3000, dim=16, k=15, seed=0):
    from sklearn.datasets import make_blobs

    X, _ = make_blobs(n, dim, centers=8, cluster_std=2.0, random_state=seed)
    Xt = torch.from_numpy(X).float()
    d, i = U.knn_graph(Xt, Xt, k)
    return d, i


@pytest.mark.parametrize("lc", [1.0, 1.5, 0.0])
def test_smooth_knn_matches_reference(gpu_device, lc):
    d, i = _graph()
    d[5, 1:4] = 0.0  # duplicate points: zero distances
    sig_ref, rho_ref = U.smooth_knn_dist(d, 15.0, local_connectivity=lc)
    w_ref = U.membership_strengths(i, d, sig_ref, rho_ref, torch.arange(d.shape[0]))
    sig, rho, w = ops.umap_smooth_knn(d.to(gpu_device), i.to(gpu_device), 15.0, local_connectivity=lc)
    torch.testing.assert_close(rho.cpu(), rho_ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(sig.cpu(), sig_ref, rtol=1e-6, atol=1e-7)
    torch.testing.assert_close(w.cpu(), w_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("mix", [1.0, 0.3])
def test_fuzzy_union_matches_reference(gpu_device, mix):
    d, i = _graph(n=2000, seed=1)
    n = d.shape[0]
    sig, rho = U.smooth_knn_dist(d, 15.0)
    w = U.membership_strengths(i, d, sig, rho, torch.arange(n))
    rows = torch.arange(n).view(-1, 1).expand_as(i).reshape(-1)
    r_ref, c_ref, v_ref = U.fuzzy_union(rows, i.reshape(-1), w.reshape(-1), n, mix)
    r, c, v = ops.umap_fuzzy_union_knn(i.to(gpu_device), w.to(gpu_device), mix)
    kr = (r_ref * n + c_ref).numpy()
    kg = (r.cpu() * n + c.cpu()).numpy()
    order = np.argsort(kr)
    assert np.array_equal(kg, kr[order])  # same entries, sorted by (row, col)
    np.testing.assert_allclose(v.cpu().numpy(), v_ref.numpy()[order], rtol=1e-5, atol=1e-7)


def test_spectral_dense_device_matches_host(gpu_device):
    # connected graph with well-separated leading eigenvalues: points in an elongated box
    rng = np.random.default_rng(2)
    X = rng.random((1500, 3)) * np.array([10.0, 3.0, 1.0])
    Xt = torch.from_numpy(X).float()
    d, i = U.knn_graph(Xt, Xt, 15)
    n = d.shape[0]
    sig, rho = U.smooth_knn_dist(d, 15.0)
    w = U.membership_strengths(i, d, sig, rho, torch.arange(n))
    rows = torch.arange(n).view(-1, 1).expand_as(i).reshape(-1)
    r, c, v = U.fuzzy_union(rows, i.reshape(-1), w.reshape(-1), n)
    host = U._spectral_host(r.numpy(), c.numpy(), v.numpy(), n, 2, 0)
    dev = U._spectral_dense_device(r.to(gpu_device), c.to(gpu_device), v.to(gpu_device), n, 2).cpu().numpy()
    for j in range(2):  # same subspace up to sign
        cos = abs(float(np.dot(host[:, j], dev[:, j]) / (np.linalg.norm(host[:, j]) * np.linalg.norm(dev[:, j]))))
        assert cos > 0.99, (j, cos)


@pytest.mark.parametrize("n", [1797, 6000])
def test_umap_device_fit_trustworthiness(gpu_device, n):
    from sklearn.datasets import load_digits, make_blobs
    from sklearn.manifold import trustworthiness

    if n == 1797:
        X, _ = load_digits(return_X_y=True)
    else:
        X, _ = make_blobs(n, 20, centers=10, cluster_std=3.0, random_state=4)
    emb = U.umap_fit(torch.from_numpy(X).float().to(gpu_device), {"n_neighbors": 15, "random_state": 1})
    assert trustworthiness(X, emb, n_neighbors=15) > 0.9


@pytest.mark.parametrize("supervised", [False, True])
def test_umap_ivf_list_order_matches_row_order(gpu_device, supervised, monkeypatch):
    """IVF graphs run the fuzzy set / spectral init / epochs in inverted-list order and scatter
    the embedding back: quality must match the row-order pipeline and rows must map back to
    their own points (checked through trustworthiness against the ORIGINAL row order)."""
    from sklearn.datasets import make_blobs
    from sklearn.manifold import trustworthiness

    X, y = make_blobs(12000, 16, centers=12, cluster_std=2.5, random_state=3)
    Xt = torch.from_numpy(X).float().to(gpu_device)
    params = {"n_neighbors": 15, "random_state": 2, "build_algo": "ivf", "n_epochs": 150,
              "build_kwds": {"nlist": 24, "nprobe": 8}}
    yt = torch.from_numpy(y).to(gpu_device) if supervised else None
    tw = {}
    for flag in (True, False):
        monkeypatch.setattr(U, "LIST_ORDER", flag)
        emb = U.umap_fit(Xt, params, y=yt)
        tw[flag] = trustworthiness(X, emb, n_neighbors=15)
    assert tw[True] > 0.9 and tw[True] > tw[False] - 0.01, tw


def test_umap_neg_lines_matches_iid_negatives(gpu_device, monkeypatch):
    """Line-shared negative draws from the per-epoch random-order snapshot keep the layout quality
    of i.i.d. per-edge draws."""
    from sklearn.datasets import make_blobs
    from sklearn.manifold import trustworthiness

    from spark_rapids_ml_nai_amd import ops

    X, _ = make_blobs(10000, 16, centers=10, cluster_std=2.5, random_state=6)
    Xt = torch.from_numpy(X).float().to(gpu_device)
    emb = torch.randn(5003, 2, device=gpu_device)
    ids = torch.randperm(5003, device=gpu_device)[:5000].int()
    tab = ops.umap_neg_table(emb, ids, torch.empty(5000, 2, device=gpu_device))
    assert torch.equal(tab, emb[ids.long()])
    tw = {}
    for flag in (True, False):
        monkeypatch.setattr(U, "NEG_LINES", flag)
        e = U.umap_fit(Xt, {"n_neighbors": 15, "random_state": 4, "n_epochs": 200})
        tw[flag] = trustworthiness(X, e, n_neighbors=15)
    assert tw[True] > 0.9 and tw[True] > tw[False] - 0.01, tw


def test_categorical_intersection_native_matches_torch(gpu_device):
    """Supervised UMAP: the native categorical intersection on the sorted, pattern-symmetric union
    equals the torch reference (scale, per-row max reset, coalescing fuzzy union) in fp64."""
    import torch

    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.models import umap as U

    g = torch.Generator().manual_seed(3)
    N, k = 4000, 12
    idx = torch.rand(N, N, generator=g).argsort(1)[:, :k]  # distinct neighbours per row, like a kNN graph
    w = torch.rand(N, k, generator=g) * 0.9 + 0.05
    rows, cols, vals = ops.umap_fuzzy_union_knn(idx.to(gpu_device), w.to(gpu_device), 1.0)
    y = torch.randint(-1, 5, (N,), generator=g)
    r1, c1, v1 = U.categorical_intersection(rows, cols, vals, y.to(gpu_device), N)
    r0, c0, v0 = U.categorical_intersection(rows.cpu(), cols.cpu(), vals.cpu(), y, N)
    k1 = (r1.cpu() * N + c1.cpu())
    k0 = (r0.long() * N + c0.long())
    o1, o0 = torch.argsort(k1), torch.argsort(k0)
    assert torch.equal(k1[o1], k0[o0])
    torch.testing.assert_close(v1.cpu()[o1].double(), v0[o0].double(), rtol=1e-5, atol=1e-7)
