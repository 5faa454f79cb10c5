"""fp64-input kernels, deterministic reductions and the large-k kNN selection (GPU), each against
a plain PyTorch fp64 reference of the same op; plus the host mirrors (CPU)."""
import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import ops
from spark_rapids_ml_nai_amd.ops import native
from spark_rapids_ml_nai_amd.utils import determinism


def _rand(m, n, dev, seed=0, dtype=torch.float64, shift=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(m, n, generator=g, dtype=torch.float64) + shift).to(dtype).to(dev)


# ---------------------------------------------------------------- fp64 inputs -------------
@pytest.mark.gpu
@pytest.mark.parametrize("m,n,k", [(1, 3, 1), (1000, 77, 130), (5000, 300, 64), (4097, 16, 7)])
def test_nearest_centroid_f64(gpu_device, m, n, k):
    X = _rand(m, n, gpu_device, seed=1)
    C = _rand(k, n, gpu_device, seed=2)
    lab, d2 = ops.nearest_centroid(X, C)
    Xh, Ch = X.cpu(), C.cpu()
    D = torch.cdist(Xh, Ch) ** 2
    ref_d, ref_l = D.min(1)
    torch.testing.assert_close(d2.cpu().double(), ref_d, rtol=1e-5, atol=1e-6)
    # labels agree except at exact fp64 near-ties
    got = D.gather(1, lab.cpu().long().view(-1, 1)).view(-1)
    assert torch.all(got <= ref_d + 1e-9 * ref_d.abs().clamp_min(1))


@pytest.mark.gpu
def test_row_sqnorm_f64(gpu_device):
    X = _rand(3001, 129, gpu_device, seed=3)
    out = ops.row_sqnorm(X)
    assert out.dtype == torch.float64
    torch.testing.assert_close(out.cpu(), (X.cpu() ** 2).sum(1), rtol=1e-12, atol=1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("M,N,K,ta,tb", [(3000, 19, 3000, False, False), (76, 19, 3000, True, False),
                                         (300, 4, 100000, True, False), (64, 64, 64, False, True)])
def test_dgemm_splitk_deterministic(gpu_device, M, N, K, ta, tb):
    A = _rand(K, M, gpu_device, seed=4) if ta else _rand(M, K, gpu_device, seed=4)
    B = _rand(N, K, gpu_device, seed=5) if tb else _rand(K, N, gpu_device, seed=5)
    C0 = _rand(M, N, gpu_device, seed=6)
    out1 = ops.dgemm(A, B, ta=ta, tb=tb, alpha=0.5, beta=2.0, out=C0.clone())
    out2 = ops.dgemm(A, B, ta=ta, tb=tb, alpha=0.5, beta=2.0, out=C0.clone())
    a = A.cpu().T if ta else A.cpu()
    b = B.cpu().T if tb else B.cpu()
    ref = 0.5 * (a @ b) + 2.0 * C0.cpu()
    torch.testing.assert_close(out1.cpu(), ref, rtol=1e-10, atol=1e-9)
    assert torch.equal(out1, out2)  # split-K folds in index order: bitwise reproducible


@pytest.mark.gpu
@pytest.mark.parametrize("k", [3, 40])
def test_xw_f64_and_wide_f32(gpu_device, k):
    X = _rand(2000, 300, gpu_device, seed=7)
    W = _rand(300, k, gpu_device, seed=8)
    b = _rand(1, k, gpu_device, seed=9).view(-1)
    out = ops.xw(X, W, b)
    assert out.dtype == torch.float64
    ref = X.cpu() @ W.cpu() + b.cpu()
    torch.testing.assert_close(out.cpu(), ref, rtol=1e-10, atol=1e-9)
    out32 = ops.xw(X.float(), W.float(), b.float())
    torch.testing.assert_close(out32.cpu().double(), ref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_xtv_f64(gpu_device):
    X = _rand(50000, 200, gpu_device, seed=10)
    V = _rand(50000, 3, gpu_device, seed=11)
    out = ops.xtv(X, V)
    torch.testing.assert_close(out.cpu(), X.cpu().T @ V.cpu(), rtol=1e-10, atol=1e-8)


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_cluster_sums_segments(gpu_device, dtype, monkeypatch):
    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    X = _rand(20000, 300, gpu_device, seed=12, dtype=dtype)
    g = torch.Generator().manual_seed(0)
    lab = torch.randint(0, 37, (20000,), generator=g).to(torch.int32)
    lab[lab == 5] = 6  # an empty cluster
    s1, c1 = ops.cluster_sums(X, lab.to(gpu_device), 37)
    s2, _ = ops.cluster_sums(X, lab.to(gpu_device), 37)
    ref = torch.zeros(37, 300, dtype=torch.float64).index_add_(0, lab.long(), X.cpu().double())
    torch.testing.assert_close(s1.cpu(), ref, rtol=1e-10, atol=1e-9)
    assert torch.equal(s1, s2)
    assert torch.equal(c1.cpu(), torch.bincount(lab.long(), minlength=37))


@pytest.mark.gpu
def test_gram_deterministic(gpu_device, monkeypatch):
    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    X = _rand(100000, 200, gpu_device, seed=13, dtype=torch.float32, shift=1.0)
    G1 = ops.gram(X)
    G2 = ops.gram(X)
    assert torch.equal(G1, G2)
    ref = X.cpu().double().T @ X.cpu().double()
    assert ((G1.cpu() - ref).abs().max() / ref.abs().max()).item() < 2e-6


@pytest.mark.gpu
def test_kmeans_fp64_fit_matches_fp32(gpu_device):
    from spark_rapids_ml_nai_amd.models.kmeans import kmeans_fit
    from spark_rapids_ml_nai_amd.parallel.context import PartitionDescriptor, WorkerContext

    rng = np.random.default_rng(0)
    centers = rng.normal(size=(5, 20)) * 10
    Xh = np.concatenate([c + rng.normal(size=(400, 20)) for c in centers])
    ctx = WorkerContext.single(gpu_device)
    desc = PartitionDescriptor.build(ctx, Xh.shape[0], Xh.shape[1])
    r64 = kmeans_fit(torch.from_numpy(Xh).to(gpu_device), desc, ctx, 5, 20, 1e-4, 1)
    r32 = kmeans_fit(torch.from_numpy(Xh).float().to(gpu_device), desc, ctx, 5, 20, 1e-4, 1)
    c64 = np.sort(r64["cluster_centers_"][:, 0])
    c32 = np.sort(r32["cluster_centers_"][:, 0])
    np.testing.assert_allclose(c64, c32, rtol=1e-4, atol=1e-4)


# ---------------------------------------------------------------- top-k / large-k kNN ---------
@pytest.mark.gpu
@pytest.mark.parametrize("rows,L,k", [(3, 10, 20), (7, 5000, 100), (5, 70000, 1024), (4, 1000, 1)])
def test_topk_rows_matches_sort(gpu_device, rows, L, k):
    g = torch.Generator().manual_seed(1)
    v = torch.randn(rows, L, generator=g)
    v[:, ::7] = 0.25  # heavy ties at one value
    gv, gi = ops.topk_rows(v.to(gpu_device), k, id_base=100)
    cv, ci = ops.topk_rows(v, k, id_base=100)
    torch.testing.assert_close(gv.cpu(), cv)
    assert torch.equal(gi.cpu(), ci)


@pytest.mark.gpu
def test_topk_rows_with_ids_multi_slice(gpu_device):
    g = torch.Generator().manual_seed(2)
    v = torch.randn(6, 9000, generator=g)
    ids = torch.randperm(6 * 9000, generator=g).view(6, 9000)
    gv, gi = ops.topk_rows(v.to(gpu_device), 300, ids=ids.to(gpu_device), slice_len=1000)
    cv, ci = ops.topk_rows(v, 300, ids=ids)
    torch.testing.assert_close(gv.cpu(), cv)
    assert torch.equal(gi.cpu(), ci)


@pytest.mark.gpu
@pytest.mark.parametrize("mq,mi,n,k", [(300, 5000, 64, 100), (129, 3000, 37, 1024), (50, 800, 16, 200),
                                         (60, 20000, 16, 100)])
def test_knn_large_k(gpu_device, mq, mi, n, k, monkeypatch):
    monkeypatch.setattr(ops, "_TOPK_SLICE", 1024)  # several slices and item chunks at test sizes
    Q = _rand(mq, n, gpu_device, seed=20, dtype=torch.float32)
    I = _rand(mi, n, gpu_device, seed=21, dtype=torch.float32)
    d, i = ops.knn(Q, I, k, id_offset=7)
    kk = min(k, mi)
    ref = torch.cdist(Q.cpu().double(), I.cpu().double()) ** 2
    rv, _ = torch.sort(ref, 1)
    torch.testing.assert_close(d.cpu().double(), rv[:, :kk], rtol=1e-4, atol=1e-3)
    got = ref.gather(1, i.cpu() - 7)
    torch.testing.assert_close(got, rv[:, :kk], rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
def test_knn_small_k_many_slices_native_merge(gpu_device):
    Q = _rand(40, 32, gpu_device, seed=22, dtype=torch.float32)
    I = _rand(60000, 32, gpu_device, seed=23, dtype=torch.float32)
    d, i = ops.knn(Q, I, 10)
    ref = torch.cdist(Q.cpu().double(), I.cpu().double()) ** 2
    rv, _ = torch.sort(ref, 1)
    torch.testing.assert_close(d.cpu().double(), rv[:, :10], rtol=1e-4, atol=1e-3)


# ---------------------------------------------------------------- CPU mirrors ----------------
def test_topk_rows_cpu_ties_and_padding():
    v = torch.tensor([[3.0, 1.0, 1.0, 2.0], [0.0, 0.0, 0.0, 0.0]])
    out_v, out_i = ops.topk_rows(v, 6, id_base=10)
    assert out_i[0, :4].tolist() == [11, 12, 13, 10]
    assert out_i[1, :4].tolist() == [10, 11, 12, 13]
    assert out_i[0, 4:].tolist() == [-1, -1] and torch.isinf(out_v[0, 4:]).all()


def test_determinism_flag(monkeypatch):
    monkeypatch.delenv("SRML_DETERMINISTIC", raising=False)
    assert not determinism.deterministic()
    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    assert determinism.deterministic()
    determinism.set_deterministic(False)
    try:
        assert not determinism.deterministic()
    finally:
        determinism.set_deterministic(None)


def test_dgemm_cpu_matches_torch():
    A = _rand(50, 30, "cpu", seed=1)
    B = _rand(50, 20, "cpu", seed=2)
    torch.testing.assert_close(ops.dgemm(A, B, ta=True), A.T @ B)
    assert ops._dgemm_splits(3000, 19, 3000, 47) > 1 and ops._dgemm_splits(3000, 3000, 3000, 2209) == 1


# ---------------------------------------------------------------- RF regression determinism ---
@pytest.mark.gpu
def test_rf_regression_hist_deterministic(gpu_device, monkeypatch):
    """Fixed-point cross-chunk folds: bit-identical repeats, equal to the fp64 CPU histogram
    within the fixed-point step, and to the default (atomic fp64) kernel within rounding."""
    g = torch.Generator().manual_seed(5)
    n, m, B, nf, nodes = 12, 60000, 32, 10, 3
    bins = torch.randint(0, B, (n, m), generator=g, dtype=torch.uint8)
    y = torch.randn(m, generator=g) * 3.0 + 1.0
    idx = torch.randperm(m, generator=g)[:50000].sort().values.int()
    w = torch.randint(0, 3, (50000,), generator=g).float()
    feats = torch.stack([torch.randperm(n, generator=g)[:nf] for _ in range(nodes)]).int()
    fb = ops.rf_hist_fb(B, 2, True)
    bounds = [0, 9000, 30000, 50000]
    items = []
    for node in range(nodes):  # several row chunks per node -> cross-chunk folds
        for rb in range(bounds[node], bounds[node + 1], 4096):
            for fc in range((nf + fb - 1) // fb):
                items.append([node, rb, min(rb + 4096, bounds[node + 1]), fc])
    items = torch.tensor(items, dtype=torch.int32)
    dev = lambda t: t.to(gpu_device)  # noqa: E731
    ys = ops.rf_yscale(dev(y))
    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    h1 = ops.rf_hist(dev(bins), dev(idx), dev(y), None, dev(items), dev(feats), nodes, B, 2, True,
                     pos_weight=dev(w), yscale=ys)
    h2 = ops.rf_hist(dev(bins), dev(idx), dev(y), None, dev(items), dev(feats), nodes, B, 2, True,
                     pos_weight=dev(w), yscale=ys)
    assert torch.equal(h1, h2)
    ref = ops.rf_hist(bins, idx, y, None, items, feats, nodes, B, 2, True, pos_weight=w)
    torch.testing.assert_close(h1.cpu(), ref, rtol=1e-6, atol=1e-5)
    monkeypatch.setenv("SRML_DETERMINISTIC", "0")
    h3 = ops.rf_hist(dev(bins), dev(idx), dev(y), None, dev(items), dev(feats), nodes, B, 2, True,
                     pos_weight=dev(w), yscale=ys)
    torch.testing.assert_close(h3, h1, rtol=1e-9, atol=1e-7)


@pytest.mark.gpu
def test_rf_regression_fixed_point_no_overflow(gpu_device, monkeypatch):
    """One bin holding 200k rows of weight 255 at y = max|y| (5.1e7 weighted rows > 2^25): the old
    per-item scale (2^38 / max|y|) wraps the i64 cross-chunk fold; the total-weight scale must not."""
    m, n, B = 200000, 2, 8
    bins = torch.zeros((n, m), dtype=torch.uint8)
    y = torch.full((m,), 7.5)
    idx = torch.arange(m, dtype=torch.int32)
    w = torch.full((m,), 255.0)
    feats = torch.tensor([[0, 1]], dtype=torch.int32)
    items = torch.tensor([[0, rb, min(rb + 4096, m), 0] for rb in range(0, m, 4096)], dtype=torch.int32)
    dev = lambda t: t.to(gpu_device)  # noqa: E731
    ys = ops.rf_yscale(dev(y), float(w.sum()))
    assert 255.0 * m * 7.5 * ys < 2.0 ** 63
    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    h = ops.rf_hist(dev(bins), dev(idx), dev(y), None, dev(items), dev(feats), 1, B, 2, True,
                    pos_weight=dev(w), yscale=ys).cpu()
    assert h[0, 0, 0, 0].item() == 255.0 * m
    assert h[0, 0, 0, 1].item() == pytest.approx(255.0 * m * 7.5, rel=1e-12)
    assert float(h[0, :, 1:].abs().sum()) == 0.0


@pytest.mark.gpu
def test_rf_node_stats_deterministic(gpu_device, monkeypatch):
    g = torch.Generator().manual_seed(6)
    m = 200000
    y = torch.randn(m, generator=g)
    idx = torch.randperm(m, generator=g).int()
    w = torch.randint(0, 4, (m,), generator=g).float()
    bounds = torch.tensor([0, 5, 70000, 70001, 150000, m], dtype=torch.int64)
    ref = ops.rf_node_stats(idx, w, y, bounds, 3, True)
    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    a = ops.rf_node_stats(idx.to(gpu_device), w.to(gpu_device), y.to(gpu_device), bounds.to(gpu_device), 3, True)
    b = ops.rf_node_stats(idx.to(gpu_device), w.to(gpu_device), y.to(gpu_device), bounds.to(gpu_device), 3, True)
    assert torch.equal(a, b)
    torch.testing.assert_close(a.cpu(), ref, rtol=1e-10, atol=1e-8)
    yc = torch.randint(0, 5, (m,), generator=g).float()
    rc = ops.rf_node_stats(idx, w, yc, bounds, 5, False)
    c = ops.rf_node_stats(idx.to(gpu_device), w.to(gpu_device), yc.to(gpu_device), bounds.to(gpu_device), 5, False)
    torch.testing.assert_close(c.cpu(), rc)


@pytest.mark.gpu
def test_rf_regressor_fit_bit_reproducible(gpu_device, monkeypatch):
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.regression import RandomForestRegressor

    monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    rng = np.random.default_rng(3)
    X = rng.standard_normal((30000, 16)).astype(np.float32)
    y = X[:, 0] * 2 + np.sin(X[:, 1]) + 0.1 * rng.standard_normal(30000)
    df = DataFrame.from_numpy(X, y)
    est = RandomForestRegressor(numTrees=6, maxDepth=7, seed=11)
    a, b = est.fit(df), est.fit(df)
    pa = a.transform(df).to_numpy("prediction")
    pb = b.transform(df).to_numpy("prediction")
    assert np.array_equal(pa, pb)
    assert np.corrcoef(pa, y)[0, 1] > 0.9


@pytest.mark.gpu
@pytest.mark.parametrize("regression", [False, True])
def test_rf_hist_record_layout_identical(gpu_device, monkeypatch, regression):
    """Histograms gathered from the 32-byte record layout (rf_interleave) equal the feature-major
    ones exactly (classification counts; deterministic fixed-point regression sums)."""
    if regression:
        monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    g = torch.Generator().manual_seed(17)
    n, m, B, nf, nodes = 70, 30000, 64, 24, 4
    bins = torch.randint(0, B, (n, m), generator=g, dtype=torch.uint8)
    S = 2 if regression else 3
    y = torch.randn(m, generator=g) if regression else torch.randint(0, S, (m,), generator=g).float()
    idx = torch.randperm(m, generator=g)[:20000].sort().values.int()
    w = torch.randint(1, 4, (20000,), generator=g).float()
    feats = torch.stack([torch.randperm(n, generator=g)[:nf].sort().values for _ in range(nodes)]).int()
    fb = ops.rf_hist_fb(B, S, regression)
    bounds = [0, 3000, 9000, 15000, 20000]
    items = [[node, rb, min(rb + 2048, bounds[node + 1]), fc] for node in range(nodes)
             for rb in range(bounds[node], bounds[node + 1], 2048) for fc in range((nf + fb - 1) // fb)]
    items = torch.tensor(items, dtype=torch.int32)
    d = lambda t: t.to(gpu_device)  # noqa: E731
    ys = ops.rf_yscale(d(y), float(w.sum())) if regression else None
    a = ops.rf_hist(d(bins), d(idx), d(y), None, d(items), d(feats), nodes, B, S, regression, pos_weight=d(w),
                    fb=fb, yscale=ys)
    il = ops.rf_interleave(d(bins))
    assert il.numel() == ((n + 31) // 32) * m * 32
    b = ops.rf_hist(d(bins), d(idx), d(y), None, d(items), d(feats), nodes, B, S, regression, pos_weight=d(w),
                    fb=fb, yscale=ys, bins_il=il)
    assert torch.equal(a, b)
    assert ops.rf_il_useful(3000, 1000, 8) and not ops.rf_il_useful(3000, 55, 8) and ops.rf_il_useful(64, 8, 8)


@pytest.mark.gpu
@pytest.mark.parametrize("regression", [False, True])
@pytest.mark.parametrize("n,nf", [(70, 24), (700, 450)])
@pytest.mark.parametrize("rec_bytes", [32, 64])
def test_rf_hist_wide_identical(gpu_device, monkeypatch, regression, n, nf, rec_bytes):
    """The 1024-thread record-layout kernel (chunks of rf_hist_fb_wide features; 450 > that spans
    several chunks) produces the same cells as the feature-major 8-feature items, including split
    row chunks (atomic folds) and exclusive single-chunk nodes (plain stores)."""
    if regression:
        monkeypatch.setenv("SRML_DETERMINISTIC", "1")
    g = torch.Generator().manual_seed(23)
    m, B, nodes = 30000, 64, 4
    bins = torch.randint(0, B, (n, m), generator=g, dtype=torch.uint8)
    S = 2 if regression else 3
    y = torch.randn(m, generator=g) if regression else torch.randint(0, S, (m,), generator=g).float()
    idx = torch.randperm(m, generator=g)[:20000].sort().values.int()
    w = torch.randint(1, 4, (20000,), generator=g).float()
    feats = torch.stack([torch.randperm(n, generator=g)[:nf].sort().values for _ in range(nodes)]).int()
    bounds = [0, 3000, 9000, 15000, 20000]

    def items_for(fb, rows, excl):
        out = []
        for node in range(nodes):
            starts = list(range(bounds[node], bounds[node + 1], rows))
            flag = (1 << 30) if excl and len(starts) == 1 else 0
            out += [[node, rb, min(rb + rows, bounds[node + 1]), fc | flag] for rb in starts
                    for fc in range((nf + fb - 1) // fb)]
        return torch.tensor(out, dtype=torch.int32)

    d = lambda t: t.to(gpu_device)  # noqa: E731
    ys = ops.rf_yscale(d(y), float(w.sum())) if regression else None
    fb = ops.rf_hist_fb(B, S, regression)
    a = ops.rf_hist(d(bins), d(idx), d(y), None, d(items_for(fb, 2048, False)), d(feats), nodes, B, S, regression,
                    pos_weight=d(w), fb=fb, yscale=ys)
    il = ops.rf_interleave(d(bins), rec_bytes)
    span = 128 if rec_bytes == 64 else rec_bytes  # 64-B records in 128-B pairs
    assert il.numel() == ((n + span - 1) // span) * m * span
    fbw = ops.rf_hist_fb_wide(B, S, regression)
    assert fbw > fb
    # node 0 (3000 rows) is one exclusive chunk; the others split into 4096-row chunks
    multi = d(torch.tensor([1, 2, 3]))
    b = ops.rf_hist(d(bins), d(idx), d(y), None, d(items_for(fbw, 4096, True)), d(feats), nodes, B, S, regression,
                    pos_weight=d(w), fb=fbw, yscale=ys, bins_il=il, wide=True, exclusive={"multi_nodes": multi},
                    rec_bytes=rec_bytes)
    assert torch.equal(a, b)


@pytest.mark.gpu
def test_rf_hist_wide_packed_regression(gpu_device):
    """Packed regression cells (one u64 LDS atomic per row and feature): counts exact, sums within
    the 2^-22 max|y| per-row quantisation of the exact deterministic histogram; split rows and
    exclusive nodes as in the unpacked test."""
    g = torch.Generator().manual_seed(29)
    n, nf, m, B, nodes = 700, 450, 30000, 64, 4
    bins = torch.randint(0, B, (n, m), generator=g, dtype=torch.uint8)
    y = torch.randn(m, generator=g) * 3.0 + 1.0
    idx = torch.randperm(m, generator=g)[:20000].sort().values.int()
    w = torch.randint(0, 5, (20000,), generator=g).float()
    feats = torch.stack([torch.randperm(n, generator=g)[:nf].sort().values for _ in range(nodes)]).int()
    bounds = [0, 3000, 9000, 15000, 20000]

    def items_for(fb, rows, excl):
        out = []
        for node in range(nodes):
            starts = list(range(bounds[node], bounds[node + 1], rows))
            flag = (1 << 30) if excl and len(starts) == 1 else 0
            out += [[node, rb, min(rb + rows, bounds[node + 1]), fc | flag] for rb in starts
                    for fc in range((nf + fb - 1) // fb)]
        return torch.tensor(out, dtype=torch.int32)

    d = lambda t: t.to(gpu_device)  # noqa: E731
    il = ops.rf_interleave(d(bins), 64)
    fbp = ops.rf_hist_fb_wide(B, 2, True, packed=True)
    assert fbp > ops.rf_hist_fb_wide(B, 2, True)
    ps = ops.rf_pack_scale(d(y))
    multi = d(torch.tensor([1, 2, 3]))
    got = ops.rf_hist(d(bins), d(idx), d(y), None, d(items_for(fbp, 4096, True)), d(feats), nodes, B, 2, True,
                      pos_weight=d(w), fb=fbp, yscale=1.0, bins_il=il, wide=True, exclusive={"multi_nodes": multi},
                      rec_bytes=64, packed_scale=ps).cpu()
    # exact fp64 oracle on the host
    ref = torch.zeros((nodes, nf, B, 2), dtype=torch.float64)
    for node in range(nodes):
        rows = idx[bounds[node]: bounds[node + 1]].long()
        wn = w[bounds[node]: bounds[node + 1]].double()
        for j in range(nf):
            b = bins[int(feats[node, j]), rows].long()
            ref[node, j, :, 0].index_add_(0, b, wn)
            ref[node, j, :, 1].index_add_(0, b, wn * y[rows].double())
    assert torch.equal(got[..., 0], ref[..., 0])
    tol = 0.5 / ps * ref[..., 0] + 1e-9  # per-row rounding of y to the 2^-22 max|y| grid
    assert bool(((got[..., 1] - ref[..., 1]).abs() <= tol).all())


@pytest.mark.gpu
def test_rf_sample_features_uniform_sorted(gpu_device):
    C, n, nf = 4000, 300, 100
    f = ops.rf_sample_features(C, n, nf, 12345, gpu_device).cpu()
    assert f.shape == (C, nf)
    assert bool((f[:, 1:] > f[:, :-1]).all())  # strictly ascending = distinct
    assert int(f.min()) >= 0 and int(f.max()) < n
    freq = torch.bincount(f.reshape(-1).long(), minlength=n).double() / C  # each feature: p = nf / n
    assert abs(freq.mean().item() - nf / n) < 1e-9 and (freq - nf / n).abs().max().item() < 0.04
    again = ops.rf_sample_features(C, n, nf, 12345, gpu_device).cpu()
    other = ops.rf_sample_features(C, n, nf, 12346, gpu_device).cpu()
    assert torch.equal(f, again) and not torch.equal(f, other)


def _algorithm_s_np(C: int, n: int, nf: int, seed: int) -> np.ndarray:
    """Knuth's Algorithm S with the kernel's counter-based draws, one node at a time in numpy."""
    M = (1 << 64) - 1
    out = np.zeros((C, nf), dtype=np.int32)
    f_all = np.arange(n, dtype=np.uint64)
    for c in range(C):
        base = int(ops._mix64_np(np.array([(seed ^ int(ops._mix64_np(np.array([c + 1], dtype=np.uint64))[0])) & M],
                                          dtype=np.uint64))[0])
        u = (ops._mix64_np(np.uint64(base) + f_all) >> np.uint64(11)).astype(np.float64) * 2.0 ** -53
        need = nf
        for f in range(n):
            if need == 0:
                break
            if u[f] * float(n - f) < float(need):
                out[c, nf - need] = f
                need -= 1
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("C,n,nf", [(37, 3000, 1000), (9, 70, 9), (5, 64, 64), (6, 129, 17)])
def test_rf_sample_features_matches_algorithm_s(gpu_device, C, n, nf):
    """The wave-parallel selection sampling (64 features per step, integer thresholds resolved by a
    scalar pass; dense subsets, nf > n / 8) is bit-identical to the sequential Algorithm S on the
    same draws."""
    assert int(native.lib().srml_rf_sample_features_floyd(n, nf)) == 0
    seed = 0x9E3779B97F4A7C15 ^ (C * n + nf)
    got = ops.rf_sample_features(C, n, nf, seed, gpu_device).cpu().numpy()
    np.testing.assert_array_equal(got, _algorithm_s_np(C, n, nf, seed))


def _floyd_np(C: int, n: int, nf: int, seed: int) -> np.ndarray:
    """Floyd's algorithm with the kernel's counter-based draws (u_i from splitmix64(base + i)),
    one node at a time in numpy, ascending output."""
    M = (1 << 64) - 1
    out = np.zeros((C, nf), dtype=np.int32)
    for c in range(C):
        base = int(ops._mix64_np(np.array([(seed ^ int(ops._mix64_np(np.array([c + 1], dtype=np.uint64))[0])) & M],
                                          dtype=np.uint64))[0])
        u = (ops._mix64_np(np.uint64(base) + np.arange(nf, dtype=np.uint64)) >> np.uint64(11)).astype(np.float64)
        u *= 2.0 ** -53
        taken = set()
        for i in range(nf):
            j = n - nf + i
            t = min(int(np.floor(u[i] * float(j + 1))), j)
            taken.add(j if t in taken else t)
        out[c] = np.sort(np.fromiter(taken, dtype=np.int64)).astype(np.int32)
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("C,n,nf", [(41, 3000, 55), (7, 5000, 71), (5, 12000, 300), (9, 64, 8), (3, 16384, 2048),
                                    (6, 129, 1)])
def test_rf_sample_features_floyd_matches_oracle(gpu_device, C, n, nf):
    """Sparse subsets take Floyd's algorithm (registers as the membership bitmap): bit-identical to
    a sequential Floyd on the same draws, ascending and distinct."""
    assert int(native.lib().srml_rf_sample_features_floyd(n, nf)) == 1
    seed = 0x5DEECE66D ^ (C * n + nf)
    got = ops.rf_sample_features(C, n, nf, seed, gpu_device).cpu().numpy()
    np.testing.assert_array_equal(got, _floyd_np(C, n, nf, seed))


@pytest.mark.gpu
def test_rf_sample_features_floyd_uniform(gpu_device):
    C, n, nf = 20000, 3000, 55
    f = ops.rf_sample_features(C, n, nf, 777, gpu_device).cpu()
    assert bool((f[:, 1:] > f[:, :-1]).all())
    freq = torch.bincount(f.reshape(-1).long(), minlength=n).double() / C
    p = nf / n  # each feature's inclusion probability; binomial sd sqrt(p (1 - p) / C) ~ 1e-3
    assert (freq - p).abs().max().item() < 6 * (p * (1 - p) / C) ** 0.5
