"""Kernel numerics: every HIP kernel vs a plain PyTorch fp32/fp64 reference of the same op."""
import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import ops

pytestmark = pytest.mark.gpu


def _rand(m, n, dev, seed=0, dtype=torch.float32, shift=0.0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return (torch.randn(m, n, generator=g, dtype=torch.float64) + shift).to(dtype).to(dev)


@pytest.mark.parametrize("m,n", [(1, 5), (1000, 3), (4097, 130), (20000, 257), (3000, 1000)])
def test_col_moments(gpu_device, m, n):
    X = _rand(m, n, gpu_device, shift=3.0)
    s, q = ops.col_moments(X)
    Xd = X.double().cpu()
    torch.testing.assert_close(s.cpu(), Xd.sum(0), rtol=1e-5, atol=1e-3)
    torch.testing.assert_close(q.cpu(), (Xd * Xd).sum(0), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("m,n,center", [(100, 3, False), (1000, 128, True), (5000, 130, True), (777, 301, False),
                                        (20000, 513, True)])
def test_gram(gpu_device, m, n, center):
    X = _rand(m, n, gpu_device, seed=1, shift=1.0)
    mu = X.double().mean(0) if center else None
    G = ops.gram(X, mu)
    Xc = X.double().cpu() - (mu.cpu() if center else 0.0)
    ref = Xc.T @ Xc
    err = (G.cpu() - ref).abs().max().item() / ref.abs().max().item()
    assert err < 2e-6, err
    assert torch.allclose(G, G.T)


def test_gram_asymmetric_columns(gpu_device):
    # asymmetric operand pattern: catches row/col swaps in the MFMA C-write
    m, n = 64, 200
    X = torch.zeros(m, n, dtype=torch.float32)
    for r in range(m):
        X[r, (r * 7) % n] = 1.0 + r
        X[r, (r * 13 + 5) % n] = -2.0
    G = ops.gram(X.to(gpu_device)).cpu()
    ref = X.double().T @ X.double()
    torch.testing.assert_close(G, ref)


@pytest.mark.parametrize("m,n,k", [(1000, 3000, 3), (12345, 128, 1), (999, 37, 5), (4000, 256, 16), (300, 64, 32),
                                   (3001, 1000, 10), (257, 333, 20), (70, 3, 4)])
def test_xw(gpu_device, m, n, k):
    X = _rand(m, n, gpu_device, seed=2)
    W = _rand(n, k, gpu_device, seed=3)
    b = _rand(1, k, gpu_device, seed=4).view(-1)
    out = ops.xw(X, W, b).cpu().double()
    ref = X.double().cpu() @ W.double().cpu() + b.double().cpu()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("ta,tb", [(False, False), (True, False), (False, True), (True, True)])
def test_dgemm(gpu_device, ta, tb):
    M, N, K = 130, 67, 301
    A = _rand(K if ta else M, M if ta else K, gpu_device, seed=5, dtype=torch.float64)
    B = _rand(N if tb else K, K if tb else N, gpu_device, seed=6, dtype=torch.float64)
    C = _rand(M, N, gpu_device, seed=7, dtype=torch.float64)
    ref = 0.5 * ((A.T if ta else A) @ (B.T if tb else B)) + 2.0 * C
    out = ops.dgemm(A, B, ta, tb, alpha=0.5, beta=2.0, out=C.clone())
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-10)


def test_sign_flip(gpu_device):
    U = _rand(500, 7, gpu_device, seed=8, dtype=torch.float64)
    ref = U.clone().cpu()
    ops.sign_flip(ref)  # CPU reference path
    out = ops.sign_flip(U.clone()).cpu()
    torch.testing.assert_close(out, ref)
    idx = out.abs().argmax(0)
    assert torch.all(out[idx, torch.arange(7)] > 0)


@pytest.mark.parametrize("m,n,k", [(1000, 3, 1), (5000, 300, 2), (20000, 3000, 1), (777, 129, 4), (100, 10, 7),
                                   (20000, 3000, 10), (3001, 2050, 16), (999, 70, 21)])
def test_xtv(gpu_device, m, n, k):
    X = _rand(m, n, gpu_device, seed=11)
    V = _rand(m, k, gpu_device, seed=12)
    out = ops.xtv(X, V).cpu()
    ref = X.double().cpu().T @ V.double().cpu()
    torch.testing.assert_close(out, ref, rtol=1e-5, atol=1e-3)


def test_xw_t_unaligned_rows(gpu_device):
    """MFMA skinny GEMM on a row-strided view (ld % 4 != 0 -> guarded scalar path) and a strided Wt."""
    base = _rand(513, 303, gpu_device, seed=21)
    X = base[:, 1:300]
    Wbase = _rand(12, 310, gpu_device, seed=22)
    Wt = Wbase[:, 2:301]
    out = ops.xw_t(X, Wt).cpu().double()
    ref = X.double().cpu() @ Wt.double().cpu().T
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-4)


def test_row_sqnorm(gpu_device):
    X = _rand(3001, 131, gpu_device, seed=13)
    torch.testing.assert_close(ops.row_sqnorm(X).cpu().double(), (X.double() ** 2).sum(1).cpu(), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("m,n", [(500, 7), (4000, 256), (3000, 1000), (5000, 3000), (2000, 4096), (1000, 1500),
                                 (130001, 2052)])
def test_logreg_binary_loss_grad(gpu_device, m, n):
    X = _rand(m, n, gpu_device, seed=14) * 0.1
    y = (torch.rand(m, generator=torch.Generator().manual_seed(1)) > 0.5).float().to(gpu_device)
    w = torch.randn(n, generator=torch.Generator().manual_seed(2), dtype=torch.float64).to(gpu_device) * 0.3
    b = 0.25
    out = ops.logreg_binary_loss_grad(X, y, w, b).cpu()
    Xd = X.double().cpu()
    z = Xd @ w.cpu() + b
    p = torch.sigmoid(z)
    r = p - y.double().cpu()
    loss = torch.nn.functional.softplus(z).sum() - (y.double().cpu() * z).sum()
    torch.testing.assert_close(out[:n], Xd.T @ r, rtol=1e-4, atol=1e-3)
    torch.testing.assert_close(out[n], r.sum(), rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(out[n + 1], loss, rtol=1e-7, atol=1e-6)
    # the grouped-fold epilogue's counters reset themselves: repeated launches agree
    for _ in range(2):
        again = ops.logreg_binary_loss_grad(X, y, w, b).cpu()
        torch.testing.assert_close(again, out, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("m,n,k", [(1000, 16, 20), (3000, 64, 5), (2000, 300, 130), (1024, 3000, 257), (777, 33, 1),
                                   (100003, 64, 20), (5001, 100, 33), (12345, 64, 64), (4096, 3, 2)])
def test_nearest_centroid(gpu_device, m, n, k):
    g = torch.Generator().manual_seed(3)
    C = torch.randn(k, n, generator=g) * 3
    lab = torch.randint(0, k, (m,), generator=g)
    X = (C[lab] + 0.5 * torch.randn(m, n, generator=g)).float()
    labels, dist = ops.nearest_centroid(X.to(gpu_device), C.float().to(gpu_device))
    D = torch.cdist(X.double(), C.double()) ** 2
    ref_d, ref_l = D.min(1)
    got = D[torch.arange(m), labels.long().cpu()]
    # chosen centroid is (numerically) optimal; distances match
    assert torch.all(got <= ref_d + 1e-3 * (1 + ref_d))
    scale = (X.double() ** 2).sum(1) + (C.double() ** 2).sum(1).max()
    assert torch.all((dist.double().cpu() - ref_d).abs() <= 1e-5 * scale + 1e-3)


@pytest.mark.parametrize("m,n,k", [(1000, 16, 20), (2000, 300, 130), (1024, 3000, 257), (777, 33, 1), (4099, 130, 1000)])
def test_nearest_centroid_split(gpu_device, m, n, k):
    """Split-bf16 (6-product) MFMA distance GEMM vs the fp64 distance matrix."""
    g = torch.Generator().manual_seed(5)
    C = torch.randn(k, n, generator=g) * 3
    lab = torch.randint(0, k, (m,), generator=g)
    X = (C[lab] + 0.5 * torch.randn(m, n, generator=g)).float()
    Xd = X.to(gpu_device)
    P = ops.split_bf16x3(Xd)
    assert P.shape[1] % 128 == 0 and P.shape[2] % 16 == 0
    torch.testing.assert_close(P.float().sum(0)[:m, :n].cpu(), X, rtol=0, atol=0)
    labels, dist = ops.nearest_centroid_split(P, m, C.float().to(gpu_device), ops.row_sqnorm(Xd))
    D = torch.cdist(X.double(), C.double()) ** 2
    ref_d, _ = D.min(1)
    got = D[torch.arange(m), labels.long().cpu()]
    assert torch.all(got <= ref_d + 1e-3 * (1 + ref_d))
    scale = (X.double() ** 2).sum(1) + (C.double() ** 2).sum(1).max()
    assert torch.all((dist.double().cpu() - ref_d).abs() <= 1e-5 * scale + 1e-3)


@pytest.mark.parametrize("m,n,k", [(5000, 16, 20), (20000, 3000, 50), (3000, 64, 200), (5000, 301, 300),
                                   (70000, 1024, 1000), (100003, 64, 20), (9999, 130, 7), (37, 64, 20)])
def test_cluster_sums(gpu_device, m, n, k):
    X = _rand(m, n, gpu_device, seed=15)
    labels = torch.randint(0, k, (m,), generator=torch.Generator().manual_seed(4)).int()
    sums, counts = ops.cluster_sums(X, labels.to(gpu_device), k)
    ref = torch.zeros(k, n, dtype=torch.float64).index_add_(0, labels.long(), X.double().cpu())
    torch.testing.assert_close(sums.cpu(), ref, rtol=1e-4, atol=1e-3)
    assert torch.equal(counts.cpu(), torch.bincount(labels.long(), minlength=k))


@pytest.mark.parametrize("kernel", ["mfma", "valu"])
@pytest.mark.parametrize("m,n,k", [(100003, 64, 20), (5000, 4, 1), (777, 16, 5), (20000, 32, 32), (33333, 60, 17),
                                   (256, 64, 24), (70001, 48, 9)])
def test_kmeans_lloyd_small_matches_reference(gpu_device, m, n, k, kernel, monkeypatch):
    """Fused small-k Lloyd step (one pass: bf16 split-MFMA distances + exact one-hot sums, or the
    VALU search + f32 one-hot MFMA) against fp64: labels are the arg-min up to fp32 near-ties,
    sums / counts / inertia are those of its own labels."""
    monkeypatch.setenv("SRML_LLOYD_KERNEL", kernel)
    g = torch.Generator().manual_seed(m + k)
    C = torch.randn(k, n, generator=g) * 2
    X = (C[torch.randint(0, k, (m,), generator=g)] + torch.randn(m, n, generator=g)).float()
    Xd, Cd = X.to(gpu_device), C.float().to(gpu_device)
    assert ops.lloyd_small_ok(Xd, k)
    lab, dist, sums, counts, inertia = ops.kmeans_lloyd_small(Xd, Cd)
    D = torch.cdist(X.double(), C.double()) ** 2
    ref_d, _ = D.min(1)
    lab_c = lab.long().cpu()
    got = D[torch.arange(m), lab_c]
    assert torch.all(got <= ref_d + 1e-4 * (1 + ref_d))
    torch.testing.assert_close(dist.double().cpu(), got, rtol=1e-4, atol=1e-3)
    ref_s = torch.zeros(k, n, dtype=torch.float64).index_add_(0, lab_c, X.double())
    torch.testing.assert_close(sums.cpu(), ref_s, rtol=1e-5, atol=1e-3)
    assert torch.equal(counts.cpu(), torch.bincount(lab_c, minlength=k))
    assert abs(float(inertia.item()) - float(dist.double().sum())) <= 1e-6 * float(dist.double().sum()) + 1e-6
    # search-only mode (nearest_centroid routes here) gives the same labels
    l2, _ = ops.nearest_centroid(Xd, Cd)
    assert torch.equal(l2.cpu(), lab.cpu())


def _rf_setup(dev, m=5000, n=40, B=32, C=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(m, n, generator=g)
    sample = torch.sort(X[torch.randperm(m, generator=g)[:1000]], 0).values
    edges = sample[torch.linspace(30, 970, B - 1).long()].T.contiguous()
    y = torch.randint(0, C, (m,), generator=g).float()
    return X, edges, y


def test_rf_quantize(gpu_device):
    X, edges, _ = _rf_setup(gpu_device)
    ref = ops.rf_quantize(X, edges)
    got = ops.rf_quantize(X.to(gpu_device), edges.to(gpu_device)).cpu()
    assert torch.equal(ref, got)


@pytest.mark.parametrize("m,n,nedges", [(3000, 37, 127), (1025, 70, 31), (5000, 33, 255), (700, 5, 1)])
def test_rf_quantize_shapes(gpu_device, m, n, nedges):
    g = torch.Generator().manual_seed(m + n)
    X = torch.randn(m, n, generator=g)
    X[::7, 3 % n] = 0.25  # ties with edges
    edges = torch.sort(torch.randn(n, nedges, generator=g), 1).values
    edges[:, nedges // 2] = 0.25
    ref = ops.rf_quantize(X, edges)
    got = ops.rf_quantize(X.to(gpu_device), edges.to(gpu_device)).cpu()
    assert torch.equal(ref, got)


@pytest.mark.parametrize("k,n,nq", [(16384, 300, 127), (10000, 64, 31), (32768, 9, 255), (1000, 3, 127), (1, 4, 7)])
def test_rf_quantiles(gpu_device, k, n, nq):
    g = torch.Generator().manual_seed(k + n)
    S = torch.randn(k, n, generator=g)
    S[::3, 0] = 1.5  # heavy ties
    ref = ops.rf_quantiles(S, nq)
    got = ops.rf_quantiles(S.to(gpu_device), nq).cpu()
    assert torch.equal(ref, got)


@pytest.mark.parametrize("regression", [False, True])
def test_rf_hist_split_route(gpu_device, regression):
    X, edges, y = _rf_setup(gpu_device)
    if regression:
        y = X[:, 0] * 2 + 0.1 * torch.randn(X.shape[0], generator=torch.Generator().manual_seed(5))
    S = 2 if regression else 3
    B = edges.shape[1] + 1
    bins = ops.rf_quantize(X, edges)
    m = X.shape[0]
    w = torch.randint(0, 3, (m,), generator=torch.Generator().manual_seed(1)).to(torch.uint8)
    idx = torch.nonzero(w).view(-1).int()
    # two nodes: first 60% / rest of the in-bag rows
    cut = int(0.6 * idx.shape[0])
    fb = ops.rf_hist_fb(B, S, regression)
    nf = fb + 4  # two feature chunks, the second one partial
    feats = torch.stack([torch.randperm(40, generator=torch.Generator().manual_seed(s))[:nf] for s in (2, 3)]).int()
    items = []
    for node, (rb, re) in enumerate([(0, cut), (cut, idx.shape[0])]):
        for r0 in range(rb, re, 1000):
            for fc in range((nf + fb - 1) // fb):
                items.append((node, r0, min(re, r0 + 1000), fc))
    items = torch.tensor(items, dtype=torch.int32)
    ref = ops.rf_hist(bins, idx, y, w, items, feats, 2, B, S, regression)
    got = ops.rf_hist(bins.to(gpu_device), idx.to(gpu_device), y.to(gpu_device), w.to(gpu_device),
                      items.to(gpu_device), feats.to(gpu_device), 2, B, S, regression).cpu()
    torch.testing.assert_close(got.double(), ref.double(), rtol=1e-5, atol=1e-3)
    crit = 2 if regression else 0
    o_ref, t_ref = ops.rf_best_split(ref, B, S, regression, crit, 1.0, 0.0)
    o_got, t_got = ops.rf_best_split(got.to(gpu_device), B, S, regression, crit, 1.0, 0.0)
    torch.testing.assert_close(t_got.cpu(), t_ref, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(o_got.cpu()[:, 0], o_ref[:, 0], rtol=1e-5, atol=1e-8)
    assert torch.equal(o_got.cpu()[:, 1:3], o_ref[:, 1:3])
    seg = torch.cat([torch.zeros(cut, dtype=torch.int32), torch.ones(idx.shape[0] - cut, dtype=torch.int32)])
    nf = torch.tensor([int(feats[0, int(o_ref[0, 1])]), -1], dtype=torch.int32)
    nb = torch.tensor([int(o_ref[0, 2]), 0], dtype=torch.int32)
    cb = torch.tensor([0, 0], dtype=torch.int32)
    k_ref = ops.rf_route(bins, idx, seg, nf, nb, cb)
    k_got = ops.rf_route(bins.to(gpu_device), idx.to(gpu_device), seg.to(gpu_device), nf.to(gpu_device),
                         nb.to(gpu_device), cb.to(gpu_device)).cpu()
    assert torch.equal(k_ref, k_got)


def test_rf_predict(gpu_device):
    from spark_rapids_ml_nai_amd.models.forest import pack_forest

    trees = [
        {"feature": [0, -1, 1, -1, -1], "threshold": [0.0, 0, 0.5, 0, 0], "left": [1, -1, 3, -1, -1],
         "right": [2, -1, 4, -1, -1], "value": [[0, 0], [1, 0], [0, 0], [0.2, 0.8], [0, 1]]},
        {"feature": [1, -1, -1], "threshold": [-0.3, 0, 0], "left": [1, -1, -1], "right": [2, -1, -1],
         "value": [[0, 0], [0.6, 0.4], [0.1, 0.9]]},
    ]
    X = torch.randn(1000, 3, generator=torch.Generator().manual_seed(0))
    pc = pack_forest(trees, 2, torch.device("cpu"))
    pg = pack_forest(trees, 2, gpu_device)
    r_ref, l_ref = ops.rf_predict(X, pc["roots"], pc["feature"], pc["threshold"], pc["left"], pc["right"],
                                  pc["value_off"], pc["values"], 2, True)
    r_got, l_got = ops.rf_predict(X.to(gpu_device), pg["roots"], pg["feature"], pg["threshold"], pg["left"],
                                  pg["right"], pg["value_off"], pg["values"], 2, True)
    torch.testing.assert_close(r_got.cpu(), r_ref)
    assert torch.equal(l_got.cpu(), l_ref)
    r_n, l_n = ops.rf_predict(X.to(gpu_device), pg["roots"], pg["feature"], pg["threshold"], pg["left"],
                              pg["right"], pg["value_off"], pg["values"], 2, True, nodes=pg["nodes"])
    torch.testing.assert_close(r_n.cpu(), r_ref)
    assert torch.equal(l_n.cpu(), l_ref)


def _random_tree(rng, n, S, depth):
    feat, thr, left, right, val = [], [], [], [], []

    def grow(d):
        i = len(feat)
        feat.append(-1); thr.append(0.0); left.append(-1); right.append(-1)
        val.append(list(rng.random(S)))
        if d < depth and rng.random() < 0.85:
            feat[i] = int(rng.integers(0, n)); thr[i] = float(rng.normal())
            left[i] = grow(d + 1)
            right[i] = grow(d + 1)
        return i

    grow(0)
    return {"feature": feat, "threshold": thr, "left": left, "right": right, "value": val}


@pytest.mark.parametrize("ntrees,S,depth", [(50, 2, 8), (130, 20, 6), (7, 1, 12)])
def test_rf_predict_nodes_random_forest(gpu_device, ntrees, S, depth):
    from spark_rapids_ml_nai_amd.models.forest import pack_forest

    rng = np.random.default_rng(ntrees)
    n = 40
    trees = [_random_tree(rng, n, S, depth) for _ in range(ntrees)]
    X = torch.randn(3000, n, generator=torch.Generator().manual_seed(1))
    pc = pack_forest(trees, S, torch.device("cpu"))
    pg = pack_forest(trees, S, gpu_device)
    r_ref, l_ref = ops.rf_predict(X, pc["roots"], pc["feature"], pc["threshold"], pc["left"], pc["right"],
                                  pc["value_off"], pc["values"], S, True)
    r_got, l_got = forest_predict_gpu(X.to(gpu_device), pg, S)
    torch.testing.assert_close(r_got.cpu(), r_ref, rtol=1e-5, atol=1e-4)
    assert torch.equal(l_got.cpu(), l_ref)


def forest_predict_gpu(X, packed, S):
    from spark_rapids_ml_nai_amd.models.forest import forest_predict

    return forest_predict(X, packed, S, want_leaves=True)


@pytest.mark.parametrize("mq,mi,n,k", [(1, 50, 3, 5), (300, 5000, 17, 10), (1000, 20000, 128, 64), (129, 300, 256, 1),
                                       (64, 100, 130, 100)])
def test_knn(gpu_device, mq, mi, n, k):
    Q = _rand(mq, n, gpu_device, seed=11)
    I = _rand(mi, n, gpu_device, seed=12)
    d, i = ops.knn(Q, I, k)
    kk = min(k, mi)
    ref = torch.cdist(Q.double().cpu(), I.double().cpu()) ** 2
    rv, _ = torch.topk(ref, kk, dim=1, largest=False)
    assert d.shape == (mq, kk) and i.shape == (mq, kk)
    scale = ref.max().item()
    assert (d.cpu().double() - rv).abs().max().item() / scale < 1e-5
    # the returned ids really are at the returned distances
    got = ref.gather(1, i.cpu())
    assert (got - rv).abs().max().item() / scale < 1e-5
    srt = i.cpu().sort(dim=1).values
    assert bool((srt[:, 1:] != srt[:, :-1]).all())


def test_knn_id_offset(gpu_device):
    Q = _rand(70, 8, gpu_device, seed=3)
    I = _rand(900, 8, gpu_device, seed=4)
    _, i0 = ops.knn(Q, I, 7)
    _, i1 = ops.knn(Q, I, 7, id_offset=1000)
    assert torch.equal(i0 + 1000, i1)


@pytest.mark.parametrize("n,nlist,nprobe,k", [(16, 10, 3, 10), (130, 32, 8, 5), (3, 5, 5, 64), (128, 40, 6, 10),
                                              (64, 20, 4, 7), (33, 12, 3, 1), (32, 16, 4, 100), (96, 8, 2, 700)])
def test_ivf_search(gpu_device, n, nlist, nprobe, k):
    from spark_rapids_ml_nai_amd.models.knn import build_ivf

    X = _rand(4000, n, gpu_device, seed=21)
    ids = torch.arange(4000, device=gpu_device) * 3
    index = build_ivf(X, ids, nlist, seed=1, iters=5)
    Q = _rand(257, n, gpu_device, seed=22)
    qn = ops.row_sqnorm(Q)
    _, probes = ops.knn(Q, index.centroids, nprobe)
    d, gi = ops.ivf_search(Q, probes.int(), index.list_off, index.items, index.inorm, index.ids, k, qnorm=qn)
    # oracle: brute force over exactly the probed lists (CPU torch path)
    dc, ic = ops.ivf_search(Q.cpu(), probes.cpu(), index.list_off.cpu(), index.items.cpu(), index.inorm.cpu(),
                            index.ids.cpu(), k, qnorm=qn.cpu())
    fin = torch.isfinite(dc)
    assert torch.equal(fin, torch.isfinite(d.cpu()))
    scale = dc[fin].abs().max().item()
    assert (d.cpu()[fin] - dc[fin]).abs().max().item() / scale < 1e-5
    assert (gi.cpu()[fin] == ic[fin]).float().mean().item() > 0.99


@pytest.mark.parametrize("N,n,nlist,nprobe,k", [(3000, 16, 12, 4, 15), (5000, 128, 20, 6, 10), (700, 7, 3, 3, 64),
                                                (2000, 130, 9, 2, 5), (3000, 24, 10, 3, 150), (1500, 65, 6, 4, 600)])
def test_knn_lists(gpu_device, N, n, nlist, nprobe, k):
    """IVF-list all-points kNN tile kernel vs brute force over exactly the probed lists."""
    from spark_rapids_ml_nai_amd.models.knn_graph import ivf_tiles

    X = _rand(N, n, gpu_device, seed=31)
    g = torch.Generator().manual_seed(N)
    lab = torch.randint(0, nlist, (N,), generator=g).to(gpu_device)
    order = torch.argsort(lab, stable=True)
    counts = torch.bincount(lab, minlength=nlist)
    off = torch.zeros(nlist + 1, dtype=torch.int64, device=gpu_device)
    off[1:] = torch.cumsum(counts, 0)
    Xs = X[order].contiguous()
    xn = ops.row_sqnorm(Xs)
    rows = []
    for c in range(nlist):  # own list first, then distinct random others
        others = [j for j in torch.randperm(nlist, generator=g).tolist() if j != c][: nprobe - 1]
        rows.append([c] + others)
    probes = torch.tensor(rows, dtype=torch.int32, device=gpu_device)
    tq, tl = ivf_tiles(counts, off)
    # a strict subset of the tiles, as one rank of a distributed build would launch
    sel = slice(1, None) if tq.shape[0] > 1 else slice(0, None)
    d, i = ops.knn_lists(Xs, xn, off, probes, tq[sel], tl[sel], k)
    dc, ic = ops.knn_lists(Xs.cpu(), xn.cpu(), off.cpu(), probes.cpu(), tq[sel].cpu(), tl[sel].cpu(), k)
    d, i = d.cpu(), i.cpu()
    fin = torch.isfinite(dc)
    assert torch.equal(fin, torch.isfinite(d))
    assert torch.equal(ic[~fin], i[~fin])
    scale = dc[fin].abs().max().item()
    assert (d[fin] - dc[fin]).abs().max().item() / scale < 1e-5
    assert (i[fin] == ic[fin]).float().mean().item() > 0.99
    # untouched rows (the skipped first tile) stay +inf / -1
    if tq.shape[0] > 1:
        r1 = int(tq[1])
        assert torch.isinf(d[:r1]).all() and (i[:r1] == -1).all()


@pytest.mark.parametrize("N,n,eps", [(5, 2, 1.5), (700, 7, 2.5), (3000, 64, 9.0), (1000, 130, 14.0)])
def test_dbscan_kernels(gpu_device, N, n, eps):
    g = torch.Generator().manual_seed(N)
    C = torch.randn(6, n, generator=g) * 6
    X = (C[torch.randint(0, 6, (N,), generator=g)] + torch.randn(N, n, generator=g)).float()
    Xg = X.to(gpu_device)
    xn, xng = ops.row_sqnorm(X), ops.row_sqnorm(Xg)
    T = ops.dbscan_num_tiles(N)
    eps2 = eps * eps
    cnt_ref = ops.dbscan_degree(X, xn, eps2, 0, T)
    # two tile ranges accumulate like two ranks
    cnt = ops.dbscan_degree(Xg, xng, eps2, 0, T // 2)
    ops.dbscan_degree(Xg, xng, eps2, T // 2, T, cnt)
    exact = ((torch.cdist(X.double(), X.double()) ** 2) <= eps2).sum(1)
    # fp32 boundary cases may flip; they must be rare and agree between CPU and GPU paths mostly
    assert (cnt.cpu() != cnt_ref).float().mean().item() < 1e-3
    assert (cnt.cpu().long() - exact).abs().sum().item() <= max(2, N // 500)
    core = (cnt_ref >= 5).to(torch.uint8)
    p_ref = torch.arange(N, dtype=torch.int32)
    b_ref = torch.full((N,), -1, dtype=torch.int64)
    ops.dbscan_link(X, xn, eps2, 0, T, core, p_ref, b_ref)
    ops.uf_compress(p_ref)
    p = torch.arange(N, dtype=torch.int32, device=gpu_device)
    b = torch.full((N,), -1, dtype=torch.int64, device=gpu_device)
    ops.dbscan_link(Xg, xng, eps2, 0, T, core.to(gpu_device), p, b)
    ops.uf_compress(p)
    cb = core.bool()
    assert torch.equal(p.cpu()[cb], p_ref[cb])
    has = b_ref != -1
    assert torch.equal(b.cpu() != -1, has)
    # nearest core neighbour: same distance (ties may pick another index)
    if bool(has.any()):
        def _dist(k):
            return ((k >> 32) & 0x7FFFFFFF).int().view(torch.float32)

        torch.testing.assert_close(_dist(b.cpu()[has]), _dist(b_ref[has]), rtol=1e-3, atol=1e-3 * eps2)


def test_uf_unite_pairs(gpu_device):
    N = 10000
    g = torch.Generator().manual_seed(0)
    a = torch.arange(N, dtype=torch.int32)
    other = torch.where(torch.rand(N, generator=g) < 0.5, torch.randint(0, N, (N,), generator=g).int(), a)
    other = torch.minimum(other, a)  # forest: parents point to smaller indices
    p_ref = a.clone()
    ops.uf_unite_pairs(p_ref, other)
    ops.uf_compress(p_ref)
    p = a.clone().to(gpu_device)
    ops.uf_unite_pairs(p, other.to(gpu_device))
    ops.uf_compress(p)
    assert torch.equal(p.cpu(), p_ref)


@pytest.mark.parametrize("dim", [2, 3, 5])
def test_umap_epoch_attraction(gpu_device, dim):
    # disjoint edges (2i -> 2i+1), no negative samples: the GPU update must equal the CPU reference
    N = 2000
    g = torch.Generator().manual_seed(dim)
    emb = torch.rand(N, dim, generator=g) * 10
    head = torch.arange(0, N, 2, dtype=torch.int32)
    tail = head + 1
    E = head.numel()
    eps = torch.ones(E)
    eps_neg = torch.zeros(E)
    args = dict(a=1.577, b=0.895, gamma=1.0, alpha=0.7, epoch=1, move_other=True, seed=3)
    e_cpu = emb.clone()
    ops.umap_epoch(head, tail, eps, eps.clone(), torch.zeros(E), eps_neg, e_cpu, e_cpu, **args)
    e_gpu = emb.clone().to(gpu_device)
    ops.umap_epoch(head.to(gpu_device), tail.to(gpu_device), eps.to(gpu_device), eps.clone().to(gpu_device),
                   torch.zeros(E, device=gpu_device), eps_neg.to(gpu_device), e_gpu, e_gpu, **args)
    torch.testing.assert_close(e_gpu.cpu(), e_cpu, rtol=1e-4, atol=1e-4)
    assert not torch.allclose(e_cpu, emb)


def test_umap_epoch_negative_samples(gpu_device):
    # repulsion only pushes points apart: mean pairwise spread must grow
    N, dim = 3000, 2
    g = torch.Generator().manual_seed(0)
    emb = (torch.rand(N, dim, generator=g) * 0.5).to(gpu_device)
    head = torch.arange(N, dtype=torch.int32, device=gpu_device)
    tail = torch.roll(head, 1)
    E = N
    eps = torch.ones(E, device=gpu_device)
    before = emb.std(0).sum().item()
    ops.umap_epoch(head, tail, eps, eps.clone(), torch.zeros(E, device=gpu_device), eps / 5, emb, emb,
                   a=1.577, b=0.895, gamma=1.0, alpha=1.0, epoch=1, move_other=True, seed=1)
    assert torch.isfinite(emb).all()
    assert emb.std(0).sum().item() > before


@pytest.mark.parametrize("n", [1, 5, 64, 65, 129, 200, 1000, 3000])
def test_spd_solve(gpu_device, n):
    g = torch.Generator().manual_seed(n)
    M = torch.randn(n, n + 3, generator=g, dtype=torch.float64)
    A = M @ M.T / n + 0.1 * torch.eye(n, dtype=torch.float64)
    b = torch.randn(n, generator=g, dtype=torch.float64)
    x, ok = ops.spd_solve(A.to(gpu_device), b.to(gpu_device))
    assert ok
    ref = torch.linalg.solve(A, b)
    torch.testing.assert_close(x.cpu(), ref, rtol=1e-9, atol=1e-9)


def test_spd_solve_detects_singular(gpu_device):
    n = 100
    g = torch.Generator().manual_seed(0)
    M = torch.randn(n, 10, generator=g, dtype=torch.float64)
    _, ok = ops.spd_solve((M @ M.T).to(gpu_device), torch.ones(n, dtype=torch.float64, device=gpu_device))
    assert not ok


@pytest.mark.parametrize("n", [3, 50, 130, 700, 3000])
def test_cd_gram(gpu_device, n):
    g = torch.Generator().manual_seed(n)
    M = torch.randn(4 * n, n, generator=g, dtype=torch.float64)
    A = M.T @ M / (4 * n)
    b = torch.randn(n, generator=g, dtype=torch.float64) * 0.3
    l1 = torch.full((n,), 0.05, dtype=torch.float64)
    l2 = torch.full((n,), 0.02, dtype=torch.float64)
    w_ref, it_ref = ops.cd_gram(A, b, l1, l2, 200, 1e-10)
    w, it = ops.cd_gram(A.to(gpu_device), b.to(gpu_device), l1.to(gpu_device), l2.to(gpu_device), 200, 1e-10)
    assert it == it_ref
    torch.testing.assert_close(w.cpu(), w_ref, rtol=1e-9, atol=1e-12)
    if n >= 50:
        assert (w_ref == 0).any()  # the L1 term produced exact zeros


def test_cd_gram_wide_global_memory(gpu_device):
    """n beyond the LDS-resident kernels: the block-cyclic global-memory sweeps run the same
    coordinate order as the CPU cyclic sweep (same iteration count, same solution)."""
    n = 10000
    g = torch.Generator().manual_seed(9)
    U = torch.randn(n, 40, generator=g, dtype=torch.float64)
    A = U @ U.T / 40.0 + 0.5 * torch.eye(n, dtype=torch.float64)
    b = torch.randn(n, generator=g, dtype=torch.float64) * 0.3
    l1 = torch.full((n,), 0.05, dtype=torch.float64)
    l2 = torch.full((n,), 0.02, dtype=torch.float64)
    w_ref, it_ref = ops.cd_gram(A, b, l1, l2, 25, 1e-9)
    w, it = ops.cd_gram(A.to(gpu_device), b.to(gpu_device), l1.to(gpu_device), l2.to(gpu_device), 25, 1e-9)
    assert it == it_ref
    torch.testing.assert_close(w.cpu(), w_ref, rtol=1e-8, atol=1e-11)
    assert (w_ref == 0).any()


def test_streamed_ingest_scatter_stats(gpu_device):
    from spark_rapids_ml_nai_amd.models.stats import scatter_stats
    from spark_rapids_ml_nai_amd.ops.ingest import StreamedRows, is_pinned
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    m, n = 50000, 96
    h = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
    g = torch.Generator().manual_seed(0)
    h.copy_(torch.randn(m, n, generator=g) * 3 + 7)
    Xh = h.numpy()
    assert is_pinned(Xh)
    y = torch.randn(m, generator=g, dtype=torch.float64)
    ctx = WorkerContext.single(gpu_device)
    st_ref = scatter_stats(torch.from_numpy(Xh).to(gpu_device), ctx, m, y=y.to(gpu_device))
    sr = StreamedRows(Xh, gpu_device, torch.float32, chunk_bytes=1 << 20)
    assert len(sr.bounds) > 10
    st = scatter_stats(sr.X, ctx, m, stream=sr, y=y.to(gpu_device))
    Xd = torch.from_numpy(Xh).double()
    Xc = Xd - Xd.mean(0)
    ref = Xc.T @ Xc
    scale = ref.abs().max().item()
    for s in (st, st_ref):
        assert (s.scatter.cpu() - ref).abs().max().item() / scale < 1e-6
        torch.testing.assert_close(s.mean.cpu(), Xd.mean(0), rtol=1e-7, atol=1e-7)
        ref_xty = Xd.T @ y.float().double()  # labels reach the kernel as fp32 (feature dtype)
        assert (s.xty.cpu() - ref_xty).abs().max().item() / ref_xty.abs().max().item() < 1e-6
    torch.testing.assert_close(sr.wait_all().cpu(), h)


def test_streamed_rf_binning_matches_in_memory(gpu_device):
    """RF binning under a streamed ingest (host-gathered sample rows, every row chunk quantised as
    it lands, ``rf_quantize(out=, col0=)``) gives the same edges and bins as the in-memory path."""
    from spark_rapids_ml_nai_amd.models.forest import quantize_features
    from spark_rapids_ml_nai_amd.ops.ingest import StreamedRows
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    m, n = 60001, 70  # odd row count: the last chunk and the unaligned byte-store path
    h = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
    g = torch.Generator().manual_seed(5)
    h.copy_(torch.randn(m, n, generator=g) * torch.rand(n, generator=g) * 10)
    h[:, 3] = torch.randint(0, 4, (m,), generator=g).float()  # heavy ties
    ctx = WorkerContext.single(gpu_device)
    bins_ref, edges_ref = quantize_features(torch.from_numpy(h.numpy()).to(gpu_device), 128, ctx, m, 11)
    sr = StreamedRows(h.numpy(), gpu_device, torch.float32, chunk_bytes=1 << 20)
    assert len(sr.bounds) > 10
    bins, edges = quantize_features(sr.X, 128, ctx, m, 11, stream=sr)
    np.testing.assert_array_equal(edges, edges_ref)
    assert torch.equal(bins.cpu(), bins_ref.cpu())
    # a chunk binned into the middle of a larger matrix leaves the other columns alone
    out = torch.full((n, 1000), 255, dtype=torch.uint8, device=gpu_device)
    ops.rf_quantize(sr.X[100:300], torch.from_numpy(edges).float().to(gpu_device), out=out, col0=501)
    assert torch.equal(out[:, 501:701].cpu(), bins_ref[:, 100:300].cpu())
    assert bool((out[:, :501] == 255).all()) and bool((out[:, 701:] == 255).all())


@pytest.mark.parametrize("regression", [True, False])
def test_rf_node_stats(gpu_device, regression):
    g = torch.Generator().manual_seed(3)
    m = 200000
    idx = torch.sort(torch.randperm(m, generator=g)[:150000]).values.int()
    wpos = torch.randint(1, 4, (idx.shape[0],), generator=g).float()
    y = (torch.randn(m, generator=g) * 5) if regression else torch.randint(0, 5, (m,), generator=g).float()
    bounds = torch.tensor([0, 10, 10, 5000, 70000, 149999, 150000], dtype=torch.int64)
    S = 5
    ref = ops.rf_node_stats(idx, wpos, y, bounds, S, regression)
    got = ops.rf_node_stats(idx.to(gpu_device), wpos.to(gpu_device), y.to(gpu_device), bounds.to(gpu_device), S,
                            regression).cpu()
    torch.testing.assert_close(got, ref, rtol=1e-9, atol=1e-6)


def test_uvm_managed_ingest(gpu_device, monkeypatch):
    from spark_rapids_ml_nai_amd.ops.ingest import host_to_device, managed_empty

    monkeypatch.setenv("SRML_UVM", "1")
    X = np.random.default_rng(0).standard_normal((50000, 64)).astype(np.float32)
    Xd = host_to_device(X, gpu_device, torch.float32)
    assert Xd.is_cuda
    torch.testing.assert_close(Xd.cpu(), torch.from_numpy(X))
    s, _ = ops.col_moments(Xd)  # kernels run on managed memory
    torch.testing.assert_close(s.cpu(), torch.from_numpy(X).double().sum(0), rtol=1e-5, atol=1e-3)
    t = managed_empty((1000,), torch.float32, gpu_device)
    t.fill_(2.0)
    assert float(t.sum()) == 2000.0


@pytest.mark.parametrize("m,n,k", [(1024, 3000, 257), (4099, 130, 1000), (300, 40, 5), (70000, 200, 600)])
def test_nearest_centroid_split_tiled(gpu_device, m, n, k):
    """LDS-DMA kernel on the tiled plane layout == the fp32 reference arg-min (ties within 1e-5)."""
    X = _rand(m, n, gpu_device, seed=11)
    C = _rand(k, n, gpu_device, seed=12)
    xnorm = ops.row_sqnorm(X)
    XP = ops.split_bf16x3(X, tiled=True)
    assert XP.dim() == 5
    lab, d2 = ops.nearest_centroid_split(XP, m, C, xnorm)
    D = torch.cdist(X.double(), C.double()) ** 2
    ref = D.min(1).values
    got = D.gather(1, lab.long().view(-1, 1)).view(-1)
    assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    torch.testing.assert_close(d2.double(), ref, rtol=1e-5, atol=1e-3)


def test_rf_hist_fb_matches_library(gpu_device):
    """Python's work-item builder and the loaded kernel library agree on features per item."""
    from spark_rapids_ml_nai_amd.ops import native

    lib = native.lib()
    assert int(lib.srml_rf_hist_fb_max()) == ops.RF_HIST_FB_MAX
    for B in (2, 32, 128, 256):
        for S in (2, 3, 10, 20, 32):
            for reg in (False, True):
                if reg and S != 2:
                    continue
                assert int(lib.srml_rf_hist_fb(B, S, int(reg))) == ops.rf_hist_fb(B, S, reg), (B, S, reg)
                assert int(lib.srml_rf_hist_wide_fb(B, S, int(reg))) == ops.rf_hist_fb_wide(B, S, reg), (B, S, reg)


def test_f16_plane_gather_matches_conversion(gpu_device):
    """Rows gathered from the filter's tiled fp16 plane == the same rows converted from X again
    (scale, centring, swizzle, zero padding rows)."""
    from spark_rapids_ml_nai_amd.ops import native

    g = torch.Generator(device=gpu_device).manual_seed(4)
    m, n = 3000, 200
    X = torch.randn(m, n, device=gpu_device, generator=g) * 3 + 1
    mu = X.double().mean(0).float()
    F = ops.F16Planes(X, mu)
    assert F.ok and F.P is not None
    rq = torch.randint(0, m, (777,), device=gpu_device, generator=g, dtype=torch.int32)
    nq, rp = 777, 1024
    st = native.stream(gpu_device)
    A = torch.full((rp // 256, F.kp // 16, 256, 16), 7.0, dtype=torch.float16, device=gpu_device)
    B = A.clone()
    scratch = torch.zeros(1, dtype=torch.int32, device=gpu_device)
    native.call("srml_f16_plane_gather_rows", F.P.data_ptr(), F.rows_pad, F.kp, rq.data_ptr(), nq, rp, A.data_ptr(), st)
    native.call("srml_split_f16_tiled_centered_rows", X.data_ptr(), X.stride(0), rq.data_ptr(), nq, F.n,
                F.mu.data_ptr(), F.kp, rp, F.scale, B.data_ptr(), scratch.data_ptr(), st)
    assert torch.equal(A.view(torch.int16).cpu(), B.view(torch.int16).cpu())


def test_rf_pack_wy_matches_gather(gpu_device):
    """One-pass (weight, label) packing in position order == the gather + stack it replaces."""
    g = torch.Generator().manual_seed(9)
    m, P = 5000, 123457
    idx = torch.randint(0, m, (P,), generator=g, dtype=torch.int32)
    w = torch.randint(1, 6, (P,), generator=g).float()
    y = torch.randn(m, generator=g)
    got = ops.rf_hist_wy(idx.to(gpu_device), y.to(gpu_device), None, w.to(gpu_device)).cpu()
    assert torch.equal(got, torch.stack([w, y[idx.long()]], 1))


@pytest.mark.parametrize("regression", [False, True])
def test_rf_streamed_root_level_matches_in_memory(gpu_device, monkeypatch, regression):
    """Forests on a pinned shard with the streamed ingest (chunks binned as they land, root-level
    histograms accumulated chunk by chunk) vs the in-memory path: identical classifier trees (exact
    integer counts); regressor trees of the same shape and predictions (fp64 sums in another order)."""
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier
    from spark_rapids_ml_nai_amd.regression import RandomForestRegressor

    g = torch.Generator(device=gpu_device).manual_seed(3)
    m, n = 60000, 48
    X = torch.randn(m, n, device=gpu_device, generator=g)
    score = X[:, :6].sum(1) + 0.3 * torch.randn(m, device=gpu_device, generator=g)
    y = (score if regression else (score > 0).float() + (score > 1.5).float()).double().cpu().numpy()
    Xh = datagen.to_pinned_numpy(X)
    est = (RandomForestRegressor if regression else RandomForestClassifier)(numTrees=6, maxDepth=7, maxBins=64,
                                                                           seed=5)
    monkeypatch.setenv("SRML_INGEST_CHUNK_MB", "1")  # ~48 chunks
    monkeypatch.setenv("SRML_STREAM_INGEST", "1")
    a = est.fit(DataFrame.from_numpy(Xh, y))
    monkeypatch.setenv("SRML_STREAM_INGEST", "0")
    b = est.fit(DataFrame.from_numpy(Xh, y))
    ta, tb = a._trees, b._trees
    assert len(ta) == len(tb) == 6
    for u, v in zip(ta, tb):
        assert np.asarray(u["feature"]).shape == np.asarray(v["feature"]).shape
        if not regression:
            np.testing.assert_array_equal(np.asarray(u["feature"]), np.asarray(v["feature"]))
            np.testing.assert_array_equal(np.asarray(u["threshold"]), np.asarray(v["threshold"]))
    pa = a.transform(DataFrame.from_numpy(Xh[:5000], y[:5000])).to_numpy("prediction")
    pb = b.transform(DataFrame.from_numpy(Xh[:5000], y[:5000])).to_numpy("prediction")
    if regression:
        assert np.mean(np.abs(pa - pb) <= 1e-6 * (1 + np.abs(pb))) > 0.99
    else:
        np.testing.assert_array_equal(pa, pb)


@pytest.mark.parametrize("classes,bins", [(20, 128), (12, 256), (32, 256)])
def test_rf_many_classes(gpu_device, classes, bins):
    """Histograms wider than the default 8-feature slab: fewer features per item."""
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier

    g = np.random.default_rng(classes)
    m, n = 4000, 12
    centers = g.standard_normal((classes, n)) * 3
    y = g.integers(0, classes, m)
    X = (centers[y] + g.standard_normal((m, n))).astype(np.float32)
    model = RandomForestClassifier(numTrees=4, maxDepth=8, maxBins=bins, seed=1).fit(
        DataFrame.from_numpy(X, y.astype(np.float64)))
    pred = model.transform(DataFrame.from_numpy(X, y.astype(np.float64))).to_numpy("prediction")
    assert (pred == y).mean() > 0.8


@pytest.mark.parametrize("mode", ["staged", "register"])
@pytest.mark.parametrize("src_dtype,dst", [(np.float32, torch.float32), (np.float64, torch.float32),
                                           (np.float32, torch.float64)])
def test_parts_to_device(gpu_device, mode, src_dtype, dst, monkeypatch):
    """Multi-batch pageable ingest (Spark-like record batches) lands exactly where it belongs."""
    from spark_rapids_ml_nai_amd.ops import ingest

    monkeypatch.setenv("SRML_INGEST_SLOT_MB", "1")  # many ring slots per call, blocks straddling slots
    rng = np.random.default_rng(0)
    sizes = [1, 700, 0, 1333, 257, 4096, 3]
    parts = [rng.standard_normal((s, 77)).astype(src_dtype) for s in sizes]
    got = ingest.parts_to_device(parts, gpu_device, dst, mode=mode).cpu()
    ref = torch.from_numpy(np.concatenate(parts, 0).astype(np.float32 if dst == torch.float32 else np.float64))
    assert got.dtype == dst and torch.equal(got, ref)


@pytest.mark.parametrize("nc,k", [(300, 20), (4001, 1000), (4093, 1096), (8000, 64)])
def test_kmeanspp_gram_matches_host(gpu_device, nc, k):
    """Device k-means++ seeding draws the same centres as the numpy reference (same uniforms)."""
    g = torch.Generator().manual_seed(nc)
    C = torch.randn(nc, 32, generator=g, dtype=torch.float64) * torch.rand(nc, 1, generator=g, dtype=torch.float64)
    w = torch.randint(1, 50, (nc,), generator=g).double()
    G = C @ C.T
    ref = ops.kmeanspp_gram(G, w, k, 1234)
    got = ops.kmeanspp_gram(G.to(gpu_device), w.to(gpu_device), k, 1234).cpu()
    assert got[0] == ref[0]
    assert (got == ref).float().mean().item() > 0.95  # prefix-sum order may flip a boundary draw
    assert len(set(got.tolist())) == k  # D^2 sampling never re-picks a chosen candidate


@pytest.mark.parametrize("nc,k", [(1000, 300), (4001, 1000)])
def test_kmeanspp_register_kernel_matches_block_kernel(gpu_device, monkeypatch, nc, k):
    """The register-resident k-means++ kernel (nc <= 4096, <= 8 trials; padded row stride) draws the
    same centres as the chunked block kernel on the same uniforms (only the reduction order of the
    trial potentials differs)."""
    g = torch.Generator().manual_seed(nc + 1)
    C = torch.randn(nc, 24, generator=g, dtype=torch.float64) * torch.rand(nc, 1, generator=g, dtype=torch.float64)
    w = torch.randint(1, 50, (nc,), generator=g).double().to(gpu_device)
    G = (C @ C.T).to(gpu_device)
    got = ops.kmeanspp_gram(G, w, k, 99).cpu()
    monkeypatch.setenv("SRML_KPP_KERNEL", "block")
    ref = ops.kmeanspp_gram(G, w, k, 99).cpu()
    assert got[0] == ref[0]
    assert (got == ref).float().mean().item() > 0.95
    assert len(set(got.tolist())) == k


@pytest.mark.parametrize("m,n,k", [(1024, 3000, 257), (70000, 200, 600)])
def test_nearest_centroid_split_tiled_approx(gpu_device, m, n, k):
    """3-product variant (k-means|| passes): distances within ~1e-4 relative of fp64, and the
    chosen centre is within that tolerance of the true nearest."""
    X = _rand(m, n, gpu_device, seed=13)
    C = _rand(k, n, gpu_device, seed=14)
    xnorm = ops.row_sqnorm(X)
    XP = ops.split_bf16x3(X, tiled=True)
    lab, d2 = ops.nearest_centroid_split(XP, m, C, xnorm, approx=True)
    D = torch.cdist(X.double(), C.double()) ** 2
    ref = D.min(1).values
    got = D.gather(1, lab.long().view(-1, 1)).view(-1)
    scale = (xnorm.double().view(-1) + (C.double() ** 2).sum(1).max()).max().item()
    assert (got - ref).abs().max().item() <= 1e-4 * scale
    assert (d2.double() - ref).abs().max().item() <= 1e-4 * scale


@pytest.mark.parametrize("m,n,k,ties", [(1024, 3000, 257, False), (70000, 200, 1000, False),
                                        (20000, 512, 600, True), (5000, 64, 300, True)])
def test_nearest_centroid_certified_matches_exact(gpu_device, m, n, k, ties):
    """Filter-and-refine (3-product pass + exact re-search of near ties) == the 6-product search:
    identical labels, identical distances on re-searched rows, 3-product-accurate elsewhere."""
    X = _rand(m, n, gpu_device, seed=21)
    C = _rand(k, n, gpu_device, seed=22)
    if ties:  # near-duplicate centres and rows sitting on bisectors: many sub-tolerance gaps
        C[1::2] = C[0::2][: C[1::2].shape[0]] + 1e-6 * torch.randn_like(C[1::2])
        X[: m // 4] = 0.5 * (C[0].view(1, -1) + C[2].view(1, -1)) + 1e-7 * torch.randn_like(X[: m // 4])
    mu = X.double().mean(0).float()  # the KMeans search runs on centred planes
    xnorm = ops.row_sqnorm(X, mu)
    torch.testing.assert_close(xnorm.double(), ((X.double() - mu.double()) ** 2).sum(1), rtol=1e-5, atol=1e-3)
    XP = ops.split_bf16x3(X, tiled=True, mu=mu)
    lab_e, d_e = ops.nearest_centroid_split(XP, m, C, xnorm, mu=mu)
    D = torch.cdist(X.double(), C.double()) ** 2  # translation-invariant truth
    ref = D.min(1).values
    got = D.gather(1, lab_e.long().view(-1, 1)).view(-1)
    assert (got - ref).abs().max().item() <= 1e-5 * ref.abs().max().item()
    before = dict(ops._CERTIFY_STATS)
    lab_c, d_c = ops.nearest_centroid_split(XP, m, C, xnorm, X=X, mu=mu)
    refined = ops._CERTIFY_STATS["refined"] - before["refined"]
    assert torch.equal(lab_c, lab_e)
    scale = (xnorm.double().view(-1) + ((C.double() - mu.double()) ** 2).sum(1).max()).max().item()
    assert (d_c.double() - d_e.double()).abs().max().item() <= 1e-4 * scale
    if ties:
        assert refined >= m // 4  # every bisector row was re-searched
    else:
        assert refined < m // 2  # the filter certifies most rows on generic data


@pytest.mark.parametrize("m,n,k,ties,shift", [(5000, 3000, 1000, False, 0.0), (4096, 200, 300, True, 0.0),
                                               (3000, 517, 257, False, 1e4), (2000, 64, 600, True, -3.0)])
def test_nearest_centroid_f16_certified_matches_exact(gpu_device, m, n, k, ties, shift):
    """fp16 one-product certified filter + exact re-search == the fp32-exact 6-product search:
    identical labels (incl. engineered near-ties, a large common offset and odd widths)."""
    X = _rand(m, n, gpu_device, seed=31) + shift
    C = _rand(k, n, gpu_device, seed=32) + shift
    if ties:
        C[1::2] = C[0::2][: C[1::2].shape[0]] + 1e-6 * torch.randn_like(C[1::2])
        X[: m // 4] = 0.5 * (C[0].view(1, -1) + C[2].view(1, -1)) + 1e-7 * torch.randn_like(X[: m // 4])
    mu = ops.col_moments(X, need_sq=False)[0].div_(m).float()
    F = ops.F16Planes(X, mu)
    assert F.ok and 2.0 ** 13 <= F.scale * (X - mu).abs().max().item() < 2.0 ** 14
    torch.testing.assert_close(F.xnorm.double(), ((X.double() - mu.double()) ** 2).sum(1), rtol=1e-5, atol=1e-3)
    # the plane holds fp16(s (x - mu)) in the tiled layout: undo the swizzle for a few rows
    P = F.P.float()  # [tiles][ks][256][16]
    for r in (0, 7, 8, 255 if m > 255 else m - 1):
        ks = 0
        phys = P[r // 256, ks, r % 256]
        sw = (r % 256 >> 3) & 1
        logical = torch.cat([phys[8 * sw: 8 * sw + 8], phys[8 * (sw ^ 1): 8 * (sw ^ 1) + 8]])
        want = ((X[r, :16] - mu[:16]) * F.scale).half().float()
        torch.testing.assert_close(logical[: min(16, n)], want[: min(16, n)], rtol=0, atol=0)
    before = dict(ops._CERTIFY_STATS)
    lab_f, d_f = ops.nearest_centroid_f16(F, C)
    refined = ops._CERTIFY_STATS["refined"] - before["refined"]
    # truth: fp64 distances of the fp32 centred operands every search uses, lowest index on ties
    V = (X - mu).double()
    Wc = (C.float() - mu).double()
    D = (V * V).sum(1, keepdim=True) - 2.0 * V @ Wc.T + (Wc * Wc).sum(1).view(1, -1)
    best = D.min(1).values
    got = D.gather(1, lab_f.long().view(-1, 1)).view(-1)
    scale = (V.norm(dim=1) * Wc.norm(dim=1).max()).max().item()
    assert (got - best).abs().max().item() <= 1e-11 * scale  # the exact arg-min (up to fp64 ties)
    ref = D.argmin(1).int()
    assert (lab_f == ref).float().mean().item() > 0.9999
    radius = 2.0 * ops.certify_tau16(n) * scale
    # certified rows report the filter's distance (within its radius; ||x - mu||^2 in fp32)
    assert (d_f.double() - best).abs().max().item() <= radius + 1e-4 * (V * V).sum(1).max().item()
    if ties:
        assert refined >= m // 4
    else:
        assert refined < m // 2


def test_kmeans_fit_f16_filter_matches_bf16(gpu_device, monkeypatch):
    """A k > 256 Lloyd fit on the fp16 filter gives the same centres as on the bf16 3-product filter
    (both certified: identical labels every iteration)."""
    from spark_rapids_ml_nai_amd.models.kmeans import kmeans_fit
    from spark_rapids_ml_nai_amd.parallel.context import PartitionDescriptor, WorkerContext

    X = _rand(20000, 300, gpu_device, seed=41)
    ctx = WorkerContext.single(gpu_device)
    desc = PartitionDescriptor.build(ctx, X.shape[0], X.shape[1])
    out = {}
    for mode in ("f16", "bf16"):
        monkeypatch.setenv("SRML_KMEANS_FILTER", mode)
        monkeypatch.setenv("SRML_KMEANS_SPLIT", "1")
        out[mode] = kmeans_fit(X, desc, ctx, k=300, max_iter=5, tol=0.0, seed=3, init="random")
        assert out[mode]["refined_frac"] is not None  # the certified path ran
    # both filters certify against exact searches (fp64 for f16, fp32 6-product for bf16): equal labels
    # away from fp32-level ties, hence (near-)identical centres
    np.testing.assert_allclose(out["f16"]["cluster_centers_"], out["bf16"]["cluster_centers_"], rtol=1e-6, atol=1e-6)


def test_kmeans_predict_certified_matches_exact(gpu_device, monkeypatch):
    """Large-batch k > 256 predict runs the certified split search: fp64 arg-min labels (up to
    near-ties) and the same labels as the fp32 MFMA search it replaces."""
    from spark_rapids_ml_nai_amd.models.kmeans import kmeans_predict

    g = torch.Generator(device=gpu_device).manual_seed(5)
    X = torch.randn(70000, 256, device=gpu_device, generator=g) + 3.0
    C = X[torch.randperm(70000, device=gpu_device, generator=g)[:300]] + 0.1 * torch.randn(
        300, 256, device=gpu_device, generator=g)
    st0 = dict(ops._CERTIFY_STATS)
    got = kmeans_predict(X, C)
    assert ops._CERTIFY_STATS["rows"] > st0.get("rows", 0)  # the certified path ran
    monkeypatch.setenv("SRML_KMEANS_PREDICT_SPLIT", "0")
    fp32 = kmeans_predict(X, C)
    Xd, Cd = X.double(), C.double()
    d = (Xd * Xd).sum(1, keepdim=True) - 2.0 * Xd @ Cd.T + (Cd * Cd).sum(1).view(1, -1)
    ref = d.argmin(1).int()
    assert got.dtype == torch.int32 and got.shape == (70000,)
    assert (got == ref).float().mean().item() > 0.9999
    assert (got == fp32).float().mean().item() > 0.9999


def test_ring_rows_chunks_match_host(gpu_device):
    """RingRows: every chunk seen through the 3-buffer ring equals its host rows, also when the
    consumer enqueues work that reads the chunk after the next copies were queued."""
    from spark_rapids_ml_nai_amd.ops.ingest import RingRows

    host = torch.empty((10007, 96), dtype=torch.float32).pin_memory()
    host.copy_(torch.randn(10007, 96))
    R = RingRows(host.numpy(), gpu_device, torch.float32, chunk_bytes=96 * 4 * 700, depth=3)
    assert len(R.bounds) == 15 and len(R.bufs) == 3
    sums = []
    for r0, r1, Xc in R.chunks():
        sums.append((r0, r1, (Xc.double() * 1.5).sum(1)))  # queued on the compute stream
    torch.cuda.synchronize()
    for r0, r1, s in sums:
        torch.testing.assert_close(s.cpu(), host[r0:r1].double().sum(1) * 1.5)


def test_kmeans_predict_streamed_matches(gpu_device):
    """Transform of a page-locked batch with the H2D streamed under the fp16 certified search
    (several chunks, each its own plane scale, centred on the centres' mean): the same labels as
    the one-shot device predict (both are the exact arg-min up to fp32 near-ties) and the fp64 one."""
    from spark_rapids_ml_nai_amd.models.kmeans import kmeans_predict, kmeans_predict_streamed, predict_streams

    g = np.random.default_rng(6)
    m, n, k = 70000, 192, 400
    host = torch.empty((m, n), dtype=torch.float32).pin_memory()
    host.copy_(torch.from_numpy((g.standard_normal((m, n)) + 2.0).astype(np.float32)))
    Xh = host.numpy()
    C = torch.from_numpy(Xh[g.choice(m, k, replace=False)] + 0.1 * g.standard_normal((k, n)).astype(np.float32))
    assert predict_streams(Xh, k)
    got = kmeans_predict_streamed(Xh, C, gpu_device, chunk_bytes=9 << 20)  # ~12k-row chunks: 6 of them
    X = torch.from_numpy(Xh).to(gpu_device)
    one = kmeans_predict(X, C.to(gpu_device))
    Xd, Cd = X.double(), C.double().to(gpu_device)
    ref = ((Xd * Xd).sum(1, keepdim=True) - 2.0 * Xd @ Cd.T + (Cd * Cd).sum(1).view(1, -1)).argmin(1).int()
    assert got.dtype == torch.int32 and got.shape == (m,)
    assert (got == ref).float().mean().item() > 0.9999
    assert (got == one).float().mean().item() > 0.9999
    # a multi-batch transform input (Arrow batches as ChunkedRows views, chunks never span batches)
    from spark_rapids_ml_nai_amd.core.dataframe import ChunkedRows

    parts = ChunkedRows([Xh[:30001], Xh[30001:30001], Xh[30001:65000], Xh[65000:]])
    assert predict_streams(parts, k)
    got2 = kmeans_predict_streamed(parts, C, gpu_device, chunk_bytes=9 << 20)
    assert got2.shape == (m,) and (got2 == got).float().mean().item() > 0.9999


@pytest.mark.parametrize("nseg,total", [(1, 5000), (37, 100000), (3000, 2_000_000)])
def test_rf_partition_matches_stable_sort(gpu_device, nseg, total):
    """Native prefix-count re-partition == stable sort of the child keys (positions, weights, bounds)."""
    g = torch.Generator().manual_seed(nseg)
    cuts = torch.sort(torch.randint(0, total + 1, (nseg - 1,), generator=g)).values
    bounds = torch.cat([torch.zeros(1, dtype=torch.int64), cuts, torch.tensor([total])])
    split = torch.rand(nseg, generator=g) < 0.7
    node_feature = torch.where(split, torch.randint(0, 50, (nseg,), generator=g), torch.full((nseg,), -1)).int()
    k = int(split.sum())
    child_base = torch.zeros(nseg, dtype=torch.int32)
    child_base[split] = 2 * torch.arange(k, dtype=torch.int32)
    seg = torch.repeat_interleave(torch.arange(nseg), bounds[1:] - bounds[:-1])
    right = torch.randint(0, 2, (total,), generator=g).int()
    keys = torch.where(split[seg], child_base[seg] + right, torch.full((total,), 0x7FFFFFFF, dtype=torch.int32)).int()
    idx = torch.randperm(total, generator=g).int()
    w = torch.rand(total, generator=g)
    ri, rw, rb = ops.rf_partition(keys, bounds, node_feature, child_base, k, idx, w)
    di, dw, db = ops.rf_partition(keys.to(gpu_device), bounds.to(gpu_device), node_feature.to(gpu_device),
                                  child_base.to(gpu_device), k, idx.to(gpu_device), w.to(gpu_device))
    assert torch.equal(db.cpu(), rb) and torch.equal(di.cpu(), ri) and torch.equal(dw.cpu(), rw)


@pytest.mark.parametrize("m,k", [(0, 5), (1, 1), (5000, 7), (300001, 1000), (70000, 16000)])
def test_label_sort_stable_and_counts(gpu_device, m, k):
    """Device counting sort (srml_label_sort) == stable torch sort on the CPU; out-of-range labels
    trail after off[k]; label counts == bincount."""
    g = torch.Generator().manual_seed(m + k)
    lab = torch.randint(0, k, (m,), generator=g, dtype=torch.int32)
    if m > 10:
        lab[::97] = k + 3  # out of range: grouped after every valid row, not counted
        lab[5::211] = -2
    perm, off, slab = ops.label_sort(lab.to(gpu_device), k)
    key = torch.where((lab >= 0) & (lab < k), lab, torch.full_like(lab, k))
    ref_s, ref_p = torch.sort(key, stable=True)
    assert torch.equal(perm.cpu().long(), ref_p)
    assert torch.equal(slab.cpu(), ref_s)
    ref_off = torch.searchsorted(ref_s, torch.arange(k + 1, dtype=torch.int32))
    assert torch.equal(off.cpu(), ref_off.long())
    cnt = ops.label_counts(lab.to(gpu_device), k)
    ok = lab[(lab >= 0) & (lab < k)].long()
    assert torch.equal(cnt.cpu(), torch.bincount(ok, minlength=k))


@pytest.mark.parametrize("n,bits", [(2, 3), (1000, 8), (100003, 20), (300000, 49), (65536, 64)])
def test_radix_sort_pairs_stable(gpu_device, n, bits):
    """srml_radix_sort_u64 == stable torch sort (keys < 2^bits, many duplicates)."""
    g = torch.Generator().manual_seed(n + bits)
    hi = min(bits, 62)
    keys = torch.randint(0, 1 << hi, (n,), generator=g, dtype=torch.int64)
    keys[::3] = keys[0]  # duplicates: stability visible through the payload
    if bits == 64:
        keys[1::7] = -5  # the full 64-bit range: negative int64 = large u64
    vals = torch.arange(n, dtype=torch.int32)
    k, v = keys.to(gpu_device), vals.to(gpu_device)
    ops.radix_sort_pairs(k, v, bits)
    ku = keys.clone()
    if bits == 64:  # compare as unsigned: flip the sign bit
        ku = ku ^ (-(1 << 63))
    ref_k, ref_o = torch.sort(ku, stable=True)
    if bits == 64:
        ref_k = ref_k ^ (-(1 << 63))
    assert torch.equal(k.cpu(), ref_k)
    assert torch.equal(v.cpu(), vals[ref_o])


@pytest.mark.parametrize("mq,n,k,ip", [(1, 3, 1, False), (777, 128, 15, False), (300, 1000, 64, True),
                                       (129, 65, 40, False), (200, 3001, 33, False), (150, 2048, 64, True)])
def test_knn_refine_sort_matches_torch(gpu_device, mq, n, k, ip):
    """Fused exact re-score + per-row sort of kNN candidates == fp64 torch oracle (-1 = missing)."""
    g = torch.Generator().manual_seed(mq + n + k)
    Q = torch.randn(mq, n, generator=g)
    X = torch.randn(500, n, generator=g)
    pos = torch.randint(0, 500, (mq, k), generator=g)
    pos[::5, -1] = -1
    X[7] = Q[0] + 1e-4  # a near-duplicate: the direct difference keeps its digits
    pos[0, 0] = 7
    r = ops.knn_refine_sort(Q.to(gpu_device), X.to(gpu_device), pos.to(gpu_device), inner_product=ip)
    assert r is not None
    d, p = r[0].cpu(), r[1].cpu()
    rows = X.double()[pos.clamp_min(0)]
    ref = -2.0 * (rows * Q.double().unsqueeze(1)).sum(-1) if ip else ((rows - Q.double().unsqueeze(1)) ** 2).sum(-1)
    ref = torch.where(pos >= 0, ref, torch.full_like(ref, float("inf")))
    rv, rj = torch.sort(ref, dim=1, stable=True)
    fin = torch.isfinite(rv)
    torch.testing.assert_close(d[fin].double(), rv[fin], rtol=1e-5, atol=1e-4)
    assert torch.equal(torch.isinf(d), ~fin)
    # the same multiset of candidates per row, ordered by distance (ties aside)
    assert torch.equal(p.sort(1).values, pos.sort(1).values)
    if not ip:
        assert d[0, 0].item() < n * 2e-8 and p[0, 0].item() == 7


@pytest.mark.parametrize("T,m,rate", [(1, 1000, 1.0), (30, 100003, 1.0), (7, 5000, 0.3)])
def test_rf_bootstrap_matches_cpu_draw(gpu_device, T, m, rate):
    """Native Poisson bagging (count / scan / scatter) == the numpy draw of the same counter-based
    RNG: identical in-bag rows, multiplicities and tree bounds."""
    i_g, w_g, b_g = ops.rf_bootstrap(T, m, rate, 1234567, gpu_device)
    i_c, w_c, b_c = ops.rf_bootstrap(T, m, rate, 1234567, torch.device("cpu"))
    np.testing.assert_array_equal(b_g, b_c)
    assert torch.equal(i_g.cpu(), i_c) and torch.equal(w_g.cpu(), w_c)


@pytest.mark.parametrize("m,n,nr", [(5000, 3000, 777), (1000, 130, 1000), (300, 64, 1)])
def test_split_rows_matches_gathered_split(gpu_device, m, n, nr):
    """Tiled centred planes read through a row index list == the planes of the gathered copy."""
    X = _rand(m, n, gpu_device, seed=51)
    mu = X.double().mean(0).float()
    g = torch.Generator(device="cpu").manual_seed(nr)
    rows = torch.randperm(m, generator=g)[:nr].to(gpu_device).int()
    got = ops.split_bf16x3_rows(X, rows, mu)
    ref = ops.split_bf16x3(X.index_select(0, rows.long()), tiled=True, mu=mu)
    assert got.shape == ref.shape and torch.equal(got.view(torch.int16), ref.view(torch.int16))


def test_nearest_centroid_f16_approx_mode(gpu_device):
    """k-means|| mode (radius 0): the filter's own arg-min — distances within the certified radius
    of the exact ones, labels equal wherever the exact gap exceeds twice that radius."""
    m, n, k = 20000, 700, 513
    X = _rand(m, n, gpu_device, seed=61)
    C = X[torch.randperm(m, generator=torch.Generator().manual_seed(3))[:k].to(gpu_device)] + 0.01
    mu = ops.col_moments(X, need_sq=False)[0].div_(m).float()
    F = ops.F16Planes(X, mu)
    lab_a, d_a = ops.nearest_centroid_f16(F, C, approx=True)
    Xd, Cd = X.double() - mu.double(), C.double() - mu.double()
    D = (Xd * Xd).sum(1, keepdim=True) - 2.0 * Xd @ Cd.T + (Cd * Cd).sum(1).view(1, -1)
    top2 = D.topk(2, dim=1, largest=False).values
    radius = 2.0 * ops.certify_tau16(n) * Xd.norm(dim=1) * Cd.norm(dim=1).max()
    got = D.gather(1, lab_a.long().view(-1, 1)).view(-1)
    assert ((got - top2[:, 0]) <= 2.0 * radius + 1e-6).all()  # never worse than the radius allows
    clear = (top2[:, 1] - top2[:, 0]) > 2.0 * radius
    assert torch.equal(lab_a[clear].long(), D.argmin(1)[clear])
    assert (d_a.double() - top2[:, 0]).abs().max().item() <= radius.max().item() + 1e-6


@pytest.mark.parametrize("m,n,rb", [(4096, 3000, 64), (1000, 70, 32), (1003, 130, 64), (20000, 64, 32)])
def test_rf_interleave_record_layout(gpu_device, m, n, rb):
    """Record layout from the feature-major bins (four-rows-per-thread kernel when m % 4 == 0, the
    row-per-thread one otherwise) == the layout built on the host byte by byte."""
    g = torch.Generator().manual_seed(m + n)
    bins = torch.randint(0, 256, (n, m), generator=g, dtype=torch.uint8)
    got = ops.rf_interleave(bins.to(gpu_device), rb).cpu().numpy()
    G = (n + rb - 1) // rb
    b = np.zeros((G * rb, m), dtype=np.uint8)
    b[:n] = bins.numpy()
    rec = b.reshape(G, rb, m).transpose(0, 2, 1)  # [group][row][rb]
    for gi in range(G):  # record (g, r) at the kernel's byte offset (64-B records line-paired)
        r = np.arange(m)
        off = ((gi >> 1) * m + r) * 128 + (gi & 1) * 64 if rb == 64 else (gi * m + r) * rb
        got_g = got[off[:, None] + np.arange(rb)[None, :]]
        np.testing.assert_array_equal(got_g, rec[gi])


def test_cluster_delta_sums_one_sort(gpu_device):
    """cluster_delta_sums (one label sort, leaving rows as ~row subtracted) == sums by the new labels
    minus sums by the old labels of the moved rows."""
    X = _rand(20000, 301, gpu_device, seed=72)
    g = torch.Generator().manual_seed(9)
    rows = torch.randperm(20000, generator=g)[:1500].to(gpu_device)
    old = torch.randint(0, 50, (1500,), generator=g).to(gpu_device)
    new = (old + 1 + torch.randint(0, 49, (1500,), generator=g).to(gpu_device)) % 50
    ds, dc = ops.cluster_delta_sums(X, rows, new, old, 50)
    Xr = X.double().cpu()[rows.cpu()]
    ref = torch.zeros(50, 301, dtype=torch.float64).index_add_(0, new.cpu(), Xr).index_add_(0, old.cpu(), -Xr)
    torch.testing.assert_close(ds.cpu(), ref, rtol=1e-5, atol=1e-4)
    assert torch.equal(dc.cpu(), torch.bincount(new.cpu(), minlength=50) - torch.bincount(old.cpu(), minlength=50))


def test_kmeans_delta_sums_match_full_sums(gpu_device, monkeypatch):
    """Lloyd sums updated from the moved rows only (+x new cluster, -x old) give the same centres
    as recomputing every iteration's sums from all rows."""
    from spark_rapids_ml_nai_amd.models import kmeans as km
    from spark_rapids_ml_nai_amd.parallel.context import PartitionDescriptor, WorkerContext

    X = _rand(30000, 300, gpu_device, seed=71)
    ctx = WorkerContext.single(gpu_device)
    desc = PartitionDescriptor.build(ctx, X.shape[0], X.shape[1])
    monkeypatch.setenv("SRML_KMEANS_SPLIT", "1")
    out = {}
    for frac in (0.2, -1.0):
        monkeypatch.setattr(km, "DELTA_FRAC", frac)
        out[frac] = km.kmeans_fit(X, desc, ctx, k=300, max_iter=12, tol=0.0, seed=5, init="random")
    assert out[0.2]["delta_iters"] > 0 and out[-1.0]["delta_iters"] == 0
    # the sorted-segment kernel folds fp32 block partials into fp64 sums, so two groupings of the same
    # rows agree to fp32 rounding of the partials (~1e-7 of a coordinate), not bit for bit
    np.testing.assert_allclose(out[0.2]["cluster_centers_"], out[-1.0]["cluster_centers_"], rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("tol", [0.0, 1e-3])
def test_kmeans_device_bookkeeping_matches_torch_loop(gpu_device, monkeypatch, tol):
    """The fp16-filter Lloyd loop with native bookkeeping (moved-row count / compaction, in-place
    delta and full sums, fp64 inertia, device centre update + shift) gives the torch loop's centres,
    iteration count and delta schedule; the moved-row kernels match a torch oracle."""
    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.models import kmeans as km
    from spark_rapids_ml_nai_amd.parallel.context import PartitionDescriptor, WorkerContext

    X = _rand(30000, 300, gpu_device, seed=73)
    ctx = WorkerContext.single(gpu_device)
    desc = PartitionDescriptor.build(ctx, X.shape[0], X.shape[1])
    monkeypatch.setenv("SRML_KMEANS_SPLIT", "1")
    out = {}
    for book in ("1", "0"):
        monkeypatch.setenv("SRML_LLOYD_BOOK", book)
        out[book] = km.kmeans_fit(X, desc, ctx, k=300, max_iter=15, tol=tol, seed=5, init="random")
    assert out["1"]["n_iter"] == out["0"]["n_iter"]
    assert out["1"]["delta_iters"] == out["0"]["delta_iters"]
    np.testing.assert_allclose(out["1"]["cluster_centers_"], out["0"]["cluster_centers_"], rtol=1e-5, atol=2e-6)

    # the moved-row pass against torch: count, ascending compaction, +-1 count updates, sorted sums
    g = torch.Generator().manual_seed(3)
    m, k = 5000, 40
    lab = torch.randint(0, k, (m,), generator=g, dtype=torch.int32)
    prev = lab.clone()
    flip = torch.randperm(m, generator=g)[:700]
    prev[flip] = torch.randint(0, k, (700,), generator=g, dtype=torch.int32)
    Xs = torch.randn(m, 12, generator=g)
    book = ops.LloydBook(Xs.to(gpu_device), k)
    nm = book.moved(lab.to(gpu_device), prev.to(gpu_device))
    moved = torch.nonzero(lab != prev).view(-1)
    assert nm == moved.numel()
    L = torch.zeros(k * 12 + k + 1, dtype=torch.float64, device=gpu_device)
    book.delta_into(Xs.to(gpu_device), lab.to(gpu_device), prev.to(gpu_device), nm, L)
    ref_s = torch.zeros(k, 12, dtype=torch.float64)
    ref_s.index_add_(0, lab[moved].long(), Xs[moved].double())
    ref_s.index_add_(0, prev[moved].long(), -Xs[moved].double())
    ref_c = (torch.bincount(lab[moved].long(), minlength=k) - torch.bincount(prev[moved].long(), minlength=k)).double()
    torch.testing.assert_close(L[: k * 12].view(k, 12).cpu(), ref_s, rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(L[k * 12: k * 12 + k].cpu(), ref_c, rtol=0, atol=0)
    # full pass + inertia + update
    book.full_into(Xs.to(gpu_device), lab.to(gpu_device), L)
    d2 = torch.rand(m, generator=g)
    book.inertia_into(d2.to(gpu_device), L)
    ref_full = torch.zeros(k, 12, dtype=torch.float64).index_add_(0, lab.long(), Xs.double())
    torch.testing.assert_close(L[: k * 12].view(k, 12).cpu(), ref_full, rtol=1e-5, atol=1e-5)
    assert float(L[-1]) == pytest.approx(float(d2.double().sum()), rel=1e-12)
    C = torch.randn(k, 12, dtype=torch.float64, generator=g)
    Cd = C.to(gpu_device)
    shift, inertia = book.update(L, Cd)
    cnt = torch.bincount(lab.long(), minlength=k).double()
    newC = torch.where(cnt.view(-1, 1) > 0, ref_full / cnt.clamp_min(1).view(-1, 1), C)
    torch.testing.assert_close(Cd.cpu(), newC, rtol=1e-6, atol=1e-6)
    assert shift == pytest.approx(float(((newC - C) ** 2).sum(1).max()), rel=1e-6)
    assert inertia == float(L[-1])


@pytest.mark.parametrize("pull", [False, True])
@pytest.mark.parametrize("dim", [2, 5])
def test_umap_epoch_head_runs(gpu_device, pull, dim):
    # head-sorted edges with runs of 1..150 (inside a wave and across 64-lane / block boundaries),
    # tails read from a separate table (no Hogwild read-after-write): the per-run head commit
    # (plain store or boundary atomic) must equal the CPU reference
    g = torch.Generator().manual_seed(11 + dim)
    nh, nt = 400, 700
    deg = torch.randint(1, 151, (nh,), generator=g)
    deg[::7] = 1
    head = torch.repeat_interleave(torch.arange(nh), deg).int()
    tail = torch.randint(0, nt, (head.numel(),), generator=g).int()
    E = head.numel()
    eps = torch.where(torch.rand(E, generator=g) < 0.8, torch.ones(E), torch.full((E,), 3.0))
    emb = torch.rand(nh, dim, generator=g) * 10
    embt = torch.rand(nt, dim, generator=g) * 10
    args = dict(a=1.577, b=0.895, gamma=1.0, alpha=0.7, epoch=1, move_other=False, seed=3, pull=pull)
    e_cpu = emb.clone()
    ops.umap_epoch(head, tail, eps, eps.clone(), torch.zeros(E), torch.zeros(E), e_cpu, embt.clone(), **args)
    e_gpu = emb.clone().to(gpu_device)
    ns = eps.clone().to(gpu_device)
    ops.umap_epoch(head.to(gpu_device), tail.to(gpu_device), eps.to(gpu_device), ns,
                   torch.zeros(E, device=gpu_device), torch.zeros(E, device=gpu_device), e_gpu,
                   embt.to(gpu_device), **args)
    # A run split over two waves commits from both with atomics, and the second wave may read the
    # head after the first one's commit (Hogwild, as umap-learn's parallel epochs): those heads are
    # only checked for finiteness; every run inside one wave must equal the reference exactly.
    starts = torch.cumsum(deg, 0) - deg
    one_wave = (starts // 64) == ((starts + deg - 1) // 64)
    eg = e_gpu.cpu()
    torch.testing.assert_close(eg[one_wave], e_cpu[one_wave], rtol=1e-4, atol=1e-4)
    assert bool(torch.isfinite(eg).all())
    assert int(one_wave.sum()) > 100  # (the exact check covers most heads)
    # only the due edges advanced their schedule
    torch.testing.assert_close(ns.cpu(), torch.where(eps <= 1, 2 * eps, eps))


@pytest.mark.parametrize("N,n,nlist,nprobe,k", [(3000, 16, 12, 4, 15), (6000, 128, 20, 6, 19), (900, 4, 40, 3, 1),
                                                (2500, 64, 7, 7, 32), (400, 128, 60, 2, 20)])
def test_knn_lists_f16_centred(gpu_device, N, n, nlist, nprobe, k):
    """fp16 centred IVF tile kernel: valid, duplicate-free candidates from the probed lists whose
    sets match the fp32 brute force over the same lists (fp16 ranking may swap near-ties)."""
    from spark_rapids_ml_nai_amd.models.knn_graph import ivf_tiles

    X = _rand(N, n, gpu_device, seed=37) * 3.0 + 5.0  # offset: centring must take it out
    g = torch.Generator().manual_seed(N + n)
    lab = torch.randint(0, nlist, (N,), generator=g).to(gpu_device)
    order = torch.argsort(lab, stable=True)
    counts = torch.bincount(lab, minlength=nlist)
    off = torch.zeros(nlist + 1, dtype=torch.int64, device=gpu_device)
    off[1:] = torch.cumsum(counts, 0)
    Xs = X[order].contiguous()
    xn = ops.row_sqnorm(Xs)
    C = torch.zeros(nlist, n, device=gpu_device).index_add_(0, lab[order], Xs) / counts.clamp_min(1).view(-1, 1)
    rows = []
    for c in range(nlist):
        others = [j for j in torch.randperm(nlist, generator=g).tolist() if j != c][: nprobe - 1]
        rows.append([c] + others)
    probes = torch.tensor(rows, dtype=torch.int32, device=gpu_device)
    tq, tl = ivf_tiles(counts, off)
    assert ops.knn_lists_f16_ok(Xs, k, C)
    d, i = ops.knn_lists(Xs, xn, off, probes, tq, tl, k, centroids=C)
    dc, ic = ops.knn_lists(Xs.cpu(), xn.cpu(), off.cpu(), probes.cpu(), tq.cpu(), tl.cpu(), k)
    i, d = i.cpu(), d.cpu()
    # validity: members of the row's probed lists, no duplicates, -1 exactly where fp32 has none
    offc, prc = off.cpu(), probes.cpu()
    row_list = torch.repeat_interleave(torch.arange(nlist), counts.cpu())
    lists_of = torch.bucketize(i.clamp_min(0), offc[1:], right=True)
    allowed = (prc[row_list].unsqueeze(1) == lists_of.unsqueeze(2)).any(2)
    assert bool((allowed | (i < 0)).all())
    assert torch.equal(i < 0, ic < 0)
    srt = torch.sort(i, 1).values
    assert not bool(((srt[:, 1:] == srt[:, :-1]) & (srt[:, 1:] >= 0)).any())
    # set recall against the fp32 selection
    hit = (i.unsqueeze(2) == ic.unsqueeze(1)).any(2) & (i >= 0)
    recall = hit.sum().item() / max(1, (ic >= 0).sum().item())
    assert recall > 0.97, recall
    # ascending ranking keys
    fin = torch.isfinite(d)
    dd = torch.where(fin, d, torch.full_like(d, 3e38))
    assert bool((dd[:, 1:] >= dd[:, :-1]).all())


def test_knn_graph_ivf_f16_recall(gpu_device, monkeypatch):
    """End to end: the fp16-candidate IVF graph (extra candidates + exact re-rank) keeps the fp32
    kernel's recall against the exact graph."""
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models import knn_graph as KG

    X, _ = datagen.blobs(30000, 64, gpu_device, seed=5, centers=8)
    _, ie = KG.knn_graph_brute(X, 15)
    rec = {}
    for flag in (True, False):
        monkeypatch.setattr(ops, "KNN_LISTS_F16", flag)
        dist, idx = KG.knn_graph_ivf(X, 15, nlist=30, nprobe=6, seed=1)
        assert torch.isfinite(dist).all()
        assert bool((dist[:, 1:] >= dist[:, :-1]).all())
        rec[flag] = (idx.unsqueeze(2) == ie.unsqueeze(1)).any(2).float().mean().item()
    assert rec[True] > rec[False] - 0.005 and rec[True] > 0.9, rec


@pytest.mark.parametrize("m,n,k", [(200003, 64, 20), (50000, 16, 7)])
def test_kmeans_device_lloyd_loop_matches_host_loop(gpu_device, m, n, k):
    """The device-resident small-k Lloyd loop (fused step + device centre update + convergence flag
    read one batch late) reproduces a host Lloyd loop (the same device search for the labels, fp64
    centre update and shift test on the host) on the same start: same centres, same iteration
    count, same inertia. The search itself is checked against fp64 by the test above."""
    from spark_rapids_ml_nai_amd.models.kmeans import _lloyd_small_loop
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    g = torch.Generator().manual_seed(m)
    Ct = torch.randn(k, n, generator=g) * 3
    X = (Ct[torch.randint(0, k, (m,), generator=g)] + torch.randn(m, n, generator=g)).float()
    ctx = WorkerContext.single(gpu_device)
    # a start from random rows (7 fixed iterations), and one near the true centres that converges
    # within a few iterations (a random start can drift for hundreds of iterations on near-ties,
    # where two fp32 searches may part ways)
    starts = ((X[torch.randperm(m, generator=g)[:k]].double(), 7, 1e-30),
              ((Ct + 0.3 * torch.randn(k, n, generator=g)).double(), 200, 1e-4))
    for C0, max_iter, tol in starts:
        C, it, inertia = _lloyd_small_loop(X.to(gpu_device), C0.to(gpu_device), ctx, k, max_iter, tol * tol)
        Xd, Ch = X.double(), C0.clone()
        ref_it = 0
        for _ in range(max_iter):
            ref_it += 1
            lab = ops.kmeans_lloyd_small(X.to(gpu_device), Ch.float().to(gpu_device), with_sums=False)[0].long().cpu()
            cnt = torch.bincount(lab, minlength=k).double()
            S = torch.zeros(k, n, dtype=torch.float64).index_add_(0, lab, Xd)
            newC = torch.where(cnt.view(-1, 1) > 0, S / cnt.clamp_min(1).view(-1, 1), Ch)
            shift = float(((newC - Ch) ** 2).sum(1).max())
            ref_inertia = float(((Xd - Ch[lab]) ** 2).sum())
            Ch = newC
            if shift <= tol * tol:
                break
        assert it == ref_it and (max_iter == 7 or it < max_iter), (it, ref_it)
        # from a random start a near-tie row or two may take the other side in one of the two
        # searches (their ||c||^2 round differently): a few rows' worth of centre movement
        tol_c = 1e-4 if max_iter > 7 else 1e-2
        torch.testing.assert_close(C.cpu(), Ch, rtol=1e-5, atol=tol_c)
        assert abs(inertia - ref_inertia) <= (1e-5 if max_iter > 7 else 1e-3) * ref_inertia


@pytest.mark.parametrize("m,n,k", [(300007, 64, 20), (40000, 12, 5)])
def test_kmeans_lloyd_step_without_row_outputs(gpu_device, m, n, k):
    """The Lloyd loop's step without per-row outputs accumulates the same sums / counts / inertia
    as the step that writes labels and distances."""
    g = torch.Generator().manual_seed(m + 7 * k)
    C = torch.randn(k, n, generator=g) * 2 + 5
    X = (C[torch.randint(0, k, (m,), generator=g)] + 1.5 * torch.randn(m, n, generator=g)).float().to(gpu_device)
    Cd = C.float().to(gpu_device)
    buf_e = torch.zeros(k * n + k + 1, dtype=torch.float64, device=gpu_device)
    buf_c = torch.zeros_like(buf_e)
    ops.kmeans_lloyd_small(X, Cd, out=buf_e)
    lab, dist, _, _, _ = ops.kmeans_lloyd_small(X, Cd, out=buf_c, rows_out=False)
    assert lab is None and dist is None
    torch.testing.assert_close(buf_c[k * n: k * n + k], buf_e[k * n: k * n + k], rtol=0, atol=0)
    torch.testing.assert_close(buf_c, buf_e, rtol=1e-9, atol=1e-6)


@pytest.mark.parametrize("m,n,k", [(300007, 64, 20), (40000, 12, 5)])
def test_kmeans_lloyd_delta_step_matches_full_step(gpu_device, m, n, k):
    """Label book of the small-k loop: a full step, then forced delta steps on the next centres
    (the sums GEMM on onehot(new) - onehot(old) of the moved rows, skipped on tiles without one).
    The running sums / counts after each equal a full step's on those centres, and the moved count
    equals the rows whose label changed."""
    g = torch.Generator().manual_seed(m + k)
    Ct = torch.randn(k, n, generator=g) * 2
    X = (Ct[torch.randint(0, k, (m,), generator=g)] + 1.5 * torch.randn(m, n, generator=g)).float().to(gpu_device)
    kn = k * n
    C64 = X[torch.randperm(m, generator=g)[:k].to(gpu_device)].double().contiguous()
    C32 = C64.float().contiguous()
    cn = (C32 * C32).sum(1).contiguous()
    flags = torch.zeros(3, dtype=torch.int32, device=gpu_device)
    book = (torch.empty(m, dtype=torch.int32, device=gpu_device), flags[2:3])
    G = torch.empty(kn + k, dtype=torch.float64, device=gpu_device)
    buf = torch.zeros(kn + k + 2, dtype=torch.float64, device=gpu_device)
    stat = torch.zeros(2, dtype=torch.float64, device=gpu_device)
    lab0 = ops.kmeans_lloyd_small(X, C32, with_sums=False)[0].clone()
    ops.kmeans_lloyd_small(X, C32, cn, out=buf, done=flags, rows_out=False, book=book)
    full0 = buf.clone()
    assert float(full0[kn + k + 1]) == 0.0  # a full step counts no moved rows
    ops.kmeans_small_update(buf, k, n, C64, C32, cn, 0.0, flags, stat, G=G)
    assert torch.equal(book[0], lab0) and int(flags[2].item()) == 1  # next: a delta step
    torch.testing.assert_close(G, full0[: kn + k], rtol=0, atol=0)
    for rnd, md in enumerate((1, 1)):  # two delta steps
        C1 = C32.clone()
        lab1 = ops.kmeans_lloyd_small(X, C1, with_sums=False)[0].clone()
        ref = torch.zeros(kn + k + 2, dtype=torch.float64, device=gpu_device)
        ops.kmeans_lloyd_small(X, C1, out=ref, rows_out=False)
        flags[2] = md  # whatever the moved count
        buf.zero_()
        ops.kmeans_lloyd_small(X, C32, cn, out=buf, done=flags, rows_out=False, book=book)
        nm = int((lab1 != lab0).sum())
        assert int(buf[kn + k + 1].item()) == nm and (rnd > 0 or nm > 0)
        ops.kmeans_small_update(buf, k, n, C64, C32, cn, 0.0, flags, stat, G=G)
        assert torch.equal(book[0], lab1)
        torch.testing.assert_close(G[kn:], ref[kn: kn + k], rtol=0, atol=0)
        torch.testing.assert_close(G[:kn], ref[:kn], rtol=1e-9, atol=1e-6 * float(ref[:kn].abs().max()))
        torch.testing.assert_close(buf[kn + k], ref[kn + k])  # the inertia is a full one
        assert int(flags[2].item()) == (1 if nm * 4 < m else 0)
        lab0 = lab1


def test_kmeans_lloyd_loop_far_from_origin(gpu_device):
    """Data offset 1e3 from the origin (spread ~1): one device Lloyd step's centres equal the fp64
    cluster means of the same labels to the data's spread precision. The MFMA kernel stages x - mu
    (mu = the start centres' mean), so its per-wave fp32 sums never carry the 1e3 offset."""
    from spark_rapids_ml_nai_amd.models.kmeans import _lloyd_small_loop
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    m, n, k = 400000, 64, 20
    g = torch.Generator().manual_seed(11)
    base = torch.randn(k, n, generator=g, dtype=torch.float64) * 3
    X = (1e3 + base[torch.randint(0, k, (m,), generator=g)] + torch.randn(m, n, generator=g, dtype=torch.float64))
    Xf = X.float()
    C0 = Xf[torch.randperm(m, generator=g)[:k]].double()
    ctx = WorkerContext.single(torch.device(gpu_device))
    C, it, _ = _lloyd_small_loop(Xf.to(gpu_device), C0.to(gpu_device), ctx, k, 1, 0.0)
    Xd = Xf.double()
    # fp64 labels (a raw-coordinate fp32 search at this offset is itself wrong: ||c||^2 ~ 6e7 rounds
    # by ~4, more than the distance gaps; the centred kernel sees the spread only)
    lab = torch.cdist(Xd, C0).argmin(1)
    cnt = torch.bincount(lab, minlength=k).double()
    S = torch.zeros(k, n, dtype=torch.float64).index_add_(0, lab, Xd)
    ref = torch.where(cnt.view(-1, 1) > 0, S / cnt.clamp_min(1).view(-1, 1), C0)
    assert it == 1
    # (a near-tie row taking the other side moves a centre by ~spread / count ~ 2e-4)
    assert float((C.cpu() - ref).abs().max()) < 1e-3


def test_dbscan_labels_match_unique_oracle(gpu_device):
    """Native label compaction (root-flag prefix scan) == the unique/searchsorted numbering."""
    g = torch.Generator().manual_seed(9)
    N = 300_001
    core = (torch.rand(N, generator=g) < 0.6).to(torch.uint8)
    # a compressed forest: every core point points at the smallest core index of its group
    grp = torch.randint(0, 5000, (N,), generator=g)
    idx = torch.arange(N)
    big = N + 1
    first = torch.full((5000,), big, dtype=torch.int64).scatter_reduce_(
        0, grp[core.bool()], idx[core.bool()], "amin", include_self=True)
    parent = torch.where(core.bool() & (first[grp] < big), first[grp], idx).int()
    best = torch.where(torch.rand(N, generator=g) < 0.5, torch.randint(0, N, (N,), generator=g),
                       torch.full((N,), -1, dtype=torch.int64))
    best = torch.where(core.bool()[best.clamp_min(0)] & (best >= 0), best, torch.full_like(best, -1))
    got = ops.dbscan_labels(parent.to(gpu_device), core.to(gpu_device), best.to(gpu_device)).cpu()
    corb, root = core.bool(), parent.long()
    nb = (best & 0xFFFFFFFF).clamp(0, N - 1)
    lab_root = torch.where(corb, root, torch.where(best != -1, root[nb], torch.full_like(root, -1)))
    roots = torch.unique(root[corb])
    ref = torch.full((N,), -1, dtype=torch.int64)
    m = lab_root >= 0
    ref[m] = torch.searchsorted(roots, lab_root[m])
    assert torch.equal(got, ref)


def _ivf_fixture(gpu_device, N, n, nlist, seed):
    X = _rand(N, n, gpu_device, seed=seed) * 3.0 + 5.0
    g = torch.Generator().manual_seed(N + n + seed)
    lab = torch.randint(0, nlist, (N,), generator=g).to(gpu_device)
    order = torch.argsort(lab, stable=True)
    counts = torch.bincount(lab, minlength=nlist)
    off = torch.zeros(nlist + 1, dtype=torch.int64, device=gpu_device)
    off[1:] = torch.cumsum(counts, 0)
    Xs = X[order].contiguous()
    C = torch.zeros(nlist, n, device=gpu_device).index_add_(0, lab[order], Xs) / counts.clamp_min(1).view(-1, 1)
    return Xs, C, counts, off, g


@pytest.mark.parametrize("N,n,nlist,p,k,seeded", [(3000, 16, 12, 4, 15, False), (6000, 128, 20, 6, 19, False),
                                                  (2500, 64, 7, 7, 32, False), (900, 4, 40, 3, 1, False),
                                                  (6000, 128, 20, 6, 19, True), (3000, 16, 12, 4, 15, True)])
def test_knn_pairs_per_query_probing(gpu_device, N, n, nlist, p, k, seeded):
    """Per-query probing, inverted (the PAIRS mode of the fp16 list kernel): every (row, list) pair
    gets the k nearest items of that list — the same sets as the fp32 torch path up to fp16
    near-ties, keys within fp16 rounding of the true squared distances, written at the pair's
    slot — with the queries gathered from anywhere in X."""
    from spark_rapids_ml_nai_amd.models.knn_graph import ivf_tiles

    Xs, C, counts, off, g = _ivf_fixture(gpu_device, N, n, nlist, 41)
    probes = torch.stack([torch.randperm(nlist, generator=g)[:p] for _ in range(N)]).int().to(gpu_device)
    flat = probes.reshape(-1)
    perm, poff, _ = ops.label_sort(flat, nlist)
    perm = perm.long()
    qrows = (perm // p).int()
    tq, tl = ivf_tiles(poff[1:] - poff[:-1], poff)
    assert ops.knn_lists_f16_ok(Xs, k, C)
    thr = None
    if seeded:  # a per-row threshold: a low quantile of the squared distances to a row sample
        smp = Xs[torch.randperm(N, generator=g)[:256].to(gpu_device)]
        thr = torch.quantile(torch.cdist(Xs, smp).pow(2), 0.02, dim=1).contiguous()
    d, i = ops.knn_pairs(Xs, off, C, poff, qrows, perm.int(), tq, tl, k, N * p, thr_row=thr)
    dc, ic = ops.knn_pairs(Xs.cpu(), off.cpu(), C.cpu(), poff.cpu(), qrows.cpu(), perm.int().cpu(), tq.cpu(), tl.cpu(),
                           k, N * p, thr_row=thr.cpu() if seeded else None)
    d, i = d.cpu(), i.cpu()
    # slot s = row * p + j holds items of list probes[row, j] only
    offc = off.cpu()
    lists_of = torch.bucketize(i.clamp_min(0).long(), offc[1:], right=True)
    want = probes.cpu().reshape(-1).long().view(-1, 1)
    assert bool(((lists_of == want) | (i < 0)).all())
    if seeded:  # fp16 keys near the threshold may land on either side of it
        assert abs(int((i >= 0).sum()) - int((ic >= 0).sum())) <= 0.01 * int((ic >= 0).sum()) + 10
        assert int((ic >= 0).sum()) < 0.9 * ic.numel()  # the threshold did cut
    else:
        assert torch.equal(i < 0, ic < 0)
    hit = (i.unsqueeze(2) == ic.unsqueeze(1)).any(2) & (i >= 0)
    assert hit.sum().item() / max(1, (ic >= 0).sum().item()) > 0.97
    # keys = fp16-rounded ||q - i||^2 of the slot's row and item
    row = torch.arange(N).repeat_interleave(p)
    ok = i >= 0
    true = ((Xs.cpu()[row].unsqueeze(1) - Xs.cpu()[i.clamp_min(0).long()]) ** 2).sum(-1)
    scale = true.max()
    err = torch.where(ok, (d - true).abs(), torch.zeros_like(d))
    assert float(err.max()) <= 2e-3 * float(scale) + 1e-3


@pytest.mark.parametrize("N,n,nlist,p,P", [(5000, 32, 40, 8, 24), (3000, 128, 25, 4, 25), (1200, 8, 64, 16, 32)])
def test_knn_pool_probes_match_cpu(gpu_device, N, n, nlist, p, P):
    """Each row's p nearest list centres among its list's pool (fp16 centred MFMA ranking of the
    pool laid out as virtual lists) equal the exact fp32 choice up to near-ties."""
    from spark_rapids_ml_nai_amd.models.knn_graph import ivf_tiles

    Xs, C, counts, off, g = _ivf_fixture(gpu_device, N, n, nlist, 43)
    cn = ops.row_sqnorm(C)
    _, pool = ops.knn(C, C, P, inorm=cn, qnorm=torch.zeros(nlist, device=gpu_device))
    tq, tl = ivf_tiles(counts, off)
    got = ops.knn_pool_probes(Xs, off, C, pool.int(), tq, tl, p, 0, N).cpu()
    ref = ops.knn_pool_probes(Xs.cpu(), off.cpu(), C.cpu(), pool.int().cpu(), tq.cpu(), tl.cpu(), p, 0, N)
    assert got.shape == ref.shape == (N, p) and bool((got >= 0).all())
    # members of the row's own list's pool, distinct
    row_list = torch.repeat_interleave(torch.arange(nlist), counts.cpu())
    assert bool((got.unsqueeze(2) == pool.cpu()[row_list].unsqueeze(1)).any(2).all())
    srt = torch.sort(got, 1).values
    assert not bool((srt[:, 1:] == srt[:, :-1]).any())
    overlap = (got.unsqueeze(2) == ref.unsqueeze(1)).any(2).float().mean().item()
    assert overlap > 0.97, overlap
    assert (got[:, 0] == ref[:, 0]).float().mean().item() > 0.97  # nearest centre first


def test_knn_graph_query_probing_recall(gpu_device):
    """End to end at a scale where list probing falls short: per-query probing (the default) beats
    probing by the list's centre at the same probe count, and reaches >= 0.95 recall."""
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models import knn_graph as KG

    X, _ = datagen.classification(120000, 64, gpu_device, seed=5, n_informative=21, n_redundant=21)
    X = X.contiguous()
    q = torch.randperm(X.shape[0], generator=torch.Generator().manual_seed(0))[:3000].to(gpu_device)
    de, ie = KG.knn_graph(X[q], X, 15)
    rec = {}
    for probe in ("list", "query"):
        dist, idx = KG.knn_graph_ivf(X, 15, nprobe=16, seed=1, probe=probe)
        assert torch.isfinite(dist).all() and bool((dist[:, 1:] >= dist[:, :-1]).all())
        rec[probe] = (idx[q].unsqueeze(2) == ie.unsqueeze(1)).any(2).float().mean().item()
    assert rec["query"] > rec["list"] + 0.05 and rec["query"] >= 0.95, rec


@pytest.mark.parametrize("seeded", [False, True])
def test_knn_pairs_precentred_items_match(gpu_device, seeded):
    """The pair search on pre-centred fp16 items (one copy per graph, plain 16-B tile copies) gives
    the per-tile-converting kernel's candidates and keys (item norms summed in another order: keys
    within a few ulps, sets equal up to exact near-ties)."""
    from spark_rapids_ml_nai_amd.models.knn_graph import ivf_tiles

    N, n, nlist, p, k = 6000, 128, 20, 6, 19
    Xs, C, counts, off, g = _ivf_fixture(gpu_device, N, n, nlist, 47)
    probes = torch.stack([torch.randperm(nlist, generator=g)[:p] for _ in range(N)]).int().to(gpu_device)
    perm, poff, _ = ops.label_sort(probes.reshape(-1), nlist)
    perm = perm.long()
    qrows = (perm // p).int()
    tq, tl = ivf_tiles(poff[1:] - poff[:-1], poff)
    thr = None
    if seeded:
        smp = Xs[torch.randperm(N, generator=g)[:256].to(gpu_device)]
        thr = torch.quantile(torch.cdist(Xs, smp).pow(2), 0.05, dim=1).contiguous()
    Xh, nr = ops.center_rows_f16(Xs, C, off)
    # the centred copy is x - C_list(x), rounded to fp16, zero past n
    row_list = torch.repeat_interleave(torch.arange(nlist, device=gpu_device), counts)
    torch.testing.assert_close(Xh[:, :n].float(), (Xs - C[row_list]).half().float(), rtol=0, atol=0)
    torch.testing.assert_close(nr, (Xh.float() ** 2).sum(1), rtol=1e-5, atol=1e-3)
    d0, i0 = ops.knn_pairs(Xs, off, C, poff, qrows, perm.int(), tq, tl, k, N * p, thr_row=thr)
    d1, i1 = ops.knn_pairs(Xs, off, C, poff, qrows, perm.int(), tq, tl, k, N * p, thr_row=thr, items_f16=(Xh, nr))
    hit = (i1.unsqueeze(2) == i0.unsqueeze(1)).any(2) & (i1 >= 0)
    assert hit.sum().item() >= 0.995 * max(1, int((i0 >= 0).sum()))
    both = (i0 == i1) & (i0 >= 0)
    torch.testing.assert_close(d1[both], d0[both], rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("m,k", [(5000, 700), (3000, 257), (777, 1800)])
def test_nearest_f16_rowloop_matches_filter_argmin(gpu_device, m, k):
    """The one-pass-per-row-tile fp16 arg-min (IVF bucketing labels) equals the top-2 filter's
    approximate arg-min, and every label is within fp16 rounding of the exact fp64 nearest centre
    (partial last centre tile, padded row tile)."""
    from spark_rapids_ml_nai_amd import ops

    X = _rand(m, 128, gpu_device, seed=m + k)
    C = X[torch.randperm(m, generator=torch.Generator().manual_seed(k))[: min(k, m)].to(gpu_device)]
    if C.shape[0] < k:
        C = torch.cat([C, C[: k - C.shape[0]] + 0.01], 0)
    F = ops.quantizer_planes(X)
    assert F is not None
    lab = ops.nearest_f16_labels(F, C)
    assert lab is not None and lab.dtype == torch.int32 and lab.shape == (m,)
    ref = ops.nearest_centroid_f16(F, C, approx=True)[0]
    assert (lab == ref).float().mean().item() > 0.999
    d = torch.cdist(X.double(), C.double()) ** 2
    exact = d.min(1).values
    got = d.gather(1, lab.long().view(-1, 1)).view(-1)
    assert bool((lab >= 0).all()) and bool((lab < k).all())
    # fp16 near-ties only: the label's distance exceeds the nearest by a small fraction of the row's scale
    assert float(((got - exact) / d.mean(1)).max()) < 5e-3
    # other widths fall back (None)
    F2 = ops.quantizer_planes(X[:, :100].contiguous())
    assert ops.nearest_f16_labels(F2, C[:, :100].contiguous()) is None
