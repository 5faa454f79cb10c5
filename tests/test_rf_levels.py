"""The random forest's level loop with one device->host copy per level (split decisions on the
device, route / partition on the candidate bound) grows exactly the trees of the two-copy loop."""
import numpy as np
import pytest

from spark_rapids_ml_nai_amd import DataFrame


def _fit(monkeypatch, one_sync: bool, regression: bool, device: str, max_leaves: int = -1):
    from spark_rapids_ml_nai_amd.models import forest

    monkeypatch.setattr(forest, "RF_ONE_SYNC", one_sync)
    g = np.random.default_rng(4)
    X = g.standard_normal((6000, 24)).astype(np.float32)
    if regression:
        from spark_rapids_ml_nai_amd.regression import RandomForestRegressor as E

        y = (X[:, 0] * 2 + np.sin(X[:, 1] * 3) + 0.1 * g.standard_normal(6000)).astype(np.float64)
    else:
        from spark_rapids_ml_nai_amd.classification import RandomForestClassifier as E

        y = ((X[:, 0] + X[:, 2] * X[:, 3]) > 0.2).astype(np.float64) + (X[:, 1] > 1.0)
    kw = dict(numTrees=6, maxDepth=7, maxBins=32, seed=3)
    est = E(**kw)
    if max_leaves > 0:
        est._backend_params["max_leaves"] = max_leaves
    return est.fit(DataFrame.from_numpy(X, y))


@pytest.mark.parametrize("regression", [False, True])
def test_one_sync_levels_match_two_sync_cpu(monkeypatch, regression):
    a = _fit(monkeypatch, False, regression, "cpu")
    b = _fit(monkeypatch, True, regression, "cpu")
    assert a.totalNumNodes == b.totalNumNodes
    fa = a.transform(DataFrame.from_numpy(np.random.default_rng(9).standard_normal((500, 24)).astype(np.float32)))
    fb = b.transform(DataFrame.from_numpy(np.random.default_rng(9).standard_normal((500, 24)).astype(np.float32)))
    np.testing.assert_array_equal(fa.to_numpy("prediction"), fb.to_numpy("prediction"))


@pytest.mark.gpu
@pytest.mark.parametrize("regression", [False, True])
def test_one_sync_levels_match_two_sync_gpu(monkeypatch, regression, gpu_device):
    a = _fit(monkeypatch, False, regression, "cuda")
    b = _fit(monkeypatch, True, regression, "cuda")
    assert a.totalNumNodes == b.totalNumNodes
    Xq = np.random.default_rng(9).standard_normal((500, 24)).astype(np.float32)
    np.testing.assert_array_equal(a.transform(DataFrame.from_numpy(Xq)).to_numpy("prediction"),
                                  b.transform(DataFrame.from_numpy(Xq)).to_numpy("prediction"))


@pytest.mark.gpu
@pytest.mark.parametrize("regression", [False, True])
def test_row_major_bins_match_feature_major_gpu(monkeypatch, regression, gpu_device):
    """Histograms gathered from the row-major copy of the bins grow the same trees."""
    from spark_rapids_ml_nai_amd.models import forest

    monkeypatch.setattr(forest, "RM_ROWS", 0.0)
    a = _fit(monkeypatch, True, regression, "cuda")
    monkeypatch.setattr(forest, "RM_ROWS", 1e12)
    b = _fit(monkeypatch, True, regression, "cuda")
    assert a.totalNumNodes == b.totalNumNodes
    Xq = np.random.default_rng(9).standard_normal((500, 24)).astype(np.float32)
    np.testing.assert_array_equal(a.transform(DataFrame.from_numpy(Xq)).to_numpy("prediction"),
                                  b.transform(DataFrame.from_numpy(Xq)).to_numpy("prediction"))


@pytest.mark.gpu
@pytest.mark.parametrize("S,B,nf,crit,min_leaf", [(2, 128, 55, 0, 1.0), (3, 32, 200, 1, 4.0), (5, 64, 17, 0, 1.0),
                                                  (2, 256, 40, 1, 1.0), (2, 128, 8, 0, 1.0), (3, 16, 1, 1, 2.0),
                                                  (2, 64, 96, 0, 1.0)])
def test_rf_node_split_matches_hist_and_best_split(S, B, nf, crit, min_leaf, gpu_device):
    """The fused small-node split (histogram in LDS + wave-parallel scan) returns exactly the records
    of rf_hist + rf_best_split and the left-child totals of the winning histogram prefix."""
    import torch

    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.models import forest

    g = torch.Generator().manual_seed(S * 1000 + nf)
    m, n, C = 60000, 300, 97
    rm = torch.randint(0, B, (m, n), generator=g, dtype=torch.uint8)
    cnt = torch.randint(0, 600, (C,), generator=g)
    cnt[3] = 1  # single-row node: no split
    cnt[5] = 2000
    starts = torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0)[:-1]])
    P = int(cnt.sum())
    assert P <= m  # positions are distinct rows
    idx = torch.randperm(m, generator=g)[:P].to(torch.int32)
    w = torch.randint(1, 4, (P,), generator=g).float()
    label = torch.randint(0, S, (m,), generator=g).float()
    feats = torch.stack([torch.randperm(n, generator=g)[:nf].sort().values for _ in range(C)]).to(torch.int32)
    dev = torch.device(gpu_device)
    rm_d, idx_d, w_d, lab_d, f_d = (t.to(dev) for t in (rm, idx, w, label, feats))
    wy = ops.rf_hist_wy(idx_d, lab_d, None, w_d)
    se = torch.stack([starts, starts + cnt], 1).to(torch.int32).to(dev)
    out_f, left_f = ops.rf_node_split(rm_d, idx_d, wy, se, f_d, B, S, crit, min_leaf, 0.0)
    fb = ops.rf_hist_fb(B, S, False)
    nfc = (nf + fb - 1) // fb
    items = torch.tensor([[c, int(starts[c]), int(starts[c] + cnt[c]), k] for c in range(C) for k in range(nfc)
                          if cnt[c] > 0], dtype=torch.int32).to(dev)
    hist = ops.rf_hist(rm_d.t().contiguous(), idx_d, lab_d, None, items, f_d, C, B, S, False, pos_weight=w_d, fb=fb)
    out_r, _ = ops.rf_best_split(hist, B, S, False, crit, min_leaf, 0.0)
    left_r = forest._left_totals(hist, out_r)
    assert torch.equal(out_f.cpu(), out_r.cpu())
    assert torch.equal(left_f.cpu(), left_r.cpu())
    assert int((out_f[:, 1] >= 0).sum()) > C // 2


@pytest.mark.gpu
@pytest.mark.parametrize("S,B,nf,crit,min_leaf", [(2, 128, 55, 0, 1.0), (3, 32, 200, 1, 4.0), (5, 64, 17, 0, 1.0),
                                                  (2, 16, 3, 1, 2.0)])
def test_rf_node_split_matches_cpu_oracle(S, B, nf, crit, min_leaf, gpu_device):
    """The fused split against a CPU oracle: numpy per-node histograms of the weighted class counts
    and the torch-CPU gini / entropy scan (``_rf_best_split_ref``). Exact ties may pick another
    (feature, bin) on the device, so the check is: same validity, the same best gain, the chosen
    split's gain equal to the maximum, and its left totals equal to the oracle histogram's prefix."""
    import torch

    from spark_rapids_ml_nai_amd import ops

    rng = np.random.default_rng(S * 31 + nf)
    m, n, C = 20000, 240, 61
    rm = rng.integers(0, B, (m, n), dtype=np.uint8)
    cnt = rng.integers(0, 400, C)
    cnt[2], cnt[7] = 1, 0
    starts = np.concatenate([[0], np.cumsum(cnt)[:-1]])
    P = int(cnt.sum())
    idx = rng.permutation(m)[:P].astype(np.int32)
    w = rng.integers(1, 4, P).astype(np.float32)
    label = rng.integers(0, S, m).astype(np.float32)
    # informative labels on a few columns so most nodes have a real best split
    label = np.where(rm[:, 5] < B // 2, label, (label + 1) % S).astype(np.float32)
    feats = np.stack([np.sort(rng.permutation(n)[:nf]) for _ in range(C)]).astype(np.int32)
    dev = torch.device(gpu_device)
    idx_d = torch.from_numpy(idx).to(dev)
    wy = ops.rf_hist_wy(idx_d, torch.from_numpy(label).to(dev), None, torch.from_numpy(w).to(dev))
    se = torch.from_numpy(np.stack([starts, starts + cnt], 1).astype(np.int32)).to(dev)
    out, left = ops.rf_node_split(torch.from_numpy(rm).to(dev), idx_d, wy, se, torch.from_numpy(feats).to(dev),
                                  B, S, crit, min_leaf, 0.0)
    out, left = out.cpu().numpy(), left.cpu().numpy()
    hist = np.zeros((C, nf, B, S), np.float64)
    for c in range(C):
        rows = idx[starts[c]: starts[c] + cnt[c]]
        ww, yy = w[starts[c]: starts[c] + cnt[c]].astype(np.float64), label[rows].astype(np.int64)
        for j in range(nf):
            np.add.at(hist[c, j], (rm[rows, feats[c, j]].astype(np.int64), yy), ww)
    ref, _ = ops._rf_best_split_ref(torch.from_numpy(hist), S, False, crit, min_leaf, 0.0)
    ref = ref.numpy()
    np.testing.assert_array_equal(out[:, 1] >= 0, ref[:, 1] >= 0)
    ok = ref[:, 1] >= 0
    assert ok.sum() > C // 2
    np.testing.assert_allclose(out[ok, 0], ref[ok, 0], rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(out[:, 5], ref[:, 5], rtol=1e-9, atol=1e-12)  # parent impurity
    for c in np.nonzero(ok)[0]:
        f, b = int(out[c, 1]), int(out[c, 2])
        lt = hist[c, f, : b + 1].sum(0)
        # the device's choice is a maximiser of the oracle's gain surface: its gain, scored by the
        # oracle on the 2-bin histogram (left | right) of exactly that split, is the best gain
        two = np.stack([lt, hist[c, f].sum(0) - lt])[None, None]
        one, _ = ops._rf_best_split_ref(torch.from_numpy(two), S, False, crit, min_leaf, 0.0)
        # its record / left totals are the oracle histogram's prefix at that bin
        np.testing.assert_array_equal(left[c], lt)
        assert out[c, 3] == lt.sum() and out[c, 4] == hist[c, 0].sum() - lt.sum()
        np.testing.assert_allclose(one[0, 0], ref[c, 0], rtol=1e-9, atol=1e-12)
    assert np.all(left[~ok] == 0)


def _fit_multi(monkeypatch, fused: bool, classes: int, crit: str, subset: str = "auto"):
    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier
    from spark_rapids_ml_nai_amd.models import forest

    monkeypatch.setattr(forest, "RM_ROWS", 1e12)
    monkeypatch.setattr(forest, "FUSED_ROWS", 1e12 if fused else 0.0)
    monkeypatch.setattr(forest, "FUSED_MIN_NODES", 1)
    monkeypatch.setattr(forest, "FUSED_MIN_NF", 1)
    g = np.random.default_rng(6)
    X = g.standard_normal((8000, 40)).astype(np.float32)
    y = (np.digitize(X[:, 0] + 0.5 * X[:, 3] * X[:, 5] + 0.3 * g.standard_normal(8000),
                     np.linspace(-1.5, 1.5, classes - 1))).astype(np.float64)
    est = RandomForestClassifier(numTrees=5, maxDepth=8, maxBins=48, seed=11, impurity=crit,
                                 minInstancesPerNode=2, featureSubsetStrategy=subset)
    return est.fit(DataFrame.from_numpy(X, y))


@pytest.mark.gpu
@pytest.mark.parametrize("classes,crit,max_rows,subset", [(2, "gini", 1 << 20, "auto"), (4, "entropy", 1 << 20, "auto"),
                                                           (3, "gini", 700, "auto"), (3, "gini", 700, "all"),
                                                           (2, "entropy", 300, "all")])
def test_fused_node_split_grows_same_forest_gpu(monkeypatch, classes, crit, max_rows, subset, gpu_device):
    """max_rows 700: nodes above it take the unfused kernels within the same level (merged by node).
    subset "all" (40 features): sibling subtraction is on, so a level that mixes fused and big
    nodes must not hand its big-node-only histogram to the next level's sibling derivation."""
    from spark_rapids_ml_nai_amd.models import forest

    monkeypatch.setattr(forest, "FUSED_MAX_ROWS", max_rows)
    a = _fit_multi(monkeypatch, False, classes, crit, subset)
    b = _fit_multi(monkeypatch, True, classes, crit, subset)
    assert a.totalNumNodes == b.totalNumNodes
    Xq = np.random.default_rng(9).standard_normal((700, 40)).astype(np.float32)
    pa = a.transform(DataFrame.from_numpy(Xq))
    pb = b.transform(DataFrame.from_numpy(Xq))
    np.testing.assert_array_equal(pa.to_numpy("prediction"), pb.to_numpy("prediction"))
    np.testing.assert_array_equal(pa.to_numpy("probability"), pb.to_numpy("probability"))


@pytest.mark.gpu
@pytest.mark.parametrize("n,m", [(37, 1007), (3000, 4101), (64, 4096), (130, 65)])
def test_rf_row_major_transpose_gpu(n, m, gpu_device):
    import torch

    from spark_rapids_ml_nai_amd import ops

    g = torch.Generator().manual_seed(n + m)
    bins = torch.randint(0, 256, (n, m), generator=g, dtype=torch.uint8)
    got = ops.rf_row_major(bins.to(gpu_device))
    assert torch.equal(got.cpu(), bins.t().contiguous())


@pytest.mark.gpu
@pytest.mark.parametrize("regression,impurity", [(False, "gini"), (False, "entropy"), (True, "variance")])
def test_native_level_bookkeeping_matches_torch_gpu(monkeypatch, regression, impurity, gpu_device):
    """The level bookkeeping in native kernels (split ranks, routing arrays, children totals,
    segment stats, packed read-back) grows the trees of the torch-op version: same structure and
    predictions, leaf values / impurities / importances to fp64 rounding."""
    from spark_rapids_ml_nai_amd.models import forest

    g = np.random.default_rng(5)
    X = g.standard_normal((5000, 20)).astype(np.float32)
    if regression:
        from spark_rapids_ml_nai_amd.regression import RandomForestRegressor as E

        y = (X[:, 0] * 2 + np.sin(X[:, 1] * 3) + 0.1 * g.standard_normal(5000)).astype(np.float64)
    else:
        from spark_rapids_ml_nai_amd.classification import RandomForestClassifier as E

        y = ((X[:, 0] + X[:, 2] * X[:, 3]) > 0.2).astype(np.float64) + (X[:, 1] > 1.0)
    models = {}
    for native_lvl in (True, False):
        monkeypatch.setattr(forest, "RF_LEVEL_NATIVE", native_lvl)
        models[native_lvl] = E(numTrees=5, maxDepth=8, maxBins=32, seed=11, impurity=impurity).fit(
            DataFrame.from_numpy(X, y))
    a, b = models[True], models[False]
    assert a.totalNumNodes == b.totalNumNodes
    Xq = g.standard_normal((400, 20)).astype(np.float32)
    pa = a.transform(DataFrame.from_numpy(Xq))
    pb = b.transform(DataFrame.from_numpy(Xq))
    np.testing.assert_allclose(pa.to_numpy("prediction"), pb.to_numpy("prediction"), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(np.asarray(a.featureImportances.toArray()), np.asarray(b.featureImportances.toArray()),
                               rtol=1e-9, atol=1e-12)
