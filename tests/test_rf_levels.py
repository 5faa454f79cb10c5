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
