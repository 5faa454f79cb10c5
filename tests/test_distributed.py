"""Multi-rank correctness on CPU ranks (gloo, world_size 2) through the LocalBarrierRunner —
the same worker closures that run one-rank-per-MI355X over RCCL. Oracle: the single-rank fit on
the same data (reference test strategy: multi-GPU vs single-GPU cuML, tests/test_pca.py:307-355,
tests/test_kmeans.py:257-330, tests/test_random_forest.py:322-417)."""
import warnings

import numpy as np
import pytest

from spark_rapids_ml_nai_amd import DataFrame

warnings.filterwarnings("ignore")
pytestmark = pytest.mark.dist


@pytest.fixture(autouse=True)
def _cpu(monkeypatch):
    monkeypatch.setenv("SRML_FORCE_CPU", "1")


def _data(m=2000, n=12, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((m, n)).astype(np.float32) * rng.uniform(0.5, 3, n).astype(np.float32) + 2.0
    return X


def test_pca_two_ranks():
    from spark_rapids_ml_nai_amd.feature import PCA

    X = _data()
    df = DataFrame.from_numpy(X, num_partitions=2)
    m1 = PCA(k=3, inputCol="features", num_workers=1).fit(df)
    m2 = PCA(k=3, inputCol="features", num_workers=2).fit(df)
    assert np.allclose(m1.mean, m2.mean, atol=1e-5)
    assert np.allclose(np.abs(m1.components_), np.abs(m2.components_), atol=1e-4)
    assert np.allclose(m1.explained_variance_ratio_, m2.explained_variance_ratio_, atol=1e-6)
    assert np.allclose(m1.singular_values_, m2.singular_values_, rtol=1e-5)


def test_linear_regression_two_ranks():
    from spark_rapids_ml_nai_amd.regression import LinearRegression

    X = _data(seed=1)
    y = X @ np.arange(1, 13, dtype=np.float32) + 0.5
    df = DataFrame.from_numpy(X, y, num_partitions=2)
    for kw in (dict(regParam=0.0), dict(regParam=0.1, elasticNetParam=0.0), dict(regParam=0.05, elasticNetParam=0.5)):
        a = LinearRegression(num_workers=1, **kw).fit(df)
        b = LinearRegression(num_workers=2, **kw).fit(df)
        assert np.allclose(a.coefficients.toArray(), b.coefficients.toArray(), rtol=1e-5, atol=1e-5)
        assert np.isclose(a.intercept, b.intercept, rtol=1e-5, atol=1e-4)


def test_kmeans_two_ranks():
    from spark_rapids_ml_nai_amd.clustering import KMeans

    rng = np.random.default_rng(3)
    C = rng.uniform(-20, 20, (5, 4))
    X = (C[rng.integers(0, 5, 3000)] + rng.standard_normal((3000, 4))).astype(np.float32)
    df = DataFrame.from_numpy(X, num_partitions=2)
    a = KMeans(k=5, seed=1, maxIter=50, num_workers=1).fit(df)
    b = KMeans(k=5, seed=1, maxIter=50, num_workers=2).fit(df)
    ca = np.array(sorted(a.clusterCenters(), key=lambda c: tuple(c)))
    cb = np.array(sorted(b.clusterCenters(), key=lambda c: tuple(c)))
    assert np.allclose(ca, cb, atol=1e-3)


def test_logistic_regression_two_ranks():
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    X = _data(seed=4)
    y = (X[:, 0] - 2 + 0.5 * X[:, 1] > 1.0).astype(np.float64)
    df = DataFrame.from_numpy(X, y, num_partitions=2)
    a = LogisticRegression(regParam=0.01, num_workers=1).fit(df)
    b = LogisticRegression(regParam=0.01, num_workers=2).fit(df)
    assert np.allclose(a.coefficients.toArray(), b.coefficients.toArray(), atol=1e-4)
    assert np.isclose(a.intercept, b.intercept, atol=1e-4)


@pytest.mark.parametrize("mode", ["ensemble", "data_parallel"])
def test_random_forest_two_ranks(mode):
    from sklearn.datasets import make_classification

    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier

    X, y = make_classification(n_samples=3000, n_features=10, n_informative=6, random_state=0)
    df = DataFrame.from_numpy(X.astype(np.float32), y.astype(float), num_partitions=2)
    a = RandomForestClassifier(numTrees=6, maxDepth=6, seed=7, num_workers=1).fit(df)
    b = RandomForestClassifier(numTrees=6, maxDepth=6, seed=7, num_workers=2, split_mode=mode).fit(df)
    assert b.getNumTrees == 6
    acc = lambda m: (m.transform(df).to_numpy("prediction") == y).mean()
    # reference gate: multi-worker accuracy within 0.07 of single worker
    assert abs(acc(a) - acc(b)) < 0.07


@pytest.mark.parametrize("mode", ["raise", "exit"])
def test_fault_injection_fails_whole_stage(monkeypatch, mode):
    """Barrier semantics (reference core.py:750-753, cuml_context.py:155-159): a failing rank fails
    the whole stage promptly with its error instead of leaving its peers hanging."""
    import time

    from spark_rapids_ml_nai_amd.regression import LinearRegression

    X = _data(seed=5)
    y = X[:, 0].astype(np.float64)
    df = DataFrame.from_numpy(X, y, num_partitions=2)
    monkeypatch.setenv("SRML_FAULT_RANK", "1")
    monkeypatch.setenv("SRML_FAULT_MODE", mode)
    monkeypatch.setenv("SRML_BARRIER_TIMEOUT", "120")
    t0 = time.time()
    with pytest.raises(RuntimeError) as ei:
        LinearRegression(num_workers=2).fit(df)
    assert time.time() - t0 < 100
    msg = str(ei.value)
    assert ("injected fault on rank 1" in msg) if mode == "raise" else ("exited with code" in msg)


def test_hung_rank_hits_stage_timeout(monkeypatch):
    from spark_rapids_ml_nai_amd.regression import LinearRegression

    X = _data(seed=6)
    df = DataFrame.from_numpy(X, X[:, 1].astype(np.float64), num_partitions=2)
    monkeypatch.setenv("SRML_FAULT_RANK", "0")
    monkeypatch.setenv("SRML_FAULT_MODE", "hang")
    monkeypatch.setenv("SRML_BARRIER_TIMEOUT", "15")
    with pytest.raises(RuntimeError, match="timed out"):
        LinearRegression(num_workers=2).fit(df)


def test_comm_watchdog_aborts_stuck_collective(monkeypatch):
    """A rank stuck before its collectives: its peer's watchdog aborts the communicator (reference
    nccl.abort(), common/cuml_context.py:155-159) and the stage fails fast with CommTimeout,
    long before the barrier-stage timeout."""
    import time

    from spark_rapids_ml_nai_amd.regression import LinearRegression

    X = _data(seed=8)
    df = DataFrame.from_numpy(X, X[:, 2].astype(np.float64), num_partitions=2)
    monkeypatch.setenv("SRML_FAULT_RANK", "1")
    monkeypatch.setenv("SRML_FAULT_MODE", "hang")
    monkeypatch.setenv("SRML_FAULT_HANG_S", "90")
    monkeypatch.setenv("SRML_COMM_TIMEOUT", "5")
    monkeypatch.setenv("SRML_BARRIER_TIMEOUT", "300")
    t0 = time.time()
    with pytest.raises(RuntimeError, match="exceeded 5s; communicator aborted"):
        LinearRegression(num_workers=2).fit(df)
    assert time.time() - t0 < 80


@pytest.mark.parametrize("world,classify", [(2, True), (3, True), (2, False)])
def test_random_forest_dp_reduce_scatter_identical(world, classify, monkeypatch):
    """Data-parallel forests: the node-partitioned reduce-scatter of each level's histograms (+ an
    all-gather of the per-node split records) grows the same trees as all-reducing every
    histogram, with about half the wire bytes (3 ranks: padded node counts)."""
    from sklearn.datasets import make_classification, make_regression

    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier
    from spark_rapids_ml_nai_amd.regression import RandomForestRegressor

    if classify:
        X, y = make_classification(n_samples=2400, n_features=12, n_informative=6, n_classes=3, random_state=1)
        Est = RandomForestClassifier
    else:
        X, y = make_regression(n_samples=2400, n_features=12, n_informative=6, noise=5.0, random_state=1)
        Est = RandomForestRegressor
    df = DataFrame.from_numpy(X.astype(np.float32), y.astype(float), num_partitions=world)
    models = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("SRML_RF_DP_SCATTER", flag)
        models[flag] = Est(numTrees=3, maxDepth=7, seed=3, num_workers=world, split_mode="data_parallel").fit(df)
    a, b = models["0"], models["1"]
    assert len(a._trees) == len(b._trees) == 3
    for ta, tb in zip(a._trees, b._trees):
        for key in ("feature", "threshold", "left", "right"):
            np.testing.assert_array_equal(np.asarray(ta[key]), np.asarray(tb[key]))
        np.testing.assert_allclose(np.asarray(ta["value"], dtype=float), np.asarray(tb["value"], dtype=float),
                                   rtol=1e-12, atol=1e-12)
    wa = sum(r["comm_wire_bytes"] for r in a._rank_stats)
    wb = sum(r["comm_wire_bytes"] for r in b._rank_stats)
    assert wb < 0.62 * wa, (wa, wb)


@pytest.mark.parametrize("world", [1, 2])
def test_random_forest_sibling_subtraction_identical(world, monkeypatch):
    """featureSubsetStrategy="all": from depth 1 only the smaller child of each split is
    histogrammed (and all-reduced) and the larger derived as parent - smaller; the classifier's
    integer histograms make the trees identical to building every node."""
    from sklearn.datasets import make_classification

    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier

    X, y = make_classification(n_samples=3000, n_features=10, n_informative=6, n_classes=3, random_state=2)
    df = DataFrame.from_numpy(X.astype(np.float32), y.astype(float), num_partitions=world)
    models = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("SRML_RF_SIBLING_SUB", flag)
        monkeypatch.setenv("SRML_RF_DP_SCATTER", "0")  # the baseline all-reduces every histogram
        import importlib

        import spark_rapids_ml_nai_amd.models.forest as F

        importlib.reload(F)
        models[flag] = RandomForestClassifier(numTrees=3, maxDepth=8, seed=5, featureSubsetStrategy="all",
                                              num_workers=world, split_mode="data_parallel").fit(df)
    monkeypatch.undo()
    importlib.reload(F)  # module constants back to the environment's defaults
    a, b = models["0"], models["1"]
    for ta, tb in zip(a._trees, b._trees):
        for key in ("feature", "threshold", "left", "right"):
            np.testing.assert_array_equal(np.asarray(ta[key]), np.asarray(tb[key]))
    if world > 1:
        wa = sum(r["comm_wire_bytes"] for r in a._rank_stats)
        wb = sum(r["comm_wire_bytes"] for r in b._rank_stats)
        assert wb < 0.75 * wa, (wa, wb)
