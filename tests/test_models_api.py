"""CPU coverage of the model-level API surface: random-forest model
accessors and quality vs scikit-learn, ML persistence round trips for every persistable
family, and the Spark-equivalent evaluators vs scikit-learn's metrics.

Reference parity: ``python/tests/test_random_forest.py`` (accessors, accuracy / RMSE bounds,
persistence), ``python/tests/test_logistic_regression.py`` (save/load), and the metric
definitions in ``python/src/spark_rapids_ml/metrics/*.py``.
"""
from __future__ import annotations

import numpy as np
import pytest
from sklearn.datasets import make_classification, make_regression
from sklearn.metrics import accuracy_score, f1_score, mean_absolute_error, mean_squared_error, r2_score, \
    roc_auc_score

from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.classification import (LogisticRegression, LogisticRegressionModel,
                                                     RandomForestClassificationModel, RandomForestClassifier)
from spark_rapids_ml_nai_amd.evaluation import (BinaryClassificationEvaluator, MulticlassClassificationEvaluator,
                                                 RegressionEvaluator)
from spark_rapids_ml_nai_amd.regression import RandomForestRegressionModel, RandomForestRegressor


DEVICES = ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.fixture(params=DEVICES)
def device(request, monkeypatch):
    """cpu: PyTorch reference path (CI); gpu: the HIP kernels on an MI355X."""
    if request.param == "cpu":
        monkeypatch.setenv("SRML_FORCE_CPU", "1")
    else:
        monkeypatch.delenv("SRML_FORCE_CPU", raising=False)
    return request.param


def _clf_data(n=1500, d=12, classes=2, seed=0):
    X, y = make_classification(n_samples=n, n_features=d, n_informative=6, n_redundant=2, n_classes=classes,
                               random_state=seed)
    return X.astype(np.float32), y.astype(np.float64)


def test_rf_classifier_accessors_and_accuracy(device):
    X, y = _clf_data()
    df = DataFrame.from_numpy(X, y)
    est = RandomForestClassifier(numTrees=8, maxDepth=6, seed=1)
    assert est.getNumTrees() == 8 and est.getMaxDepth() == 6
    model = est.fit(df)
    assert isinstance(model, RandomForestClassificationModel)
    n_trees = model.getNumTrees
    assert (n_trees() if callable(n_trees) else n_trees) == 8
    assert model.numClasses == 2
    assert len(model.trees) == 8
    assert all(t.depth <= 6 for t in model.trees)
    assert model.totalNumNodes == sum(t.numNodes for t in model.trees)
    assert list(model.treeWeights) == [1.0] * 8
    imp = np.asarray(model.featureImportances.toArray())
    assert imp.shape == (12,) and np.all(imp >= 0) and abs(imp.sum() - 1.0) < 1e-6
    s = model.toDebugString
    s = s() if callable(s) else s
    assert "Tree 0" in s or "tree 0" in s.lower()

    out = model.transform(df)
    pred = out.to_numpy("prediction")
    prob = out.to_numpy("probability")
    raw = out.to_numpy("rawPrediction")
    assert prob.shape == (1500, 2) and raw.shape == (1500, 2)
    np.testing.assert_allclose(prob.sum(1), 1.0, atol=1e-5)
    np.testing.assert_array_equal(pred, raw.argmax(1))
    assert accuracy_score(y, pred) > 0.85
    # single-row helpers agree with the batch path
    for i in (0, 7, 123):
        assert model.predict(X[i]) == pred[i]
        np.testing.assert_allclose(np.asarray(model.predictProbability(X[i]).toArray()), prob[i], atol=1e-5)


def test_rf_classifier_multiclass_and_persistence(device, tmp_path):
    X, y = _clf_data(n=1200, classes=3, seed=3)
    df = DataFrame.from_numpy(X, y)
    model = RandomForestClassifier(numTrees=6, maxDepth=7, seed=2).fit(df)
    assert model.numClasses == 3
    pred = model.transform(df).to_numpy("prediction")
    assert accuracy_score(y, pred) > 0.8
    path = str(tmp_path / "rfc")
    model.write().overwrite().save(path)
    m2 = RandomForestClassificationModel.load(path)
    np.testing.assert_array_equal(m2.transform(df).to_numpy("prediction"), pred)
    assert m2.totalNumNodes == model.totalNumNodes


def test_rf_regressor_quality_and_persistence(device, tmp_path):
    X, y = make_regression(n_samples=2000, n_features=10, n_informative=5, noise=5.0, random_state=4)
    X = X.astype(np.float32)
    df = DataFrame.from_numpy(X, y)
    model = RandomForestRegressor(numTrees=10, maxDepth=8, seed=5).fit(df)
    assert isinstance(model, RandomForestRegressionModel)
    pred = model.transform(df).to_numpy("prediction")
    assert r2_score(y, pred) > 0.8
    assert abs(model.predict(X[3]) - pred[3]) < 1e-3 * max(1.0, abs(pred[3]))
    path = str(tmp_path / "rfr")
    model.write().overwrite().save(path)
    m2 = RandomForestRegressionModel.load(path)
    np.testing.assert_allclose(m2.transform(df).to_numpy("prediction"), pred, rtol=1e-6, atol=1e-6)


def test_logistic_regression_persistence(device, tmp_path):
    X, y = _clf_data(n=800, seed=6)
    df = DataFrame.from_numpy(X, y)
    est = LogisticRegression(maxIter=50, regParam=0.01)
    model = est.fit(df)
    path = str(tmp_path / "logreg")
    model.write().overwrite().save(path)
    m2 = LogisticRegressionModel.load(path)
    np.testing.assert_allclose(np.asarray(m2.coefficients.toArray()), np.asarray(model.coefficients.toArray()))
    assert m2.intercept == pytest.approx(model.intercept)
    np.testing.assert_array_equal(m2.transform(df).to_numpy("prediction"), model.transform(df).to_numpy("prediction"))
    est.save(str(tmp_path / "logreg_est"))
    assert LogisticRegression.load(str(tmp_path / "logreg_est")).getMaxIter() == 50


def test_regression_evaluator_matches_sklearn():
    rng = np.random.default_rng(7)
    y = rng.standard_normal(500)
    p = y + 0.3 * rng.standard_normal(500)
    df = DataFrame.from_numpy(np.zeros((500, 1), np.float32), y, extra={"prediction": p})
    ev = RegressionEvaluator()
    assert ev.setMetricName("rmse").evaluate(df) == pytest.approx(np.sqrt(mean_squared_error(y, p)), rel=1e-9)
    assert ev.setMetricName("mse").evaluate(df) == pytest.approx(mean_squared_error(y, p), rel=1e-9)
    assert ev.setMetricName("mae").evaluate(df) == pytest.approx(mean_absolute_error(y, p), rel=1e-9)
    assert ev.setMetricName("r2").evaluate(df) == pytest.approx(r2_score(y, p), rel=1e-9)
    assert ev.isLargerBetter()
    assert not ev.setMetricName("rmse").isLargerBetter()


def test_classification_evaluators_match_sklearn():
    rng = np.random.default_rng(8)
    y = rng.integers(0, 3, 600).astype(np.float64)
    p = np.where(rng.random(600) < 0.7, y, rng.integers(0, 3, 600)).astype(np.float64)
    df = DataFrame.from_numpy(np.zeros((600, 1), np.float32), y, extra={"prediction": p})
    ev = MulticlassClassificationEvaluator(metricName="accuracy")
    assert ev.evaluate(df) == pytest.approx(accuracy_score(y, p), rel=1e-9)
    assert ev.setMetricName("f1").evaluate(df) == pytest.approx(f1_score(y, p, average="weighted"), rel=1e-9)

    yb = rng.integers(0, 2, 700).astype(np.float64)
    score = yb + 1.2 * rng.standard_normal(700)
    raw = np.stack([-score, score], 1)
    dfb = DataFrame.from_numpy(np.zeros((700, 1), np.float32), yb, extra={"rawPrediction": raw})
    auc = BinaryClassificationEvaluator(metricName="areaUnderROC").evaluate(dfb)
    assert auc == pytest.approx(roc_auc_score(yb, score), abs=1e-6)


def test_pca_attributes_match_sklearn(device):
    from sklearn.decomposition import PCA as SkPCA

    from spark_rapids_ml_nai_amd.feature import PCA

    rng = np.random.default_rng(9)
    X = (rng.standard_normal((800, 6)) @ rng.standard_normal((6, 6))).astype(np.float32)
    m = PCA(k=3, inputCol="features", outputCol="o").fit(DataFrame.from_numpy(X))
    sk = SkPCA(n_components=3).fit(X.astype(np.float64))
    comp = np.asarray(m.components_)
    signs = np.sign((comp * sk.components_).sum(1))
    np.testing.assert_allclose(comp * signs[:, None], sk.components_, atol=1e-4)
    np.testing.assert_allclose(m.explained_variance_ratio_, sk.explained_variance_ratio_, rtol=1e-4)
    np.testing.assert_allclose(m.singular_values_, sk.singular_values_, rtol=1e-4)
    np.testing.assert_allclose(m.mean_, sk.mean_, atol=1e-5)
    pc = m.pc.toArray()
    assert pc.shape == (6, 3)
    np.testing.assert_allclose(pc.T, comp, atol=1e-6)


def test_kmeans_and_logreg_model_accessors(device):
    from spark_rapids_ml_nai_amd.clustering import KMeans

    rng = np.random.default_rng(10)
    X = np.concatenate([rng.standard_normal((200, 4)) + 8 * i for i in range(3)]).astype(np.float32)
    df = DataFrame.from_numpy(X, (X[:, 0] > 8).astype(np.float64))
    km = KMeans(k=3, seed=1).fit(df)
    assert not km.hasSummary
    assert np.asarray(km.cluster_centers_).shape == (3, 4)
    pred = km.transform(df).to_numpy("prediction")
    assert len(np.unique(pred)) == 3
    assert all(km.predict(X[i]) == pred[i] for i in (0, 250, 599))
    with pytest.raises(ValueError):
        KMeans().setWeightCol("w")

    g = LogisticRegression(maxIter=30).fit(df)
    assert g.numClasses == 2 and list(g.classes_) == [0.0, 1.0]
    assert g.coefficientMatrix.numRows == 1 and g.coefficientMatrix.numCols == 4
    assert len(g.interceptVector) == 1 and g.num_iters > 0 and np.isfinite(g.objective)
    assert not g.hasSummary
    with pytest.raises(RuntimeError):
        _ = g.summary
    raw = g.transform(df).to_numpy("rawPrediction")
    np.testing.assert_allclose(np.asarray(g.predictRaw(X[5]).toArray()), raw[5], rtol=1e-5, atol=1e-6)


def test_rf_hist_features_per_item_rule():
    """Features per histogram work item shrink so the LDS slab fits (20+ classes at
    128 bins used to fail at launch); the library export is cross-checked in test_ops_gpu."""
    from spark_rapids_ml_nai_amd import ops

    assert ops.rf_hist_fb(128, 3, False) == ops.RF_HIST_FB_MAX
    assert ops.rf_hist_fb(128, 2, True) == ops.RF_HIST_FB_MAX
    for B, S in ((128, 20), (256, 12), (256, 32), (128, 32)):
        fb = ops.rf_hist_fb(B, S, False)
        assert 1 <= fb < ops.RF_HIST_FB_MAX and fb * B * S * 4 <= 64 * 1024


def test_rf_fit_multiple_shares_binning_and_matches_single_fits(monkeypatch):
    """RF hyper-parameter batching: param maps with the same maxBins / seed share ONE quantile
    binning pass; every model equals the model of its own single fit."""
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.models import forest
    from spark_rapids_ml_nai_amd.regression import RandomForestRegressor

    rng = np.random.default_rng(4)
    X = rng.standard_normal((3000, 8)).astype(np.float32)
    y = X[:, 0] - 2 * X[:, 3] + 0.1 * rng.standard_normal(3000)
    df = DataFrame.from_numpy(X, y)
    calls = []
    orig = forest.quantize_features
    monkeypatch.setattr(forest, "quantize_features", lambda *a, **k: calls.append(1) or orig(*a, **k))
    est = RandomForestRegressor(numTrees=3, maxDepth=4, seed=7)
    maps = [{est.numTrees: 3}, {est.numTrees: 5, est.maxDepth: 3}, {est.maxBins: 16}]
    models = dict(est.fitMultiple(df, maps))
    assert len(calls) == 2  # maxBins 32 (two maps) + maxBins 16
    for i, mp in enumerate(maps):
        single = est.copy(mp).fit(df)
        a = models[i].transform(df).to_numpy("prediction")
        b = single.transform(df).to_numpy("prediction")
        np.testing.assert_allclose(a, b, rtol=1e-6, atol=1e-6)
