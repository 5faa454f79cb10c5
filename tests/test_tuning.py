"""CrossValidator (reference tests/test_tuning.py:35-101 and the tuning.py docstring example)."""
import warnings

import numpy as np
import pytest

from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.classification import LogisticRegression, RandomForestClassifier
from spark_rapids_ml_nai_amd.evaluation import MulticlassClassificationEvaluator, RegressionEvaluator
from spark_rapids_ml_nai_amd.regression import LinearRegression, RandomForestRegressor
from spark_rapids_ml_nai_amd.tuning import CrossValidator, CrossValidatorModel, ParamGridBuilder

warnings.filterwarnings("ignore")


def test_param_grid_builder():
    lr = LinearRegression()
    grid = ParamGridBuilder().addGrid(lr.regParam, [0.0, 0.1]).addGrid(lr.maxIter, [5, 10, 20]).build()
    assert len(grid) == 6
    assert {tuple(sorted((p.name, v) for p, v in g.items())) for g in grid} == {
        (("maxIter", m), ("regParam", r)) for r in (0.0, 0.1) for m in (5, 10, 20)}


def test_docstring_example_rf(tmp_path):
    from spark_rapids_ml_nai_amd.core.linalg import Vectors

    rows = [(Vectors.dense([0.0]), 0.0), (Vectors.dense([0.4]), 1.0), (Vectors.dense([0.5]), 0.0),
            (Vectors.dense([0.6]), 2.0), (Vectors.dense([1.0]), 1.0)] * 10
    df = DataFrame.createDataFrame(rows, ["features", "label"])
    rfc = RandomForestClassifier()
    grid = ParamGridBuilder().addGrid(rfc.maxBins, [8, 16]).build()
    evaluator = MulticlassClassificationEvaluator()
    cv = CrossValidator(estimator=rfc, estimatorParamMaps=grid, evaluator=evaluator, parallelism=2)
    cvModel = cv.fit(df)
    assert cvModel.getNumFolds() == 3
    assert cvModel.avgMetrics[0] == pytest.approx(1.0)
    assert evaluator.evaluate(cvModel.transform(df)) == pytest.approx(1.0)
    path = str(tmp_path / "model")
    cvModel.write().save(path)
    read = CrossValidatorModel.read().load(path)
    assert read.avgMetrics == pytest.approx(cvModel.avgMetrics)
    assert evaluator.evaluate(read.transform(df)) == pytest.approx(1.0)
    cv_path = str(tmp_path / "cv")
    cv.write().save(cv_path)
    cv2 = CrossValidator.load(cv_path)
    assert cv2.getNumFolds() == 3 and len(cv2.getEstimatorParamMaps()) == 2
    assert isinstance(cv2.getEstimator(), RandomForestClassifier)
    assert isinstance(cv2.getEvaluator(), MulticlassClassificationEvaluator)


@pytest.mark.parametrize("est_name", ["linreg", "rfr"])
def test_cv_regression_single_pass_matches_generic(est_name):
    rng = np.random.default_rng(0)
    X = rng.standard_normal((600, 5)).astype(np.float32)
    y = X @ np.array([1.0, -2.0, 0.5, 0.0, 3.0]) + 0.1 * rng.standard_normal(600)
    df = DataFrame.from_numpy(X, y)
    if est_name == "linreg":
        est = LinearRegression()
        grid = ParamGridBuilder().addGrid(est.regParam, [0.0, 0.5, 5.0]).build()
    else:
        est = RandomForestRegressor(numTrees=5, seed=1)
        grid = ParamGridBuilder().addGrid(est.maxDepth, [2, 6]).build()
    ev = RegressionEvaluator(metricName="rmse")
    cvm = CrossValidator(estimator=est, estimatorParamMaps=grid, evaluator=ev, numFolds=3, seed=7).fit(df)
    assert len(cvm.avgMetrics) == len(grid)
    # oracle: the same folds evaluated model by model
    cv = CrossValidator(estimator=est, estimatorParamMaps=grid, evaluator=ev, numFolds=3, seed=7)
    folds = cv._kFold(df)
    ref = []
    for pm in grid:
        ms = []
        for train, val in folds:
            ms.append(ev.evaluate(est.fit(train, pm).transform(val)))
        ref.append(np.mean(ms))
    # GPU forests accumulate histograms with float atomics: refits may pick other near-tied splits
    rtol = 1e-6 if est_name == "linreg" else 2e-2
    assert np.allclose(cvm.avgMetrics, ref, rtol=rtol, atol=1e-8)
    assert np.argmin(cvm.avgMetrics) == np.argmin(ref)


def test_cv_logreg_and_submodels():
    rng = np.random.default_rng(1)
    X = rng.standard_normal((500, 4)).astype(np.float32)
    y = (X[:, 0] + 0.3 * X[:, 1] > 0).astype(np.float64)
    df = DataFrame.from_numpy(X, y)
    lr = LogisticRegression()
    grid = ParamGridBuilder().addGrid(lr.regParam, [0.0, 0.1]).build()
    ev = MulticlassClassificationEvaluator(metricName="accuracy")
    cvm = CrossValidator(estimator=lr, estimatorParamMaps=grid, evaluator=ev, collectSubModels=True,
                         numFolds=2).fit(df)
    assert len(cvm.subModels) == 2 and len(cvm.subModels[0]) == 2
    assert min(cvm.avgMetrics) > 0.9


def test_fold_col():
    X = np.random.default_rng(2).standard_normal((90, 3)).astype(np.float32)
    y = X.sum(1)
    df = DataFrame.from_numpy(X, y, extra={"fold": np.arange(90) % 3})
    est = LinearRegression()
    grid = ParamGridBuilder().addGrid(est.regParam, [0.0, 1.0]).build()
    cvm = CrossValidator(estimator=est, estimatorParamMaps=grid, evaluator=RegressionEvaluator(),
                         foldCol="fold").fit(df)
    assert cvm.avgMetrics[0] < cvm.avgMetrics[1]


@pytest.mark.dist
@pytest.mark.parametrize("nw", [2, 4])
@pytest.mark.parametrize("task", ["regression", "logloss", "f1"])
def test_distributed_transform_evaluate_matches_generic(monkeypatch, nw, task):
    """Single-pass transform-evaluate on nw gloo ranks (per-partition sufficient statistics merged
    on the driver) equals evaluating each model's transformed frame with the evaluator."""
    monkeypatch.setenv("SRML_FORCE_CPU", "1")
    rng = np.random.default_rng(5)
    X = rng.standard_normal((900, 4)).astype(np.float32)
    if task == "regression":
        y = X @ np.array([1.0, -2.0, 0.5, 3.0]) + 0.1 * rng.standard_normal(900)
        est, ev = LinearRegression(num_workers=nw), RegressionEvaluator(metricName="r2")
        grid = ParamGridBuilder().addGrid(est.regParam, [0.0, 1.0]).build()
    else:
        y = (X[:, 0] - 0.5 * X[:, 1] + 0.3 * rng.standard_normal(900) > 0).astype(np.float64)
        est = LogisticRegression(num_workers=nw)
        ev = MulticlassClassificationEvaluator(metricName="logLoss" if task == "logloss" else "f1")
        grid = ParamGridBuilder().addGrid(est.regParam, [0.01, 0.5]).build()
    df = DataFrame.from_numpy(X, y, num_partitions=nw)
    models = [m for _, m in sorted(est.fitMultiple(df, grid), key=lambda t: t[0])]
    combined = models[0]._combine(models)
    fast = combined._transformEvaluate(df, ev)
    generic = [ev.evaluate(m.transform(df)) for m in models]
    np.testing.assert_allclose(fast, generic, rtol=1e-9, atol=1e-12)
