"""Spark-compatibility oracle tests (reference: tests/test_pca.py:358-443, test_kmeans.py:333-437,
test_linear_model.py:389-490, test_logistic_regression.py:441-600). Expected values are the ones
Apache Spark (and the reference) produce on the same inputs. Each check runs on the CPU path
(CI) and, marked ``gpu``, through the HIP kernels on an MI355X."""
import warnings

import numpy as np
import pytest

from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.core.linalg import Vectors

warnings.filterwarnings("ignore")

DEVICES = ["cpu", pytest.param("gpu", marks=pytest.mark.gpu)]


@pytest.fixture(params=DEVICES)
def device(request, monkeypatch):
    if request.param == "cpu":
        monkeypatch.setenv("SRML_FORCE_CPU", "1")
    else:
        monkeypatch.delenv("SRML_FORCE_CPU", raising=False)
    return request.param


def _close_abs(a, b, tol=1e-3):
    return np.allclose(np.abs(np.asarray(a)), np.abs(np.asarray(b)), atol=tol)


@pytest.mark.compat
def test_pca_spark_compat(device, tmp_path):
    from spark_rapids_ml_nai_amd.feature import PCA, PCAModel

    data = [
        (Vectors.sparse(5, [(1, 1.0), (3, 7.0)]),),
        (Vectors.dense([2.0, 0.0, 3.0, 4.0, 5.0]),),
        (Vectors.dense([4.0, 0.0, 0.0, 6.0, 7.0]),),
    ]
    df = DataFrame.createDataFrame(data, ["features"])
    pca = PCA(k=2, inputCol="features").setOutputCol("pcaFeatures")
    assert pca.getK() == 2
    model = pca.fit(df)
    assert model.getK() == 2
    out = model.transform(df)
    assert df.is_vector("features") and out.is_vector("pcaFeatures")
    first = out.first().pcaFeatures.toArray()
    assert _close_abs(first, [1.6485728230883814, -4.0132827005162985], 1e-6)
    assert np.allclose(model.explainedVariance.toArray(), [0.7943932532230531, 0.20560674677694699], atol=1e-6)
    pc = model.pc.toArray()
    expected = np.array([-0.4486, 0.133, -0.1252, 0.2165, -0.8477, -0.2842, -0.0562, 0.7636, -0.5653,
                         -0.1156]).reshape(5, 2, order="F")
    assert _close_abs(pc, expected, 1e-3)
    path = str(tmp_path / "pca_model")
    model.write().overwrite().save(path)
    m2 = PCAModel.load(path)
    assert np.allclose(m2.pc.toArray(), model.pc.toArray())
    assert np.allclose(m2.transform(df).first().pcaFeatures.toArray(), first)
    est_path = str(tmp_path / "pca")
    pca.save(est_path)
    assert PCA.load(est_path).getK() == 2


@pytest.mark.parametrize("data,mean,comps,ratio", [
    ([[1.0, 1.0], [2.0, 2.0], [3.0, 3.0]], [2.0, 2.0], [[0.707, 0.707]], [1.0]),
    ([[1.0, 1.0], [1.0, 3.0], [5.0, 1.0], [5.0, 3.0]], [3.0, 2.0], [[1.0, 0.0], [0.0, 1.0]], [0.8, 0.2]),
])
def test_pca_toy(device, data, mean, comps, ratio):
    from spark_rapids_ml_nai_amd.feature import PCA

    df = DataFrame.from_numpy(np.asarray(data, dtype=np.float32))
    m = PCA(k=len(comps), inputCol="features").fit(df)
    assert np.allclose(m.mean, mean, atol=1e-5)
    assert _close_abs(m.components_, comps, 1e-3)
    assert np.allclose(m.explained_variance_ratio_, ratio, atol=1e-5)


@pytest.mark.compat
def test_kmeans_spark_compat(device, tmp_path):
    from spark_rapids_ml_nai_amd.clustering import KMeans, KMeansModel

    data = [(Vectors.dense([0.0, 0.0]),), (Vectors.dense([1.0, 1.0]),), (Vectors.dense([9.0, 8.0]),),
            (Vectors.dense([8.0, 9.0]),)]
    df = DataFrame.createDataFrame(data, ["features"])
    km = KMeans(k=2)
    km.setSeed(1)
    km.setMaxIter(10)
    assert km.getMaxIter() == 10
    km.clear(km.maxIter)
    assert km.getMaxIter() == 20
    with pytest.raises(ValueError):
        km.setWeightCol("w")
    model = km.fit(df)
    centers = sorted(model.clusterCenters(), key=lambda c: c[0])
    assert np.allclose(centers, [[0.5, 0.5], [8.5, 8.5]])
    rows = model.transform(df).collect()
    assert rows[0].prediction == rows[1].prediction and rows[2].prediction == rows[3].prediction
    assert rows[0].prediction != rows[2].prediction
    path = str(tmp_path / "km")
    model.write().overwrite().save(path)
    m2 = KMeansModel.load(path)
    assert np.allclose(sorted(m2.clusterCenters(), key=lambda c: c[0]), centers)
    assert model.predict(Vectors.dense([0.1, 0.1])) == rows[0].prediction


def test_kmeans_tol_zero(device):
    from spark_rapids_ml_nai_amd.clustering import KMeans

    df = DataFrame.from_numpy(np.array([[1, 1], [1, 2], [3, 2], [4, 3]], dtype=np.float32))
    m = KMeans(k=2, seed=0, tol=0.0).fit(df)
    assert np.allclose(sorted(m.clusterCenters(), key=lambda c: c[0]), [[1.0, 1.5], [3.5, 2.5]])
    assert m.dtype == "float32" and m.n_cols == 2


@pytest.mark.compat
def test_linear_regression_spark_compat(device, tmp_path):
    from spark_rapids_ml_nai_amd.regression import LinearRegression, LinearRegressionModel

    X = np.array([[-0.20515826, 1.4940791], [0.12167501, 0.7610377], [1.4542735, 0.14404356],
                  [-0.85409576, 0.3130677], [2.2408931, 0.978738], [-0.1513572, 0.95008844],
                  [-0.9772779, 1.867558], [0.41059852, -0.10321885]], dtype=np.float32)
    y = np.array([2.0374513, 22.403986, 139.4456, -76.19584, 225.72075, -0.6784152, -65.54835, 37.30829],
                 dtype=np.float32)
    df = DataFrame.from_numpy(X, y, vector=True)
    lr = LinearRegression(regParam=0.1, solver="normal")
    assert lr.getRegParam() == 0.1
    lr.setFeaturesCol("features").setMaxIter(5).setRegParam(0.0).setLabelCol("label")
    assert lr.getMaxIter() == 5 and lr.getRegParam() == 0.0
    model = lr.fit(df)
    assert np.allclose(model.coefficients.toArray(), [94.46689350900762, 14.33532962562045], atol=1e-3)
    assert np.isclose(model.intercept, -3.3089753423400734e-07, atol=1.0e-4)
    model.setPredictionCol("prediction")
    out = model.transform(df)
    assert out.is_vector("features")
    assert np.isclose(out.first().prediction, 2.037452415464224, rtol=1e-5)
    lr.save(str(tmp_path / "lr"))
    assert LinearRegression.load(str(tmp_path / "lr")).getMaxIter() == 5
    model.save(str(tmp_path / "lr_model"))
    m2 = LinearRegressionModel.load(str(tmp_path / "lr_model"))
    assert model.coefficients.toArray()[0] == m2.coefficients.toArray()[0]
    assert model.intercept == m2.intercept
    assert model.numFeatures == 2


@pytest.mark.compat
@pytest.mark.parametrize("standardization,coef,prob", [
    (True, [-2.48197058, 2.48197058], [0.0771, 0.9229]),
    (False, [-2.42377087, 2.42377087], [0.0814, 0.9186]),
])
def test_logistic_regression_spark_compat(device, standardization, coef, prob, tmp_path):
    from spark_rapids_ml_nai_amd.classification import LogisticRegression, LogisticRegressionModel

    X = np.array([[1.0, 2.0], [1.0, 3.0], [2.0, 1.0], [3.0, 1.0]], dtype=np.float32)
    y = np.array([1.0, 1.0, 0.0, 0.0])
    df = DataFrame.from_numpy(X, y, vector=True)
    lr = LogisticRegression(regParam=0.01, standardization=standardization)
    lr.setMaxIter(20)
    lr.clear(lr.maxIter)
    assert lr.getMaxIter() == 100
    model = lr.fit(df)
    assert np.allclose(model.coefficients.toArray(), coef, atol=1e-3)
    assert abs(model.intercept) < 1e-3
    first = model.transform(df).first()
    assert np.allclose(first.probability.toArray(), prob, atol=1e-3)
    assert np.allclose(first.rawPrediction.toArray(), np.array(coef) @ np.array([1.0, 2.0]) * np.array([-1, 1]), atol=1e-2)
    assert first.prediction == 1.0
    model.save(str(tmp_path / "m"))
    m2 = LogisticRegressionModel.load(str(tmp_path / "m"))
    assert np.allclose(m2.coefficients.toArray(), model.coefficients.toArray())


def test_logistic_regression_toy(device):
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    X = np.array([[1.0, 2.0], [1.0, 3.0], [2.0, 1.0], [3.0, 1.0]], dtype=np.float32)
    y = np.array([1.0, 1.0, 0.0, 0.0])
    lr = LogisticRegression(regParam=1.0, standardization=False)
    assert lr.cuml_params["C"] == 1.0
    assert LogisticRegression(regParam=0.0).cuml_params["C"] == 0.0
    model = lr.fit(DataFrame.from_numpy(X, y))
    assert np.allclose(model.coefficients.toArray(), [-0.287264, 0.287264], atol=1e-5)
    assert [r.prediction for r in model.transform(DataFrame.from_numpy(X, y)).collect()] == [1.0, 1.0, 0.0, 0.0]


def test_logistic_regression_one_label(device):
    from spark_rapids_ml_nai_amd.classification import LogisticRegression

    X = np.array([[1.0, 2.0], [1.0, 3.0]], dtype=np.float32)
    m = LogisticRegression().fit(DataFrame.from_numpy(X, np.array([1.0, 1.0])))
    assert m.intercept == float("inf") and np.allclose(m.coefficients.toArray(), 0)
    with pytest.raises(Exception):
        LogisticRegression().fit(DataFrame.from_numpy(X, np.array([2.5, 1.0])))


def test_kmeans_parallel_init_recovers_blobs(device):
    """Default initMode (k-means||): D^2 over-sampling + device k-means++ reduction finds
    well-separated blobs (reference default init="scalable-k-means++")."""
    from spark_rapids_ml_nai_amd.clustering import KMeans

    rng = np.random.default_rng(7)
    centers = rng.uniform(-50, 50, (12, 5))
    lab = rng.integers(0, 12, 6000)
    X = (centers[lab] + 0.3 * rng.standard_normal((6000, 5))).astype(np.float32)
    ok = 0
    for seed in (1, 2, 4, 5):  # 2 over-sampling rounds (Spark initSteps=2) can miss a blob: ~3 % per seed here
        m = KMeans(k=12, seed=seed, maxIter=20).fit(DataFrame.from_numpy(X))
        got = np.asarray(m.clusterCenters())
        d = np.sqrt(((got[:, None, :] - centers[None]) ** 2).sum(-1))
        ok += int(np.all(d.min(0) < 0.1) and np.all(d.min(1) < 0.1))
    assert ok >= 3
