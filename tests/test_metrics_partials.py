"""Device-side evaluation partials (reference classification.py:113-155, regression.py:144-173):
the CrossValidator transform-evaluate pass reduces confusion counts / log-loss / regression moments
where the predictions are; the metrics must equal the host summaries (from_arrays) to 1e-12."""
import numpy as np
import pytest
import torch

from spark_rapids_ml_nai_amd import DataFrame, ops
from spark_rapids_ml_nai_amd.metrics import (ClassificationSummary, MulticlassMetrics, RegressionMetrics,
                                             RegressionSummary)


class _Ev:
    def __init__(self, name):
        self.name = name

    def getMetricName(self):
        return self.name

    def getThroughOrigin(self):
        return False

    def getMetricLabel(self):
        return 1.0

    def getBeta(self):
        return 1.0

    def getEps(self):
        return 1e-15


CLS_METRICS = ["f1", "accuracy", "weightedPrecision", "weightedRecall", "weightedTruePositiveRate",
               "weightedFalsePositiveRate", "weightedFMeasure", "truePositiveRateByLabel", "falsePositiveRateByLabel",
               "precisionByLabel", "recallByLabel", "fMeasureByLabel", "hammingLoss", "logLoss"]


def _cls_data(dev, m=5000, C=4, seed=0):
    g = np.random.default_rng(seed)
    y = g.integers(0, C, m).astype(np.float64)
    prob = g.random((m, C))
    prob /= prob.sum(1, keepdims=True)
    p = prob.argmax(1).astype(np.float64)
    return y, p, prob


def _check_cls(dev):
    y, p, prob = _cls_data(dev)
    host = ClassificationSummary.from_arrays(y, p, prob, 1e-15)
    yd, pd, probd = (torch.from_numpy(a).to(dev) for a in (y, p, prob))
    cm = ops.confusion_counts(yd, pd, 4)
    devs = ClassificationSummary.from_confusion(cm, len(y), ops.logloss_sum(probd, yd, 1e-15))
    for name in CLS_METRICS:
        a = MulticlassMetrics(host).evaluate(_Ev(name))
        b = MulticlassMetrics(devs).evaluate(_Ev(name))
        assert abs(a - b) <= 1e-12 * max(1.0, abs(a)), (name, a, b)
    # an out-of-range prediction flags the fallback
    bad = pd.clone()
    bad[3] = 7.0
    assert ops.confusion_counts(yd, bad, 4) is None


def _check_reg(dev):
    g = np.random.default_rng(1)
    y = g.standard_normal(7000) * 3 + 10
    p = (y + g.standard_normal(7000) * 0.5).astype(np.float32)  # fp32 predictions, widened on the fly
    host = RegressionSummary.from_arrays(y, p.astype(np.float64))
    devs = RegressionSummary.from_moments(len(y), ops.reg_moments(torch.from_numpy(y).to(dev),
                                                                   torch.from_numpy(p).to(dev)))
    for name in ("rmse", "mse", "r2", "mae", "var"):
        a = RegressionMetrics(host).evaluate(_Ev(name))
        b = RegressionMetrics(devs).evaluate(_Ev(name))
        assert abs(a - b) <= 1e-12 * max(1.0, abs(a)), (name, a, b)


def test_partials_cpu():
    _check_cls(torch.device("cpu"))
    _check_reg(torch.device("cpu"))


@pytest.mark.gpu
def test_partials_gpu(gpu_device):
    _check_cls(gpu_device)
    _check_reg(gpu_device)
    # fp32 / int predictions and a 100-class (global-atomic) confusion matrix
    g = np.random.default_rng(3)
    y = g.integers(0, 100, 20000)
    p = g.integers(0, 100, 20000)
    cm = ops.confusion_counts(torch.from_numpy(y.astype(np.float32)).to(gpu_device),
                              torch.from_numpy(p).to(gpu_device), 100)
    ref = np.zeros((100, 100), np.int64)
    np.add.at(ref, (y, p), 1)
    assert np.array_equal(cm, ref)


def _eval_host(models, X, y, kind, need_prob, eps):
    out = []
    for m in models:
        res = m._transform_df(DataFrame.from_numpy(X, y))
        p = res.to_numpy(m.getOrDefault("predictionCol"))
        if kind == "regression":
            out.append(RegressionSummary.from_arrays(y, p))
        else:
            prob = res.to_numpy(m.getOrDefault("probabilityCol")) if need_prob else None
            out.append(ClassificationSummary.from_arrays(y, p, prob, eps))
    return out


@pytest.mark.parametrize("kind", ["classification", "regression"])
def test_eval_worker_device_partials_match_host(kind):
    """``_eval_worker`` (predictions kept on the device, partials reduced there) gives the same
    metrics as summaries of the host predictions."""
    from spark_rapids_ml_nai_amd.core.base import _eval_worker
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    g = np.random.default_rng(5)
    X = g.standard_normal((3000, 8)).astype(np.float32)
    if kind == "regression":
        from spark_rapids_ml_nai_amd.regression import LinearRegression

        y = X @ g.standard_normal(8) + 0.1 * g.standard_normal(3000)
        models = [LinearRegression(regParam=r).fit(DataFrame.from_numpy(X, y)) for r in (0.0, 0.1)]
        names = ("rmse", "r2", "mae", "var")
    else:
        from spark_rapids_ml_nai_amd.classification import LogisticRegression

        y = (X[:, 0] + 0.3 * g.standard_normal(3000) > 0).astype(np.float64)
        models = [LogisticRegression(regParam=r, maxIter=30).fit(DataFrame.from_numpy(X, y)) for r in (0.0, 0.1)]
        names = CLS_METRICS
    table = DataFrame.from_numpy(X, y).partitions[0]
    rows = _eval_worker(WorkerContext.single(torch.device("cpu")),
                        (models, [table], "label", (kind, True, 1e-15)))
    host = _eval_host(models, X, y, kind, True, 1e-15)
    Met = RegressionMetrics if kind == "regression" else MulticlassMetrics
    for dev_s, host_s in zip(rows[0], host):
        for name in names:
            a, b = Met(host_s).evaluate(_Ev(name)), Met(dev_s).evaluate(_Ev(name))
            assert abs(a - b) <= 1e-12 * max(1.0, abs(a)), (name, a, b)
