"""Spark integration without a JVM: the barrier fit task body (parallel/spark.py) driven by a
multi-process BarrierTaskContext stand-in (gloo, 2 ranks), and the stage-level scheduling
decision table (reference core.py:901-1004)."""
import warnings

import numpy as np
import pandas as pd
import pytest

from spark_rapids_ml_nai_amd.parallel.spark import is_spark_dataframe, stage_level_scheduling_plan

warnings.filterwarnings("ignore")


def test_stage_level_scheduling_plan():
    conf = {"spark.executor.cores": "12", "spark.executor.resource.gpu.amount": "1",
            "spark.task.resource.gpu.amount": "0.08"}
    assert stage_level_scheduling_plan("3.5.1", conf, "yarn") == (7, 1.0)
    assert stage_level_scheduling_plan("3.5.1", conf, "yarn", "com.nvidia.spark.SQLPlugin", "true") == (12, 1.0)
    assert stage_level_scheduling_plan("3.3.2", conf, "yarn") is None
    assert stage_level_scheduling_plan("3.4.1", conf, "yarn") is None          # needs standalone before 3.5.1
    assert stage_level_scheduling_plan("3.4.1", conf, "spark://h:7077") == (7, 1.0)
    assert stage_level_scheduling_plan("3.10.0", conf, "yarn") == (7, 1.0)     # numeric version compare
    assert stage_level_scheduling_plan("3.5.1", conf, "local[4]") is None
    assert stage_level_scheduling_plan("3.5.1", dict(conf, **{"spark.executor.cores": "1"}), "yarn") is None
    assert stage_level_scheduling_plan("3.5.1", dict(conf, **{"spark.executor.resource.gpu.amount": "2"}),
                                       "yarn") is None
    assert stage_level_scheduling_plan("3.5.1", dict(conf, **{"spark.task.resource.gpu.amount": "1"}),
                                       "yarn") is None
    no_task = {k: v for k, v in conf.items() if k != "spark.task.resource.gpu.amount"}
    assert stage_level_scheduling_plan("3.5.1", no_task, "yarn") == (7, 1.0)


def test_is_spark_dataframe():
    from spark_rapids_ml_nai_amd import DataFrame

    assert not is_spark_dataframe(DataFrame.from_numpy(np.zeros((2, 2), np.float32)))
    assert not is_spark_dataframe(pd.DataFrame({"a": [1]}))


def _fit_payload(est, float32=True):
    import cloudpickle

    fit_fn = est._get_fit_func(None, None)
    params = {"cuml_init": dict(est._backend_params), "fit_multiple_params": []}
    return cloudpickle.dumps((est, fit_fn, params, float32, [], False))


def _task(payload):
    from spark_rapids_ml_nai_amd.parallel.spark import spark_worker_entry

    def fn(ctx, it):
        return spark_worker_entry(ctx, it, payload)

    return fn


@pytest.mark.dist
def test_barrier_worker_linear_regression(monkeypatch):
    import cloudpickle

    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.parallel.testing import run_fake_barrier_stage
    from spark_rapids_ml_nai_amd.regression import LinearRegression

    monkeypatch.setenv("SRML_FORCE_CPU", "1")
    rng = np.random.default_rng(0)
    X = rng.standard_normal((400, 5)).astype(np.float32)
    y = X @ np.array([1.0, 2.0, 3.0, -1.0, 0.5]) + 0.25
    pdf = pd.DataFrame({"features": list(X), "label": y})
    # two partitions, the second delivered as two Arrow batches (as mapInPandas would)
    parts = [[pdf.iloc[:200]], [pdf.iloc[200:300], pdf.iloc[300:]]]
    est = LinearRegression(featuresCol="features", labelCol="label", num_workers=2)
    rows = run_fake_barrier_stage(_task(_fit_payload(est)), parts)
    assert len(rows) == 1  # rank 0 yields the model
    out = cloudpickle.loads(rows[0]["result"][0])
    res = out.result  # core.base._FitOut: the model attributes + every rank's time split
    assert len(out.ranks) == 2 and all("h2d_exposed_s" in r for r in out.ranks)
    ref = LinearRegression(num_workers=1).fit(DataFrame.from_numpy(X, y))
    assert np.allclose(res["coef_"], ref.coefficients.toArray(), atol=1e-5)
    assert np.isclose(res["intercept_"], ref.intercept, atol=1e-5)
