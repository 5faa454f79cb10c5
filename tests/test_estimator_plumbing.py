"""Framework plumbing with a dummy device solver (the role of the reference's
``python/tests/test_common_estimator.py``: a fake backend exercising param mapping, copy/extra,
fit-with-param-map, fitMultiple, persistence, num_workers validation and the barrier fit job,
without any numerics). Our own dummy; assertions follow the reference's documented semantics:
Param mapped to ``None`` -> error when set, ``""`` -> warning and ignored, value translators,
backend kwargs accepted under their own names, Spark/backend alias conflicts rejected."""
import warnings
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import pytest

from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.core.base import FitInput, _Estimator, _Model
from spark_rapids_ml_nai_amd.core.params import (
    HasInputCol,
    HasInputCols,
    HasOutputCol,
    Param,
    Params,
    TypeConverters,
    _BackendClass,
    _BackendParams,
    keyword_only,
)
from spark_rapids_ml_nai_amd.parallel.context import WorkerContext


@pytest.fixture(autouse=True)
def _cpu(monkeypatch):
    monkeypatch.setenv("SRML_FORCE_CPU", "1")


class DummyClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        # alpha -> a, k -> k, beta unsupported, gamma accepted but unused
        return {"alpha": "a", "beta": None, "gamma": "", "k": "k"}

    @classmethod
    def _param_value_mapping(cls) -> Dict[str, Callable[[Any], Any]]:
        # the backend wants a strictly positive float; 0 is "unsupported"
        return {"a": lambda v: float(v) if v > 0 else None}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {"a": 10.0, "k": 3, "x": 40.0}


class _DummyParams(_BackendParams, HasInputCol, HasInputCols, HasOutputCol):
    alpha = Param(Params._dummy(), "alpha", "mapped to backend a", typeConverter=TypeConverters.toFloat)
    beta = Param(Params._dummy(), "beta", "unsupported on the backend", typeConverter=TypeConverters.toInt)
    gamma = Param(Params._dummy(), "gamma", "ignored by the backend", typeConverter=TypeConverters.toFloat)
    k = Param(Params._dummy(), "k", "mapped to backend k", typeConverter=TypeConverters.toInt)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(alpha=10.0, k=3, outputCol="dummy_out")

    def setAlpha(self, v: float) -> Any:
        return self._set_params(alpha=v)

    def setBeta(self, v: int) -> Any:
        return self._set_params(beta=v)

    def setGamma(self, v: float) -> Any:
        return self._set_params(gamma=v)




class DummyEstimator(DummyClass, _Estimator, _DummyParams):
    @keyword_only
    def __init__(self, **kwargs: Any) -> None:
        super().__init__()
        self._set_params(**self._input_kwargs)

    def _enable_fit_multiple_in_single_pass(self) -> bool:
        return True

    def _get_fit_func(self, dataset: Any, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        def _fit(inp: FitInput, ctx: WorkerContext, params: Dict[str, Any]) -> Any:
            d = inp.desc
            # partition descriptor invariants (reference PartitionDescriptor.build)
            assert d.rank == ctx.rank and len(d.parts_rank_size) == ctx.world_size
            assert d.m == sum(s for _, s in d.parts_rank_size) and d.n == inp.X.shape[1]
            assert inp.X.shape[0] == d.parts_rank_size[ctx.rank][1]
            col_sum = inp.X.double().sum(0)
            ctx.comm.allreduce(col_sum)
            maps = params["fit_multiple_params"] or [{}]
            out = []
            for mp in maps:
                p = dict(params["cuml_init"], **mp)
                out.append({"a_used": p["a"], "k_used": p["k"], "m": d.m, "n": d.n, "world": ctx.world_size,
                            "col_sum": col_sum.cpu().numpy().tolist()})
            return out if params["fit_multiple_params"] else out[0]

        return _fit

    def _create_model(self, result: Dict[str, Any]) -> "DummyModel":
        return DummyModel._from_row(result)


class DummyModel(DummyClass, _Model, _DummyParams):
    def __init__(self, a_used: float, k_used: int, m: int, n: int, world: int, col_sum: List[float]) -> None:
        super().__init__(a_used=a_used, k_used=k_used, m=m, n=n, world=world, col_sum=col_sum)
        self.a_used, self.k_used, self.m, self.world = a_used, k_used, m, world
        self.col_sum = col_sum

    def _get_transform_func(self, dataset: Any) -> Any:
        def construct(ctx: WorkerContext) -> Any:
            return float(self.a_used)

        def predict(state: Any, X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            return {self.getOrDefault("outputCol"): np.asarray(X).sum(1) * state}

        return construct, predict


def _df(parts=2):
    X = np.arange(60, dtype=np.float32).reshape(20, 3)
    return DataFrame.from_numpy(X, num_partitions=parts), X


def test_defaults_and_spark_or_backend_names():
    est = DummyEstimator()
    assert est.cuml_params == {"a": 10.0, "k": 3, "x": 40.0} and est.backend_params is est.cuml_params
    est = DummyEstimator(alpha=2.0, k=5)
    assert est.getOrDefault("alpha") == 2.0 and est.cuml_params["a"] == 2.0 and est.cuml_params["k"] == 5
    est = DummyEstimator(a=7.0, x=1.5)  # backend names reflect into the aliased Spark Param
    assert est.cuml_params["a"] == 7.0 and est.getOrDefault("alpha") == 7.0 and est.cuml_params["x"] == 1.5


def test_unsupported_ignored_invalid_and_alias_conflict():
    with pytest.raises(ValueError, match="Spark Param 'beta' is not supported"):
        DummyEstimator(beta=1)
    with pytest.raises(ValueError, match="not supported"):
        DummyEstimator().setBeta(2)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        est = DummyEstimator(gamma=0.5)
    assert any("gamma" in str(x.message) for x in w)
    assert est.getOrDefault("gamma") == 0.5 and "gamma" not in est.cuml_params
    with pytest.raises(ValueError, match="given invalid value"):
        DummyEstimator(alpha=0.0)
    with pytest.raises(ValueError, match="alias of 'alpha'"):
        DummyEstimator(alpha=1.0, a=2.0)
    with pytest.raises(ValueError, match="Unsupported param 'zzz'"):
        DummyEstimator(zzz=1)


def test_copy_extra_and_clear():
    est = DummyEstimator(alpha=3.0)
    c = est.copy({est.alpha: 1111.0})
    assert c.getOrDefault("alpha") == 1111.0 and c.cuml_params["a"] == 1111.0
    assert est.getOrDefault("alpha") == 3.0 and est.cuml_params["a"] == 3.0  # original untouched
    with pytest.raises(ValueError, match="not supported"):
        est.copy({est.beta: 1})
    est.clear(est.alpha)
    assert est.getOrDefault("alpha") == 10.0 and est.cuml_params["a"] == 10.0


def test_input_col_routing():
    assert DummyEstimator(inputCol="f").getInputCol() == "f"
    assert DummyEstimator(inputCol=["f1", "f2"]).getInputCols() == ["f1", "f2"]
    assert DummyEstimator(inputCols=["f1", "f2"]).getInputCols() == ["f1", "f2"]


@pytest.mark.parametrize("workers", [1, 2])
def test_fit_paths(workers, tmp_path):
    df, X = _df(parts=workers)
    est = DummyEstimator(inputCol="features", alpha=100.0, k=4, num_workers=workers)
    m = est.fit(df)
    assert (m.a_used, m.k_used, m.m, m.world) == (100.0, 4, 20, workers)
    np.testing.assert_allclose(m.col_sum, X.astype(np.float64).sum(0))
    assert m.cuml_params["a"] == 100.0 and m.num_workers == workers
    # fit with a param map: the model sees the override, the estimator does not change
    m2 = est.fit(df, {est.alpha: 9876.0})
    assert m2.a_used == 9876.0 and m2.getOrDefault("alpha") == 9876.0 and m2.cuml_params["a"] == 9876.0
    assert est.cuml_params["a"] == 100.0 and est.getOrDefault("alpha") == 100.0
    # fitMultiple in ONE job (single pass), models in param-map order
    maps = [{est.alpha: 1.0}, {est.alpha: 2.0, est.k: 9}]
    got = dict(est.fitMultiple(df, maps))
    assert [got[i].a_used for i in range(2)] == [1.0, 2.0] and got[1].k_used == 9
    # transform with the model's device closure
    out = m.transform(df)
    col = m.getOrDefault("outputCol")
    np.testing.assert_allclose(out.to_numpy(col), X.sum(1) * 100.0)


def test_persistence_roundtrip(tmp_path):
    df, _ = _df(parts=1)
    est = DummyEstimator(inputCol="features", alpha=42.0, x=2.5, num_workers=1, float32_inputs=False)
    est.save(str(tmp_path / "est"))
    e2 = DummyEstimator.load(str(tmp_path / "est"))
    assert e2.cuml_params == est.cuml_params and e2.getOrDefault("alpha") == 42.0
    assert e2.num_workers == 1 and e2._float32_inputs is False
    m = est.fit(df)
    m.save(str(tmp_path / "model"))
    m2 = DummyModel.load(str(tmp_path / "model"))
    assert m2.a_used == 42.0 and m2.col_sum == m.col_sum and m2.cuml_params == m.cuml_params


def test_num_workers_validation():
    est = DummyEstimator(num_workers=0)
    with pytest.raises(ValueError, match="num_workers must be >= 1"):
        _ = est.num_workers
    assert DummyEstimator(num_workers=3).num_workers == 3


def test_empty_partition_fails_the_job():
    X = np.arange(6, dtype=np.float32).reshape(2, 3)
    df = DataFrame.from_numpy(X, num_partitions=1)
    with pytest.raises(RuntimeError, match="no data"):
        DummyEstimator(inputCol="features", num_workers=3).fit(df)
