"""``regression.LinearRegression`` / ``LinearRegressionModel`` (reference ``regression.py:176-796``)
and ``RandomForestRegressor`` / ``RandomForestRegressionModel`` (``regression.py:799-1080``).

Param mapping and defaults follow the reference (``regParam -> alpha``, ``elasticNetParam ->
l1_ratio``, ``standardization -> normalize``, ``loss``/``solver`` value maps, unsupported
``weightCol``/``huber``/``l-bfgs``). Numerics follow Spark's objective exactly (see
``models/linear.py``), fitMultiple runs every param map off ONE set of device statistics.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .core.base import FitInput, _EstimatorSupervised, _ModelWithPredictionCol
from .core.dataframe import DataFrame
from .core.linalg import DenseVector, as_dense_array
from .core.params import (
    HasAggregationDepth,
    HasElasticNetParam,
    HasFeaturesCol,
    HasFeaturesCols,
    HasFitIntercept,
    HasLabelCol,
    HasLoss,
    HasMaxBlockSizeInMB,
    HasMaxIter,
    HasPredictionCol,
    HasRegParam,
    HasSolver,
    HasStandardization,
    HasTol,
    HasWeightCol,
    Param,
    Params,
    TypeConverters,
    _BackendClass,
    _BackendParams,
    keyword_only,
)
from .parallel.context import WorkerContext


from .core.params import _FeaturesColMixin  # noqa: E402  (re-exported for tree.py / clustering.py)


# ======================================================================================
# LinearRegression
# ======================================================================================
class LinearRegressionClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {
            "aggregationDepth": "",
            "elasticNetParam": "l1_ratio",
            "epsilon": "",
            "fitIntercept": "fit_intercept",
            "loss": "loss",
            "maxBlockSizeInMB": "",
            "maxIter": "max_iter",
            "regParam": "alpha",
            "solver": "solver",
            "standardization": "normalize",
            "tol": "tol",
            "weightCol": None,
        }

    @classmethod
    def _param_value_mapping(cls) -> Dict[str, Callable[[Any], Any]]:
        return {
            "loss": lambda x: {"squaredError": "squared_loss", "huber": None, "squared_loss": "squared_loss"}.get(x),
            "solver": lambda x: {"auto": "eig", "normal": "eig", "l-bfgs": None, "eig": "eig"}.get(x),
        }

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {
            "algorithm": "eig", "fit_intercept": True, "copy_X": None, "normalize": False, "verbose": False,
            "alpha": 0.0001, "solver": "eig", "loss": "squared_loss", "l1_ratio": 0.15, "max_iter": 1000,
            "tol": 0.001, "shuffle": True,
        }


class _LinearRegressionParams(_BackendParams, HasFeaturesCol, HasFeaturesCols, HasLabelCol, HasPredictionCol,
                              HasMaxIter, HasRegParam, HasElasticNetParam, HasTol, HasFitIntercept,
                              HasStandardization, HasWeightCol, HasSolver, HasAggregationDepth, HasLoss,
                              HasMaxBlockSizeInMB, _FeaturesColMixin):
    epsilon = Param(Params._dummy(), "epsilon", "The shape parameter to control the amount of robustness (huber).",
                    typeConverter=TypeConverters.toFloat)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(maxIter=100, regParam=0.0, tol=1e-6, fitIntercept=True, standardization=True,
                         solver="auto", loss="squaredError", epsilon=1.35, elasticNetParam=0.0,
                         aggregationDepth=2, maxBlockSizeInMB=0.0, featuresCol="features", labelCol="label",
                         predictionCol="prediction")

    def getEpsilon(self) -> float:
        return self.getOrDefault("epsilon")


class LinearRegression(LinearRegressionClass, _EstimatorSupervised, _LinearRegressionParams):
    """Distributed OLS / Ridge / ElasticNet on MI355X (Gram + X'y all-reduce, Spark objective).

    >>> lr = LinearRegression(regParam=0.0, solver="normal")
    >>> model = lr.fit(df)   # doctest: +SKIP
    """

    @keyword_only
    def __init__(self, *, featuresCol: Union[str, List[str]] = "features", labelCol: str = "label",
                 predictionCol: str = "prediction", maxIter: int = 100, regParam: float = 0.0,
                 elasticNetParam: float = 0.0, tol: float = 1e-6, fitIntercept: bool = True,
                 standardization: bool = True, solver: str = "auto", loss: str = "squaredError",
                 num_workers: Optional[int] = None, verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._set_params(**self._input_kwargs)

    def setMaxIter(self, value: int) -> "LinearRegression":
        return self._set_params(maxIter=value)

    def setRegParam(self, value: float) -> "LinearRegression":
        return self._set_params(regParam=value)

    def setElasticNetParam(self, value: float) -> "LinearRegression":
        return self._set_params(elasticNetParam=value)

    def setLoss(self, value: str) -> "LinearRegression":
        return self._set_params(loss=value)

    def setStandardization(self, value: bool) -> "LinearRegression":
        return self._set_params(standardization=value)

    def setTol(self, value: float) -> "LinearRegression":
        return self._set_params(tol=value)

    def setFitIntercept(self, value: bool) -> "LinearRegression":
        return self._set_params(fitIntercept=value)

    def setSolver(self, value: str) -> "LinearRegression":
        return self._set_params(solver=value)

    def _enable_fit_multiple_in_single_pass(self) -> bool:
        return True

    def _supportsTransformEvaluate(self, evaluator: Any) -> bool:
        return type(evaluator).__name__ == "RegressionEvaluator"

    def _validate_parameters(self) -> None:
        if self.isSet("weightCol") and self.getOrDefault("weightCol"):
            raise ValueError("weightCol is not supported")

    def _get_fit_func(self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        def _fit(inp: FitInput, ctx: WorkerContext, params: Dict[str, Any]) -> Any:
            from .models.linear import lsq_solve, lsq_stats

            n = inp.desc.n
            init = params["cuml_init"]
            maps = params["fit_multiple_params"] or [{}]
            for mp in maps:
                p = dict(init, **mp)
                if n == 1 and (p["alpha"] == 0 or p["l1_ratio"] == 0):
                    raise RuntimeError("LinearRegression doesn't support training data with 1 column")
            st = lsq_stats(inp.X, inp.y, inp.desc.m, ctx, stream=inp.stream)
            out = []
            for mp in maps:
                p = dict(init, **mp)
                res = lsq_solve(st, float(p["alpha"]), float(p["l1_ratio"]), bool(p["fit_intercept"]),
                                bool(p["normalize"]), int(p["max_iter"]), float(p["tol"]))
                res.update(n_cols=n, dtype="float32" if inp.X.dtype == torch.float32 else "float64")
                out.append(res)
            return out if params["fit_multiple_params"] else out[0]

        _fit.streaming_ingest = True  # type: ignore[attr-defined]
        return _fit

    def _create_model(self, result: Dict[str, Any]) -> "LinearRegressionModel":
        return LinearRegressionModel._from_row(result)


class LinearRegressionSummary:
    def __init__(self, metrics: Any, predictions: Any) -> None:
        self._m = metrics
        self.predictions = predictions

    @property
    def rootMeanSquaredError(self) -> float:
        return self._m.root_mean_squared_error

    @property
    def meanSquaredError(self) -> float:
        return self._m.mean_squared_error

    @property
    def meanAbsoluteError(self) -> float:
        return self._m.mean_absolute_error

    @property
    def r2(self) -> float:
        return self._m.r2(False)

    @property
    def explainedVariance(self) -> float:
        return self._m.explained_variance


class LinearRegressionModel(LinearRegressionClass, _ModelWithPredictionCol, _LinearRegressionParams):
    def __init__(self, coef_: Union[List[float], List[List[float]]], intercept_: Union[float, List[float]],
                 n_cols: int, dtype: str) -> None:
        super().__init__(coef_=coef_, intercept_=intercept_, n_cols=n_cols, dtype=dtype)
        self.coef_ = coef_
        self.intercept_ = intercept_
        self.n_cols = n_cols
        self.dtype = dtype
        self._lr_ml_model = None

    @property
    def coefficients(self) -> DenseVector:
        return DenseVector(self.coef_)

    @property
    def intercept(self) -> float:
        return float(self.intercept_)

    @property
    def scale(self) -> float:
        return 1.0

    @property
    def hasSummary(self) -> bool:
        return False

    def predict(self, value: Any) -> float:
        return float(np.dot(as_dense_array(value), np.asarray(self.coef_, dtype=np.float64)) + self.intercept)

    def evaluate(self, dataset: Any) -> LinearRegressionSummary:
        from .metrics import RegressionMetrics, RegressionSummary

        out = self.transform(dataset)
        from .core.dataframe import as_dataframe

        df, _ = as_dataframe(out)
        y = df.to_numpy(self.getLabelCol(), np.float64)
        p = df.to_numpy(self.getPredictionCol(), np.float64)
        return LinearRegressionSummary(RegressionMetrics(RegressionSummary.from_arrays(y, p)), out)

    def cpu(self) -> Any:
        from .utils.spark_compat import to_spark_linear_regression_model

        return to_spark_linear_regression_model(self)

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        coef = np.asarray(self.coef_, dtype=np.float64)
        intercept = float(self.intercept_)
        pred_col = self.getPredictionCol()
        np_dt = np.float32 if self.dtype == "float32" else np.float64

        def construct(ctx: WorkerContext) -> torch.Tensor:
            return torch.from_numpy(coef.astype(np_dt)).to(ctx.device)

        def predict(w: torch.Tensor, X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            from .core.base import to_device
            from .models.linear import linear_predict

            Xd = to_device(X, ctx.device, w.dtype)
            return {pred_col: ctx.output(linear_predict(Xd, w, intercept).double())}

        return construct, predict

    @classmethod
    def _combine(cls, models: List["LinearRegressionModel"]) -> "LinearRegressionModel":
        first = models[0]
        out = cls(coef_=first.coef_, intercept_=first.intercept_, n_cols=first.n_cols, dtype=first.dtype)
        first._copyValues(out)
        first._copy_backend_params(out)
        out._combined_models = list(models)
        return out


# ======================================================================================
# RandomForestRegressor
# ======================================================================================
from .tree import _RandomForestEstimator, _RandomForestModel  # noqa: E402


class RandomForestRegressor(_RandomForestEstimator):
    """Random forest regressor (variance impurity) grown level-wise on MI355X."""

    _is_classification = False

    @classmethod
    def _param_value_mapping(cls) -> Dict[str, Callable[[Any], Any]]:
        m = dict(super()._param_value_mapping())
        m["split_criterion"] = lambda x: {"variance": "mse", "mse": "mse"}.get(x)
        return m

    @keyword_only
    def __init__(self, *, featuresCol: Union[str, List[str]] = "features", labelCol: str = "label",
                 predictionCol: str = "prediction", maxDepth: int = 5, maxBins: int = 32,
                 minInstancesPerNode: int = 1, minInfoGain: float = 0.0, maxMemoryInMB: int = 256,
                 cacheNodeIds: bool = False, checkpointInterval: int = 10, impurity: str = "variance",
                 subsamplingRate: float = 1.0, seed: Optional[int] = None, numTrees: int = 20,
                 featureSubsetStrategy: str = "auto", leafCol: str = "", minWeightFractionPerNode: float = 0.0,
                 weightCol: Optional[str] = None, bootstrap: Optional[bool] = True,
                 num_workers: Optional[int] = None, verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._setDefault(impurity="variance")
        self._initialize_backend_params()
        self._set_params(**self._input_kwargs)

    def _supportsTransformEvaluate(self, evaluator: Any) -> bool:
        return type(evaluator).__name__ == "RegressionEvaluator"

    def _create_model(self, result: Dict[str, Any]) -> "RandomForestRegressionModel":
        return RandomForestRegressionModel._from_row(result)


class RandomForestRegressionModel(_RandomForestModel):
    _is_classification = False

    def predict(self, value: Any) -> float:
        x = np.asarray(as_dense_array(value), dtype=np.float32).reshape(1, -1)
        return float(self._raw_sum(x, torch.device("cpu")).numpy()[0, 0] / max(len(self._trees), 1))

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        pc = self.getPredictionCol()
        T = max(len(self._trees), 1)

        def construct(ctx: WorkerContext) -> Any:
            self._pack(ctx.device)
            return ctx.device

        def predict(device: Any, X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            raw = self._raw_sum(X, ctx.device)
            return {pc: ctx.output(raw[:, 0] / T)}

        return construct, predict

    def evaluate(self, dataset: Any) -> Any:
        from .core.dataframe import as_dataframe
        from .metrics import RegressionMetrics, RegressionSummary

        out = self.transform(dataset)
        df, _ = as_dataframe(out)
        y = df.to_numpy(self.getLabelCol(), np.float64)
        p = df.to_numpy(self.getPredictionCol(), np.float64)
        return LinearRegressionSummary(RegressionMetrics(RegressionSummary.from_arrays(y, p)), out)
