"""``classification.LogisticRegression`` / ``LogisticRegressionModel`` (reference
``classification.py:665-1569``) and ``RandomForestClassifier`` /
``RandomForestClassificationModel`` (``classification.py:279-662``).

LogisticRegression param mapping: ``regParam -> C = 1/regParam`` (0 -> 0), ``elasticNetParam ->
l1_ratio``, ``maxIter``, ``tol``, ``fitIntercept``, ``standardization``; ``threshold(s)``,
``weightCol``, bounds, ``aggregationDepth``, ``maxBlockSizeInMB`` unsupported; ``family`` ignored
(binomial/multinomial chosen from the labels). Sparse VectorUDT input is consumed as CSR when
``enable_sparse_data_optim`` allows.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .core.base import FitInput, _EstimatorSupervised, _ModelWithPredictionCol
from .core.dataframe import DataFrame
from .core.linalg import DenseMatrix, Vectors, as_dense_array, compressed_vector
from .core.params import (
    HasAggregationDepth,
    HasElasticNetParam,
    HasEnableSparseDataOptim,
    HasFeaturesCol,
    HasFeaturesCols,
    HasFitIntercept,
    HasLabelCol,
    HasMaxBlockSizeInMB,
    HasMaxIter,
    HasPredictionCol,
    HasProbabilityCol,
    HasRawPredictionCol,
    HasRegParam,
    HasStandardization,
    HasThreshold,
    HasThresholds,
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
from .core.params import _FeaturesColMixin


class _ClassifierColsMixin(_FeaturesColMixin):
    def setProbabilityCol(self, value: str) -> Any:
        return self._set_params(probabilityCol=value)

    def setRawPredictionCol(self, value: str) -> Any:
        return self._set(rawPredictionCol=value)


# ======================================================================================
# LogisticRegression
# ======================================================================================
class LogisticRegressionClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {
            "maxIter": "max_iter",
            "regParam": "C",
            "elasticNetParam": "l1_ratio",
            "tol": "tol",
            "fitIntercept": "fit_intercept",
            "threshold": None,
            "thresholds": None,
            "standardization": "standardization",
            "weightCol": None,
            "aggregationDepth": None,
            "family": "",
            "lowerBoundsOnCoefficients": None,
            "upperBoundsOnCoefficients": None,
            "lowerBoundsOnIntercepts": None,
            "upperBoundsOnIntercepts": None,
            "maxBlockSizeInMB": None,
        }

    @classmethod
    def _param_value_mapping(cls) -> Dict[str, Callable[[Any], Any]]:
        return {"C": lambda x: 1 / x if x > 0.0 else (0.0 if x == 0.0 else None)}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {"fit_intercept": True, "standardization": False, "verbose": False, "C": 1.0, "penalty": "l2",
                "l1_ratio": None, "max_iter": 1000, "tol": 0.0001}

    @classmethod
    def _reg_params_value_mapping(cls, reg_param: float, elasticNet_param: float) -> Tuple[Optional[str], float, float]:
        if reg_param == 0.0:
            return None, 0.0, elasticNet_param
        if elasticNet_param == 0.0:
            return "l2", 1.0 / reg_param, elasticNet_param
        if elasticNet_param == 1.0:
            return "l1", 1.0 / reg_param, elasticNet_param
        return "elasticnet", 1.0 / reg_param, elasticNet_param


class _LogisticRegressionParams(_BackendParams, HasFeaturesCol, HasFeaturesCols, HasLabelCol, HasPredictionCol,
                                HasProbabilityCol, HasRawPredictionCol, HasMaxIter, HasRegParam, HasElasticNetParam,
                                HasTol, HasFitIntercept, HasStandardization, HasWeightCol, HasAggregationDepth,
                                HasThreshold, HasThresholds, HasMaxBlockSizeInMB, HasEnableSparseDataOptim,
                                _ClassifierColsMixin):
    family = Param(Params._dummy(), "family", "The name of family: auto, binomial, multinomial",
                   typeConverter=TypeConverters.toString)
    lowerBoundsOnCoefficients = Param(Params._dummy(), "lowerBoundsOnCoefficients", "lower bounds on coefficients")
    upperBoundsOnCoefficients = Param(Params._dummy(), "upperBoundsOnCoefficients", "upper bounds on coefficients")
    lowerBoundsOnIntercepts = Param(Params._dummy(), "lowerBoundsOnIntercepts", "lower bounds on intercepts")
    upperBoundsOnIntercepts = Param(Params._dummy(), "upperBoundsOnIntercepts", "upper bounds on intercepts")

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(maxIter=100, regParam=0.0, elasticNetParam=0.0, tol=1e-6, fitIntercept=True,
                         standardization=True, threshold=0.5, family="auto", aggregationDepth=2,
                         maxBlockSizeInMB=0.0, featuresCol="features", labelCol="label", predictionCol="prediction",
                         probabilityCol="probability", rawPredictionCol="rawPrediction")

    def getFamily(self) -> str:
        return self.getOrDefault("family")


class LogisticRegression(LogisticRegressionClass, _EstimatorSupervised, _LogisticRegressionParams):
    """Distributed logistic regression: fused one-pass loss/gradient HIP kernel + RCCL all-reduce,
    replicated fp64 quasi-Newton driver (L-BFGS, memory 10; OWL-QN problem for L1)."""

    @keyword_only
    def __init__(self, *, featuresCol: Union[str, List[str]] = "features", labelCol: str = "label",
                 predictionCol: str = "prediction", probabilityCol: str = "probability",
                 rawPredictionCol: str = "rawPrediction", maxIter: int = 100, regParam: float = 0.0,
                 elasticNetParam: float = 0.0, tol: float = 1e-6, fitIntercept: bool = True,
                 standardization: bool = True, enable_sparse_data_optim: Optional[bool] = None,
                 float32_inputs: bool = True, num_workers: Optional[int] = None,
                 verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._set_params(**self._input_kwargs)

    def setMaxIter(self, value: int) -> "LogisticRegression":
        return self._set_params(maxIter=value)

    def setRegParam(self, value: float) -> "LogisticRegression":
        return self._set_params(regParam=value)

    def setElasticNetParam(self, value: float) -> "LogisticRegression":
        return self._set_params(elasticNetParam=value)

    def setTol(self, value: float) -> "LogisticRegression":
        return self._set_params(tol=value)

    def setFitIntercept(self, value: bool) -> "LogisticRegression":
        return self._set_params(fitIntercept=value)

    def setStandardization(self, value: bool) -> "LogisticRegression":
        return self._set_params(standardization=value)

    def _supports_sparse(self) -> bool:
        return True

    def _enable_fit_multiple_in_single_pass(self) -> bool:
        return True

    def _supportsTransformEvaluate(self, evaluator: Any) -> bool:
        if type(evaluator).__name__ != "MulticlassClassificationEvaluator":
            return False
        return evaluator.getMetricName() in (
            "f1", "accuracy", "weightedPrecision", "weightedRecall", "weightedTruePositiveRate",
            "weightedFalsePositiveRate", "weightedFMeasure", "truePositiveRateByLabel", "falsePositiveRateByLabel",
            "precisionByLabel", "recallByLabel", "fMeasureByLabel", "hammingLoss", "logLoss")

    def _validate_parameters(self) -> None:
        if self.isSet("weightCol") and self.getOrDefault("weightCol"):
            raise ValueError("weightCol is not supported")

    def _get_fit_func(self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        def _fit(inp: FitInput, ctx: WorkerContext, params: Dict[str, Any]) -> Any:
            from .core.base import CSR
            from .models.logistic import logistic_fit_multi, logistic_stats

            sparse = isinstance(inp.X, CSR)
            stats = logistic_stats(inp.X, inp.y, inp.desc.m, ctx, sparse)
            init = params["cuml_init"]
            maps = params["fit_multiple_params"] or [{}]
            settings = []
            for mp in maps:
                p = dict(init, **mp)
                C = float(p["C"])
                settings.append({"reg": 0.0 if C == 0.0 else 1.0 / C,
                                 "l1_ratio": float(p["l1_ratio"]) if p.get("l1_ratio") is not None else 0.0,
                                 "fit_intercept": bool(p["fit_intercept"]), "standardization": bool(p["standardization"]),
                                 "max_iter": int(p["max_iter"]), "tol": float(p["tol"])})
            # one setting: the single-model path; several: batched passes over X (hyper-parameter batching)
            out = logistic_fit_multi(inp.X, inp.y, inp.desc.m, ctx, settings, sparse=sparse, stats=stats)
            return out if params["fit_multiple_params"] else out[0]

        return _fit

    def _create_model(self, result: Dict[str, Any]) -> "LogisticRegressionModel":
        result = dict(result)
        info = result.pop("_solver", None)  # device QN diagnostics (evaluations, stop reason, pass)
        model = LogisticRegressionModel._from_row(result)
        model._solver_info = info
        return model


class LogisticRegressionModel(LogisticRegressionClass, _ModelWithPredictionCol, _LogisticRegressionParams):
    def __init__(self, coef_: List[List[float]], intercept_: List[float], classes_: List[float], n_cols: int,
                 dtype: str, num_iters: int = 0, objective: float = 0.0) -> None:
        super().__init__(coef_=coef_, intercept_=intercept_, classes_=classes_, n_cols=n_cols, dtype=dtype,
                         num_iters=num_iters, objective=objective)
        self.coef_ = coef_
        self.intercept_ = intercept_
        self.classes_ = classes_
        self.n_cols = n_cols
        self.dtype = dtype
        self.num_iters = num_iters
        self.objective = objective
        self._num_classes = max(len(classes_), 2) if len(coef_) == 1 else len(coef_)

    @property
    def coefficients(self) -> Any:
        if len(self.coef_) == 1:
            return Vectors.dense(self.coef_[0])
        raise Exception("Multinomial models contain a matrix of coefficients, use coefficientMatrix instead.")

    @property
    def intercept(self) -> float:
        if len(self.intercept_) == 1:
            return float(self.intercept_[0])
        raise Exception("Multinomial models contain a vector of intercepts, use interceptVector instead.")

    @property
    def coefficientMatrix(self) -> DenseMatrix:
        rows, cols = len(self.coef_), len(self.coef_[0])
        flat = [float(c) for row in self.coef_ for c in row]
        return DenseMatrix(rows, cols, flat, True)

    @property
    def interceptVector(self) -> Any:
        return compressed_vector(np.asarray(self.intercept_, dtype=np.float64))

    @property
    def numClasses(self) -> int:
        return self._num_classes

    @property
    def hasSummary(self) -> bool:
        return False

    @property
    def summary(self) -> Any:
        raise RuntimeError("No training summary available for this LogisticRegressionModel")

    def _scores_np(self, X: np.ndarray) -> np.ndarray:
        W = np.asarray(self.coef_, dtype=np.float64)
        b = np.asarray(self.intercept_, dtype=np.float64)
        return X @ W.T + b

    def predictRaw(self, value: Any) -> Any:
        s = self._scores_np(as_dense_array(value).reshape(1, -1))[0]
        return Vectors.dense([-s[0], s[0]] if len(s) == 1 else s)

    def predictProbability(self, value: Any) -> Any:
        s = self._scores_np(as_dense_array(value).reshape(1, -1))[0]
        if len(s) == 1:
            p = 1.0 / (1.0 + np.exp(-s[0]))
            return Vectors.dense([1 - p, p])
        e = np.exp(s - s.max())
        return Vectors.dense(e / e.sum())

    def predict(self, value: Any) -> float:
        s = self._scores_np(as_dense_array(value).reshape(1, -1))[0]
        return float(s[0] > 0) if len(s) == 1 else float(np.argmax(s))

    def evaluate(self, dataset: Any) -> Any:
        raise NotImplementedError("evaluate() summaries are not supported; use an Evaluator on transform()")

    def cpu(self) -> Any:
        from .utils.spark_compat import to_spark_logistic_regression_model

        return to_spark_logistic_regression_model(self)

    def _vector_output_cols(self) -> List[str]:
        return [self.getOrDefault("probabilityCol"), self.getOrDefault("rawPredictionCol")]

    def _transform_supports_sparse(self) -> bool:
        return True

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        W = np.asarray(self.coef_, dtype=np.float64)
        b = np.asarray(self.intercept_, dtype=np.float64)
        pc, prc, rc = self.getPredictionCol(), self.getOrDefault("probabilityCol"), self.getOrDefault("rawPredictionCol")
        np_dt = np.float32 if self.dtype == "float32" else np.float64

        def construct(ctx: WorkerContext) -> Tuple[torch.Tensor, torch.Tensor]:
            return torch.from_numpy(W.astype(np_dt)).to(ctx.device), torch.from_numpy(b.astype(np_dt)).to(ctx.device)

        def predict(state: Tuple[torch.Tensor, torch.Tensor], X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            from .core.base import CSR, to_device
            from .models.logistic import logistic_scores

            Wd, bd = state
            Xd = to_device(X, ctx.device, Wd.dtype)
            if isinstance(Xd, CSR):
                from . import ops

                S = ops.csr_spmm(Xd, Wd.T, bd)
            else:
                S = logistic_scores(Xd, Wd, bd)
            S = S.double()
            if S.shape[1] == 1:
                z = S[:, 0]
                p1 = torch.sigmoid(z)
                prob = torch.stack([1 - p1, p1], 1)
                raw = torch.stack([-z, z], 1)
                lab = (z > 0).double()
            else:
                prob = torch.softmax(S, 1)
                raw = S
                lab = S.argmax(1).double()
            return {pc: ctx.output(lab), prc: ctx.output(prob), rc: ctx.output(raw)}

        return construct, predict

    @classmethod
    def _combine(cls, models: List["LogisticRegressionModel"]) -> "LogisticRegressionModel":
        first = models[0]
        out = cls(**first._get_model_attributes())
        first._copyValues(out)
        first._copy_backend_params(out)
        out._combined_models = list(models)
        return out


# ======================================================================================
# RandomForestClassifier
# ======================================================================================
from .tree import _RandomForestEstimator, _RandomForestModel  # noqa: E402


class _RFClassifierParams:
    def setProbabilityCol(self, value: str) -> Any:
        return self._set_params(probabilityCol=value)

    def setRawPredictionCol(self, value: str) -> Any:
        return self._set(rawPredictionCol=value)


class RandomForestClassifier(_RandomForestEstimator, HasProbabilityCol, HasRawPredictionCol, _RFClassifierParams):
    """Random forest classifier grown level-wise on MI355X (LDS histograms, device split search).

    Defaults follow Spark (numTrees=20, maxDepth=5, maxBins=32, impurity="gini"); each rank grows
    its share of the trees on its local rows (reference parity) unless ``split_mode="data_parallel"``.
    """

    _is_classification = True

    @keyword_only
    def __init__(self, *, featuresCol: Union[str, List[str]] = "features", labelCol: str = "label",
                 predictionCol: str = "prediction", probabilityCol: str = "probability",
                 rawPredictionCol: str = "rawPrediction", maxDepth: int = 5, maxBins: int = 32,
                 minInstancesPerNode: int = 1, minInfoGain: float = 0.0, maxMemoryInMB: int = 256,
                 cacheNodeIds: bool = False, checkpointInterval: int = 10, impurity: str = "gini",
                 numTrees: int = 20, featureSubsetStrategy: str = "auto", seed: Optional[int] = None,
                 subsamplingRate: float = 1.0, leafCol: str = "", minWeightFractionPerNode: float = 0.0,
                 weightCol: Optional[str] = None, bootstrap: Optional[bool] = True,
                 num_workers: Optional[int] = None, verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._setDefault(impurity="gini", probabilityCol="probability", rawPredictionCol="rawPrediction")
        self._initialize_backend_params()
        self._set_params(**self._input_kwargs)

    def _supportsTransformEvaluate(self, evaluator: Any) -> bool:
        return type(evaluator).__name__ == "MulticlassClassificationEvaluator"

    def _create_model(self, result: Dict[str, Any]) -> "RandomForestClassificationModel":
        return RandomForestClassificationModel._from_row(result)


class RandomForestClassificationModel(_RandomForestModel, HasProbabilityCol, HasRawPredictionCol,
                                      _RFClassifierParams):
    _is_classification = True

    def __init__(self, trees: List[Dict[str, Any]], n_cols: int, dtype: str = "float32", num_classes: int = 2) -> None:
        super().__init__(trees=trees, n_cols=n_cols, dtype=dtype, num_classes=num_classes)
        self._setDefault(probabilityCol="probability", rawPredictionCol="rawPrediction")

    @property
    def numClasses(self) -> int:
        return self._num_classes

    def _raw_np(self, value: Any) -> np.ndarray:
        return self._raw_sum(np.asarray(as_dense_array(value), dtype=np.float32).reshape(1, -1),
                             torch.device("cpu")).numpy()[0]

    def predictRaw(self, value: Any) -> Any:
        return Vectors.dense(self._raw_np(value))

    def predictProbability(self, value: Any) -> Any:
        r = self._raw_np(value)
        return Vectors.dense(r / r.sum() if r.sum() > 0 else r)

    def predict(self, value: Any) -> float:
        return float(np.argmax(self._raw_np(value)))

    def _vector_output_cols(self) -> List[str]:
        return [self.getOrDefault("probabilityCol"), self.getOrDefault("rawPredictionCol")]

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        pc, prc, rc = self.getPredictionCol(), self.getOrDefault("probabilityCol"), self.getOrDefault("rawPredictionCol")

        def construct(ctx: WorkerContext) -> Any:
            self._pack(ctx.device)
            return ctx.device

        def predict(device: Any, X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            raw = self._raw_sum(X, ctx.device)  # Spark rawPrediction: sum of per-tree class distributions
            tot = raw.sum(1, keepdim=True)
            prob = torch.where(tot > 0, raw / tot.clamp_min(1e-300), raw)
            lab = raw.argmax(1).double()
            return {pc: ctx.output(lab), prc: ctx.output(prob), rc: ctx.output(raw)}

        return construct, predict

    def evaluate(self, dataset: Any) -> Any:
        raise NotImplementedError("use an Evaluator on transform()")
