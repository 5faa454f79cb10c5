"""Spark-ML-compatible Param system plus the Spark<->backend parameter mapping layer.

The reference builds on ``pyspark.ml.param`` (``python/src/spark_rapids_ml/params.py:131-554``).
pyspark is an optional dependency here, so this module provides an API-compatible
``Param``/``Params``/``TypeConverters``/``keyword_only`` implementation (same method names and
semantics: defaults vs. user-set values, ``copy(extra)``, ``extractParamMap``, ``explainParams``)
and, on top of it, ``_BackendParams`` — the Spark-param <-> device-solver kwarg mapping:

* a Spark Param mapped to ``None`` raises when it is set (unsupported),
* mapped to ``""`` warns and is ignored,
* value mappers translate enum-like values (``params.py:137-212`` of the reference),
* ``_set_params`` accepts Spark names, backend names, ``num_workers`` and ``float32_inputs``.

The backend kwargs are exposed as ``backend_params`` with the reference's ``cuml_params`` kept
as an alias so user code written against the reference keeps working.
"""
from __future__ import annotations

import os
import warnings
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple, TypeVar, Union


__all__ = [
    "Param",
    "Params",
    "TypeConverters",
    "keyword_only",
    "_BackendParams",
]


# --------------------------------------------------------------------------------------
# Param API: pyspark's own classes when pyspark is importable (estimators then are genuine
# pyspark.ml Params/Estimators/Models that Pipeline / CrossValidator / evaluators accept), else the
# API-compatible built-in implementation.
# --------------------------------------------------------------------------------------
def _use_pyspark() -> bool:
    if os.environ.get("SRML_PYSPARK", "1") == "0":
        return False
    try:
        import pyspark.ml.param  # noqa: F401

        return True
    except Exception:  # noqa: BLE001
        return False


PYSPARK_PARAMS = _use_pyspark()
if PYSPARK_PARAMS:
    from pyspark import keyword_only  # type: ignore  # noqa: F401
    from pyspark.ml.param import Param, Params, TypeConverters  # type: ignore  # noqa: F401
else:
    from ._params_builtin import Param, Params, TypeConverters, keyword_only  # noqa: F401

P_ = TypeVar("P_", bound=Params)


# --------------------------------------------------------------------------------------
# Shared Spark params (pyspark.ml.param.shared equivalents that the API needs)
# --------------------------------------------------------------------------------------
def _shared(name: str, doc: str, conv: Callable, getter: str) -> type:
    """``Has<Name>`` mixin: pyspark's own ``pyspark.ml.param.shared`` class when pyspark is in use
    (isinstance checks in pyspark code then hold), else a built-in class with the same Param."""
    cls_name = "Has" + name[0].upper() + name[1:]
    if PYSPARK_PARAMS:
        try:
            import pyspark.ml.param.shared as _sh  # type: ignore

            if hasattr(_sh, cls_name):
                return getattr(_sh, cls_name)
        except Exception:  # noqa: BLE001
            pass

    def _get(self: Any) -> Any:
        return self.getOrDefault(getattr(self, name))

    cls = type(
        cls_name,
        (Params,),
        {name: Param(Params._dummy(), name, doc, typeConverter=conv), getter: _get},
    )
    return cls


HasFeaturesCol = _shared("featuresCol", "features column name.", TypeConverters.toString, "getFeaturesCol")
HasFeaturesCols = _shared(
    "featuresCols", "features column names for multi-column input.", TypeConverters.toListString, "getFeaturesCols"
)
HasInputCol = _shared("inputCol", "input column name.", TypeConverters.toString, "getInputCol")
HasInputCols = _shared("inputCols", "input column names.", TypeConverters.toListString, "getInputCols")
HasOutputCol = _shared("outputCol", "output column name.", TypeConverters.toString, "getOutputCol")
HasLabelCol = _shared("labelCol", "label column name.", TypeConverters.toString, "getLabelCol")
HasPredictionCol = _shared("predictionCol", "prediction column name.", TypeConverters.toString, "getPredictionCol")
HasProbabilityCol = _shared(
    "probabilityCol",
    "Column name for predicted class conditional probabilities.",
    TypeConverters.toString,
    "getProbabilityCol",
)
HasRawPredictionCol = _shared(
    "rawPredictionCol", "raw prediction (a.k.a. confidence) column name.", TypeConverters.toString, "getRawPredictionCol"
)
HasMaxIter = _shared("maxIter", "max number of iterations (>= 0).", TypeConverters.toInt, "getMaxIter")
HasTol = _shared("tol", "the convergence tolerance for iterative algorithms (>= 0).", TypeConverters.toFloat, "getTol")
HasSeed = _shared("seed", "random seed.", TypeConverters.toInt, "getSeed")
HasRegParam = _shared("regParam", "regularization parameter (>= 0).", TypeConverters.toFloat, "getRegParam")
HasElasticNetParam = _shared(
    "elasticNetParam",
    "the ElasticNet mixing parameter, in range [0, 1]. For alpha = 0, the penalty is an L2 penalty. "
    "For alpha = 1, it is an L1 penalty.",
    TypeConverters.toFloat,
    "getElasticNetParam",
)
HasFitIntercept = _shared("fitIntercept", "whether to fit an intercept term.", TypeConverters.toBoolean, "getFitIntercept")
HasStandardization = _shared(
    "standardization",
    "whether to standardize the training features before fitting the model.",
    TypeConverters.toBoolean,
    "getStandardization",
)
HasWeightCol = _shared(
    "weightCol",
    "weight column name. If this is not set or empty, we treat all instance weights as 1.0.",
    TypeConverters.toString,
    "getWeightCol",
)
HasAggregationDepth = _shared(
    "aggregationDepth", "suggested depth for treeAggregate (>= 2).", TypeConverters.toInt, "getAggregationDepth"
)
HasMaxBlockSizeInMB = _shared(
    "maxBlockSizeInMB",
    "maximum memory in MB for stacking input data into blocks.",
    TypeConverters.toFloat,
    "getMaxBlockSizeInMB",
)
HasSolver = _shared("solver", "the solver algorithm for optimization.", TypeConverters.toString, "getSolver")
HasLoss = _shared("loss", "the loss function to be optimized.", TypeConverters.toString, "getLoss")
HasThreshold = _shared(
    "threshold", "threshold in binary classification prediction, in range [0, 1].", TypeConverters.toFloat, "getThreshold"
)
HasThresholds = _shared(
    "thresholds", "Thresholds in multi-class classification.", TypeConverters.toListFloat, "getThresholds"
)
HasDistanceMeasure = _shared(
    "distanceMeasure",
    "the distance measure. Supported options: 'euclidean' and 'cosine'.",
    TypeConverters.toString,
    "getDistanceMeasure",
)
HasCheckpointInterval = _shared(
    "checkpointInterval", "set checkpoint interval (>= 1) or disable checkpoint (-1).", TypeConverters.toInt,
    "getCheckpointInterval",
)
HasLeafCol = _shared("leafCol", "Leaf indices column name.", TypeConverters.toString, "getLeafCol")


class HasIDCol(Params):
    """Mixin for param idCol (reference ``params.py:90-128``)."""

    idCol = Param(Params._dummy(), "idCol", "id column name.", typeConverter=TypeConverters.toString)

    def getIdCol(self) -> str:
        return self.getOrDefault("idCol")

    def _ensureIdCol(self, df: Any) -> Any:
        """Add a monotonically increasing id column unless the user set one that exists (a Spark
        DataFrame gets ``monotonically_increasing_id()``, reference ``params.py:107-128``)."""
        def add(d: Any) -> Any:
            if hasattr(d, "with_row_id"):
                # under torchrun the frame is this rank's shard: ids start at the rank's global
                # row offset, so they are unique across ranks (collective, every rank calls it)
                from ..parallel.context import spmd_row_offset

                return d.with_row_id(self.getIdCol(), spmd_row_offset(d.count()))
            from pyspark.sql import functions as F  # type: ignore

            return d.withColumn(self.getIdCol(), F.monotonically_increasing_id())

        if not self.isSet("idCol"):
            while self.getIdCol() in df.columns:
                self._set(**{"idCol": self.getIdCol() + "_dedup"})
            return add(df)
        if self.getIdCol() not in df.columns:
            return add(df)
        return df


class HasEnableSparseDataOptim(Params):
    """enable_sparse_data_optim: None=auto (first row decides), True=CSR, False=dense."""

    enable_sparse_data_optim = Param(
        Params._dummy(),
        "enable_sparse_data_optim",
        "If None, use sparse arrays when the first vector of the features column is sparse; "
        "if True always build CSR; if False always densify.",
        typeConverter=TypeConverters.toBoolean,
    )

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(enable_sparse_data_optim=None)


# --------------------------------------------------------------------------------------
# Spark <-> backend parameter mapping
# --------------------------------------------------------------------------------------
class ParamBridge:
    """Translation table between one class's Spark ML Params and its device-solver kwargs.

    Built from the class hooks ``_param_mapping()`` (Spark name -> backend name, ``""`` = accepted
    but unused, ``None`` = unsupported) and ``_param_value_mapping()`` (backend name -> value
    translator returning ``None`` for unsupported values). Every estimator / model routes its
    parameter traffic (constructor kwargs, setters, ``copy(extra)``, ``clear``, ``fitMultiple``
    param maps) through ``lookup`` + ``to_backend`` so the semantics live in one place
    (reference behaviour: ``python/src/spark_rapids_ml/params.py:268-531``).
    """

    UNSUPPORTED = None
    IGNORED = ""

    def __init__(self, names: Dict[str, Optional[str]], values: Dict[str, Callable[[Any], Any]]) -> None:
        self.names = dict(names)
        self.values = dict(values)

    def lookup(self, spark_name: str, strict: bool) -> Optional[str]:
        """Backend kwarg for a Spark Param; ``strict`` raises on unsupported params and warns on
        ignored ones (silent lookups just return None for both)."""
        if spark_name not in self.names:
            return None
        target = self.names[spark_name]
        if target is self.UNSUPPORTED:
            if strict:
                raise ValueError(f"Spark Param '{spark_name}' is not supported on the device backend.")
            return None
        if target == self.IGNORED:
            if strict:
                warnings.warn(f"Spark Param '{spark_name}' is not used by the device backend.")
            return None
        return target

    def to_backend(self, backend_name: str, value: Any) -> Any:
        conv = self.values.get(backend_name)
        if conv is None:
            return value
        out = conv(value)
        if out is None:
            raise ValueError(f"Value '{value}' for '{backend_name}' param is unsupported")
        return out

    def spark_names_for(self, backend_name: str) -> List[str]:
        return [k for k, v in self.names.items() if v == backend_name]

    def conflicting(self, kwargs: Dict[str, Any]) -> List[Tuple[str, str]]:
        """(spark, backend) name pairs that were BOTH given (they alias one value)."""
        return [(sp, be) for sp, be in self.names.items()
                if be and sp != be and sp in kwargs and be in kwargs]


class _BackendClass:
    """Helper hooks for mapping Spark ML Params to device-solver kwargs."""

    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        """Spark Param name -> backend kwarg name ('' = ignore with warning, None = unsupported)."""
        return {}

    @classmethod
    def _param_value_mapping(cls) -> Dict[str, Callable[[Any], Union[None, str, float, int]]]:
        """backend kwarg name -> function mapping a Spark value to a backend value (None = unsupported)."""
        return {}

    @classmethod
    def _bridge(cls) -> ParamBridge:
        return ParamBridge(cls._param_mapping(), cls._param_value_mapping())

    def _get_backend_params_default(self) -> Dict[str, Any]:
        raise NotImplementedError()


def _route_columns(single: str, multi: str) -> Callable[[Any, Any], None]:
    """``inputCol`` / ``featuresCol`` accept one name or a list (which lands in the plural Param)."""

    def route(obj: Any, value: Any) -> None:
        if isinstance(value, (list, tuple)):
            obj._set(**{multi: list(value)})
        elif isinstance(value, str):
            obj._set(**{single: value})

    return route


class _BackendParams(_BackendClass, Params):
    """Common param handling for every estimator and model (reference ``params.py:215-554``):
    Spark Params on the Params side, device kwargs in ``backend_params`` (``cuml_params`` alias),
    kept consistent by ``ParamBridge``."""

    _backend_params: Dict[str, Any] = {}
    _num_workers: Optional[int] = None
    _float32_inputs: bool = True

    # kwargs that are neither Spark Params nor backend kwargs
    _FRAMEWORK_KWARGS: Dict[str, Callable[[Any, Any], None]] = {
        "inputCol": _route_columns("inputCol", "inputCols"),
        "featuresCol": _route_columns("featuresCol", "featuresCols"),
        "num_workers": lambda obj, v: setattr(obj, "_num_workers", v),
        "float32_inputs": lambda obj, v: setattr(obj, "_float32_inputs", v),
    }

    # --- backend kwargs ------------------------------------------------------------
    @property
    def backend_params(self) -> Dict[str, Any]:
        return self._backend_params

    @property
    def cuml_params(self) -> Dict[str, Any]:
        """Alias kept for source compatibility with spark-rapids-ml user code."""
        return self._backend_params

    @property
    def num_workers(self) -> int:
        """Number of device workers (one rank per GPU)."""
        from ..parallel.context import infer_num_workers

        if self._num_workers is None:
            return infer_num_workers()
        if self._num_workers < 1:
            raise ValueError("num_workers must be >= 1")
        return self._num_workers

    @num_workers.setter
    def num_workers(self, value: int) -> None:
        self._num_workers = value

    def _initialize_backend_params(self) -> None:
        """Backend defaults, then every mapped Spark Param's default pushed through the bridge."""
        self._backend_params = self._get_backend_params_default()
        for name in self._bridge().names:
            if self.hasParam(name) and self.hasDefault(name):
                self._set_backend_param(name, self.getOrDefault(name))

    _initialize_cuml_params = _initialize_backend_params  # reference-compatible name

    def _mirror_spark(self, name: str, value: Any) -> None:
        """Spark Param set by name: record it and translate it into the backend kwarg."""
        self._set(**{name: value})
        self._set_backend_param(name, value, silent=False)

    def _mirror_backend(self, name: str, value: Any) -> None:
        """Backend kwarg set by name: store it and reflect it in the Spark Params that alias it
        (best effort: a backend value the Spark Param's type converter rejects stays backend-only)."""
        self._backend_params[name] = value
        for spark_name in self._bridge().spark_names_for(name):
            if not self.hasParam(spark_name):
                continue
            try:
                self._set(**{spark_name: value})
            except TypeError:
                continue

    def _set_params(self: "BP", **kwargs: Any) -> "BP":
        clash = self._bridge().conflicting(kwargs)
        if clash:
            sp, be = clash[0]
            raise ValueError(f"'{be}' is an alias of '{sp}', set one or the other.")
        for key, value in kwargs.items():
            special = self._FRAMEWORK_KWARGS.get(key)
            if special is not None:
                special(self, value)
            elif self.hasParam(key):
                self._mirror_spark(key, value)
            elif key in self._backend_params:
                self._mirror_backend(key, value)
            else:
                raise ValueError(f"Unsupported param '{key}'.")
        return self

    def copy(self: "BP", extra: Optional[Dict[Param, Any]] = None) -> "BP":
        """Params copy (Spark semantics) with ``extra`` also translated into the backend kwargs."""
        clone: BP = super().copy(extra)  # type: ignore[assignment]
        backend = dict(clone._backend_params)
        bridge = self._bridge()
        for param, value in (extra or {}).items():
            if not isinstance(param, Param):
                raise TypeError("Expecting a valid instance of Param, but received: {}".format(param))
            target = bridge.lookup(param.name, strict=True)
            if target is not None:
                backend[target] = bridge.to_backend(target, value)
        clone._backend_params = backend
        return clone

    def clear(self, param: Param) -> None:
        """Unset a Spark Param and restore its backend kwarg from the Param's default."""
        super().clear(param)
        target = self._bridge().names.get(param.name)
        if target:
            self._backend_params[target] = self._get_backend_mapping_value(target, self.getOrDefault(param.name))

    def _copy_backend_params(self, to: "BP") -> "BP":
        to._backend_params.update({k: v for k, v in self._backend_params.items() if k in to._backend_params})
        return to

    _copy_cuml_params = _copy_backend_params

    def _get_input_columns(self) -> Tuple[Optional[str], Optional[List[str]]]:
        """(single column, None) or (None, column list), plural Params first."""
        for plural, single in (("inputCols", "inputCol"), ("featuresCols", "featuresCol")):
            if self.hasParam(plural) and self.isDefined(plural):
                return None, self.getOrDefault(plural)
            if self.hasParam(single) and self.isDefined(single):
                return self.getOrDefault(single), None
        raise ValueError("Please set inputCol(s) or featuresCol(s)")

    def _get_backend_param(self, spark_param: str, silent: bool = True) -> Optional[str]:
        return self._bridge().lookup(spark_param, strict=not silent)

    _get_cuml_param = _get_backend_param

    def _set_backend_param(self, spark_param: str, spark_value: Any, silent: bool = True) -> None:
        bridge = self._bridge()
        target = bridge.lookup(spark_param, strict=not silent)
        if target is None:
            return
        try:
            self._backend_params[target] = bridge.to_backend(target, spark_value)
        except ValueError:
            names = spark_param if target == spark_param else f"{target} or {spark_param}"
            raise ValueError(f"{names} given invalid value {spark_value}")

    _set_cuml_param = _set_backend_param

    def _get_backend_mapping_value(self, k: str, v: Any) -> Any:
        return self._bridge().to_backend(k, v)

    _get_cuml_mapping_value = _get_backend_mapping_value


BP = TypeVar("BP", bound=_BackendParams)


def _params_getters_setters(cls: type, names: Iterable[str]) -> None:
    """Attach ``getX``/``setX`` methods for Params declared on ``cls`` (keeps API surface uniform)."""
    for n in names:
        cap = n[0].upper() + n[1:]
        if not hasattr(cls, "get" + cap):
            setattr(cls, "get" + cap, lambda self, _n=n: self.getOrDefault(_n))
        if not hasattr(cls, "set" + cap):
            def _setter(self: Any, value: Any, _n: str = n) -> Any:
                return self._set_params(**{_n: value})

            setattr(cls, "set" + cap, _setter)


class _FeaturesColMixin:
    """featuresCol / featuresCols (single vector/array column or multiple numeric columns)."""

    def getFeaturesCol(self) -> Union[str, List[str]]:  # type: ignore[override]
        if self.isDefined("featuresCols"):
            return self.getOrDefault("featuresCols")
        if self.isDefined("featuresCol"):
            return self.getOrDefault("featuresCol")
        raise RuntimeError("featuresCol is not set")

    def setFeaturesCol(self, value: Union[str, List[str]]) -> Any:
        if isinstance(value, str):
            return self._set_params(featuresCol=value)
        return self._set_params(featuresCols=value)

    def setFeaturesCols(self, value: List[str]) -> Any:
        return self._set_params(featuresCols=value)

    def setLabelCol(self, value: str) -> Any:
        return self._set_params(labelCol=value)

    def setPredictionCol(self, value: str) -> Any:
        return self._set_params(predictionCol=value)
