"""``tuning.CrossValidator`` / ``CrossValidatorModel`` / ``ParamGridBuilder`` (reference ``tuning.py:39-177``).

Fast path (reference ``tuning.py:91-148``): when the estimator can fit all param maps in one pass
(``fitMultiple`` -> one barrier job) and its models can transform + evaluate all of them in one
pass over the validation fold (``_supportsTransformEvaluate``), each fold costs ONE fit job and
ONE data pass instead of ``numModels`` of each. Folds run in a thread pool of
``min(parallelism, numModels)`` threads. Otherwise it falls back to the generic loop (fit and
evaluate every map separately) — what pyspark's CrossValidator does. The best param map is
refit on the whole dataset.

Folds follow Spark's ``_kFold``: a uniform random number per row (``seed``) assigns row r to fold
``floor(u * numFolds)``; or the integer ``foldCol`` when set.
"""
from __future__ import annotations

import json
import os
import zlib
from multiprocessing.pool import ThreadPool
from typing import Any, Dict, List, Optional, Sequence, Tuple

import numpy as np

from .core.dataframe import as_dataframe
from .core.params import HasSeed, Param, Params, TypeConverters, keyword_only
from .core.persistence import MLReadable, MLWritable, MLReader, MLWriter, _jsonable, _load_class, _read_text, \
    _write_text


class ParamGridBuilder:
    """Builder for a param grid used in grid search-based model selection (pyspark-compatible)."""

    def __init__(self) -> None:
        self._param_grid: Dict[Param, List[Any]] = {}

    def addGrid(self, param: Param, values: Sequence[Any]) -> "ParamGridBuilder":
        self._param_grid[param] = list(values)
        return self

    def baseOn(self, *args: Any) -> "ParamGridBuilder":
        if len(args) == 1 and isinstance(args[0], dict):
            for p, v in args[0].items():
                self.addGrid(p, [v])
        else:
            for p, v in args:
                self.addGrid(p, [v])
        return self

    def build(self) -> List[Dict[Param, Any]]:
        keys = list(self._param_grid.keys())
        grid: List[Dict[Param, Any]] = [{}]
        for k in keys:
            grid = [{**g, k: v} for g in grid for v in self._param_grid[k]]
        return grid


def _gen_avg_and_std_metrics(metrics_all: List[List[float]]) -> Tuple[List[float], List[float]]:
    return list(np.mean(metrics_all, axis=0)), list(np.std(metrics_all, axis=0))


class _CrossValidatorParams(HasSeed):
    estimator = Param(Params._dummy(), "estimator", "estimator to be cross-validated")
    estimatorParamMaps = Param(Params._dummy(), "estimatorParamMaps", "estimator param maps")
    evaluator = Param(Params._dummy(), "evaluator", "evaluator used to select hyper-parameters that maximize the "
                      "validator metric")
    numFolds = Param(Params._dummy(), "numFolds", "number of folds for cross validation",
                     typeConverter=TypeConverters.toInt)
    foldCol = Param(Params._dummy(), "foldCol", "Param for the column name of user specified fold number.",
                    typeConverter=TypeConverters.toString)
    parallelism = Param(Params._dummy(), "parallelism", "the number of threads to use when running parallel "
                        "algorithms (>= 1).", typeConverter=TypeConverters.toInt)
    collectSubModels = Param(Params._dummy(), "collectSubModels", "whether to collect a list of sub-models trained "
                             "during tuning.", typeConverter=TypeConverters.toBoolean)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(numFolds=3, foldCol="", parallelism=1, collectSubModels=False,
                         seed=zlib.crc32(type(self).__name__.encode()) & 0x7FFFFFFF)

    def getEstimator(self) -> Any:
        return self.getOrDefault(self.estimator)

    def getEstimatorParamMaps(self) -> List[Dict[Param, Any]]:
        return self.getOrDefault(self.estimatorParamMaps)

    def getEvaluator(self) -> Any:
        return self.getOrDefault(self.evaluator)

    def getNumFolds(self) -> int:
        return self.getOrDefault(self.numFolds)

    def getFoldCol(self) -> str:
        return self.getOrDefault(self.foldCol)

    def getParallelism(self) -> int:
        return self.getOrDefault(self.parallelism)

    def getCollectSubModels(self) -> bool:
        return self.getOrDefault(self.collectSubModels)

    def setEstimator(self, value: Any) -> Any:
        return self._set(estimator=value)

    def setEstimatorParamMaps(self, value: List[Dict[Param, Any]]) -> Any:
        return self._set(estimatorParamMaps=value)

    def setEvaluator(self, value: Any) -> Any:
        return self._set(evaluator=value)

    def setNumFolds(self, value: int) -> Any:
        return self._set(numFolds=value)

    def setFoldCol(self, value: str) -> Any:
        return self._set(foldCol=value)

    def setParallelism(self, value: int) -> Any:
        return self._set(parallelism=value)

    def setCollectSubModels(self, value: bool) -> Any:
        return self._set(collectSubModels=value)

    def setSeed(self, value: int) -> Any:
        return self._set(seed=value)


def _pyspark_tuning() -> Tuple[Any, Any]:
    try:
        from pyspark.ml.tuning import CrossValidator as _S, CrossValidatorModel as _SM  # type: ignore

        return _S, _SM
    except Exception:  # noqa: BLE001 - pyspark absent: standalone classes
        return None, None


_SparkCV, _SparkCVModel = _pyspark_tuning()
# With pyspark the classes ARE pyspark CrossValidator / CrossValidatorModel subclasses (reference
# tuning.py:39): isinstance checks, pyspark's params and _kFold on Spark DataFrames all hold.
_CV_BASES = (_SparkCV,) if _SparkCV is not None else (_CrossValidatorParams, MLWritable, MLReadable)
_CVM_BASES = (_SparkCVModel,) if _SparkCVModel is not None else (_CrossValidatorParams, MLWritable, MLReadable)


class CrossValidator(*_CV_BASES):  # type: ignore[misc]
    """K-fold cross validation with single-pass multi-model fit and evaluation.

    >>> from spark_rapids_ml_nai_amd.tuning import CrossValidator, ParamGridBuilder
    >>> from spark_rapids_ml_nai_amd.classification import RandomForestClassifier
    >>> from spark_rapids_ml_nai_amd.evaluation import MulticlassClassificationEvaluator
    >>> rfc = RandomForestClassifier()
    >>> grid = ParamGridBuilder().addGrid(rfc.maxBins, [8, 16]).build()
    >>> cv = CrossValidator(estimator=rfc, estimatorParamMaps=grid,
    ...                     evaluator=MulticlassClassificationEvaluator(), parallelism=2)
    """

    @keyword_only
    def __init__(self, *, estimator: Any = None, estimatorParamMaps: Optional[List[Dict[Param, Any]]] = None,
                 evaluator: Any = None, numFolds: int = 3, seed: Optional[int] = None, parallelism: int = 1,
                 collectSubModels: bool = False, foldCol: str = "") -> None:
        kwargs = dict(self._input_kwargs)  # a pyspark base __init__ resets _input_kwargs
        super().__init__()
        self._set(**{k: v for k, v in kwargs.items() if v is not None})

    def fit(self, dataset: Any, params: Optional[Dict[Param, Any]] = None) -> "CrossValidatorModel":
        if params:
            return self.copy(params)._fit(dataset)
        return self._fit(dataset)

    def _kFold(self, dataset: Any) -> List[Tuple[Any, Any]]:
        from .parallel.spark import is_spark_dataframe

        if is_spark_dataframe(dataset):  # pyspark's rand(seed)-column split, evaluated by Spark
            return super()._kFold(dataset)  # type: ignore[misc]
        nFolds = self.getNumFolds()
        foldCol = self.getFoldCol()
        m = dataset.count()
        if foldCol:
            fold = dataset.to_numpy(foldCol).astype(np.int64)
            if np.any((fold < 0) | (fold >= nFolds)):
                raise ValueError("Fold number must be in range [0, %d)" % nFolds)
        else:
            u = np.random.default_rng(self.getOrDefault(self.seed)).random(m)
            fold = np.minimum((u * nFolds).astype(np.int64), nFolds - 1)
        out = []
        for i in range(nFolds):
            test = fold == i
            train, validation = dataset.filter(~test), dataset.filter(test)
            if foldCol:
                train, validation = train.drop(foldCol), validation.drop(foldCol)
            out.append((train, validation))
        return out

    def _fit(self, dataset: Any) -> "CrossValidatorModel":
        from .parallel.spark import is_spark_dataframe

        est = self.getEstimator()
        eva = self.getEvaluator()
        fast = hasattr(est, "_supportsTransformEvaluate") and est._supportsTransformEvaluate(eva)
        if is_spark_dataframe(dataset):
            if not fast:  # not one of ours / unsupported evaluator: pyspark's generic loop
                return super()._fit(dataset)  # type: ignore[misc]
            df = dataset
        else:
            df, _ = as_dataframe(dataset)
        epm = self.getEstimatorParamMaps()
        numModels = len(epm)
        nFolds = self.getNumFolds()
        collect = self.getCollectSubModels()
        datasets = self._kFold(df)

        def single_pass(fold: int) -> Tuple[int, List[float], Optional[List[Any]]]:
            train, validation = datasets[fold]
            models = [None] * numModels
            for idx, model in est.fitMultiple(train, epm):
                models[idx] = model
            combined = models[0]._combine(models)
            metrics = combined._transformEvaluate(validation, eva)
            return fold, metrics, models if collect else None

        def generic(fold: int) -> Tuple[int, List[float], Optional[List[Any]]]:
            train, validation = datasets[fold]
            models = [None] * numModels
            for idx, model in est.fitMultiple(train, epm):
                models[idx] = model
            metrics = [float(eva.evaluate(models[j].transform(validation, epm[j]))) for j in range(numModels)]
            return fold, metrics, models if collect else None

        task = single_pass if fast else generic
        metrics_all: List[List[float]] = [[0.0] * numModels for _ in range(nFolds)]
        subModels: Optional[List[List[Any]]] = [[None] * numModels for _ in range(nFolds)] if collect else None
        nthreads = max(1, min(self.getParallelism(), numModels))
        if nthreads == 1:
            results = [task(f) for f in range(nFolds)]
        else:
            with ThreadPool(processes=nthreads) as pool:
                results = list(pool.imap_unordered(task, range(nFolds)))
        for fold, metrics, models in results:
            metrics_all[fold] = metrics
            if collect and subModels is not None:
                subModels[fold] = models  # type: ignore[assignment]
        avg, std = _gen_avg_and_std_metrics(metrics_all)
        best = int(np.argmax(avg)) if eva.isLargerBetter() else int(np.argmin(avg))
        bestModel = est.fit(df, epm[best])
        model = CrossValidatorModel(bestModel, avg, subModels, std)
        return self._copyValues(model)

    def copy(self, extra: Optional[Dict[Param, Any]] = None) -> "CrossValidator":
        new = super().copy(extra)
        if self.isDefined(self.estimator):
            new.setEstimator(self.getEstimator().copy(extra))
        if self.isDefined(self.evaluator):
            new.setEvaluator(self.getEvaluator().copy(extra))
        return new

    def write(self) -> MLWriter:
        return _CVWriter(self)

    @classmethod
    def read(cls) -> MLReader:
        return _CVReader(cls)


class CrossValidatorModel(*_CVM_BASES):  # type: ignore[misc]
    def __init__(self, bestModel: Any = None, avgMetrics: Optional[List[float]] = None,
                 subModels: Optional[List[List[Any]]] = None, stdMetrics: Optional[List[float]] = None) -> None:
        if _SparkCVModel is not None:
            super().__init__(bestModel, avgMetrics, subModels, stdMetrics)
        else:
            super().__init__()
        self.bestModel = bestModel
        self.avgMetrics = list(avgMetrics or [])
        self.subModels = subModels
        self.stdMetrics = list(stdMetrics or [])

    def transform(self, dataset: Any, params: Optional[Dict[Param, Any]] = None) -> Any:
        return self.bestModel.transform(dataset, params)

    def copy(self, extra: Optional[Dict[Param, Any]] = None) -> "CrossValidatorModel":
        sub = [[m.copy(extra) for m in fold] for fold in self.subModels] if self.subModels else None
        out = CrossValidatorModel(self.bestModel.copy(extra), self.avgMetrics, sub, self.stdMetrics)
        return self._copyValues(out, extra)

    def write(self) -> MLWriter:
        return _CVWriter(self)

    @classmethod
    def read(cls) -> MLReader:
        return _CVReader(cls)


# ------------------------------------------------------------------------------------------
# persistence: metadata + estimator + evaluator + param maps (+ bestModel / subModels)
# ------------------------------------------------------------------------------------------
def _save_params_obj(obj: Any, path: str) -> None:
    """Evaluators and other plain Params objects: class + explicitly set params as JSON."""
    if hasattr(obj, "write"):
        try:
            obj.write().overwrite().save(path)
            return
        except NotImplementedError:
            pass
    md = {"class": obj.__class__.__module__ + "." + obj.__class__.__name__, "uid": obj.uid,
          "paramMap": {p.name: _jsonable(v) for p, v in obj._paramMap.items()}}
    _write_text(os.path.join(path, "metadata"), json.dumps(md))


def _load_params_obj(path: str) -> Any:
    md = json.loads(_read_text(os.path.join(path, "metadata")))
    cls = _load_class(md["class"])
    if "paramMap" in md and not os.path.exists(os.path.join(path, "data")) and "_cuml_params" not in md:
        inst = cls()
        inst._resetUid(md["uid"])
        for k, v in md["paramMap"].items():
            if inst.hasParam(k):
                inst._set(**{k: v})
        return inst
    return cls.load(path)


def _epm_to_json(epm: List[Dict[Param, Any]]) -> List[List[Dict[str, Any]]]:
    return [[{"parent": p.parent, "name": p.name, "value": _jsonable(v)} for p, v in pm.items()] for pm in epm]


def _epm_from_json(data: List[List[Dict[str, Any]]], est: Any) -> List[Dict[Param, Any]]:
    return [{est.getParam(d["name"]): d["value"] for d in pm} for pm in data]


class _CVWriter(MLWriter):
    def saveImpl(self, path: str) -> None:
        inst = self.instance
        is_model = isinstance(inst, CrossValidatorModel)
        extra: Dict[str, Any] = {"estimatorParamMaps": _epm_to_json(inst.getEstimatorParamMaps())
                                 if inst.isDefined(inst.estimatorParamMaps) else []}
        if is_model:
            extra.update(avgMetrics=inst.avgMetrics, stdMetrics=inst.stdMetrics,
                         persistSubModels=inst.subModels is not None)
        md = {"class": inst.__class__.__module__ + "." + inst.__class__.__name__, "uid": inst.uid,
              "paramMap": {p.name: _jsonable(v) for p, v in inst._paramMap.items()
                           if p.name not in ("estimator", "evaluator", "estimatorParamMaps")}}
        md.update(extra)
        _write_text(os.path.join(path, "metadata"), json.dumps(md))
        if inst.isDefined(inst.estimator):
            _save_params_obj(inst.getEstimator(), os.path.join(path, "estimator"))
        if inst.isDefined(inst.evaluator):
            _save_params_obj(inst.getEvaluator(), os.path.join(path, "evaluator"))
        if is_model:
            inst.bestModel.write().overwrite().save(os.path.join(path, "bestModel"))
            if inst.subModels is not None:
                for f, fold in enumerate(inst.subModels):
                    for j, m in enumerate(fold):
                        m.write().overwrite().save(os.path.join(path, "subModels", "fold%d" % f, str(j)))


class _CVReader(MLReader):
    def load(self, path: str) -> Any:
        md = json.loads(_read_text(os.path.join(path, "metadata")))
        cls = _load_class(md["class"])
        est = _load_params_obj(os.path.join(path, "estimator")) if os.path.exists(os.path.join(path, "estimator")) \
            else None
        eva = _load_params_obj(os.path.join(path, "evaluator")) if os.path.exists(os.path.join(path, "evaluator")) \
            else None
        if cls is CrossValidatorModel:
            best_md = json.loads(_read_text(os.path.join(path, "bestModel", "metadata")))
            best = _load_class(best_md["class"]).load(os.path.join(path, "bestModel"))
            sub = None
            if md.get("persistSubModels"):
                sub = []
                fdir = os.path.join(path, "subModels")
                for f in sorted(os.listdir(fdir), key=lambda s: int(s[4:])):
                    fold = []
                    for j in sorted(os.listdir(os.path.join(fdir, f)), key=int):
                        mp = os.path.join(fdir, f, j)
                        mmd = json.loads(_read_text(os.path.join(mp, "metadata")))
                        fold.append(_load_class(mmd["class"]).load(mp))
                    sub.append(fold)
            inst = CrossValidatorModel(best, md.get("avgMetrics"), sub, md.get("stdMetrics"))
        else:
            inst = cls()
        inst._resetUid(md["uid"])
        for k, v in md.get("paramMap", {}).items():
            if inst.hasParam(k):
                inst._set(**{k: v})
        if est is not None:
            inst._set(estimator=est)
            inst._set(estimatorParamMaps=_epm_from_json(md.get("estimatorParamMaps", []), est))
        if eva is not None:
            inst._set(evaluator=eva)
        return inst
