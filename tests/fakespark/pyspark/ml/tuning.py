"""``pyspark.ml.tuning`` slice: ``CrossValidator`` (pyspark's constructor, params, ``_kFold`` by a
``rand(seed)`` column and the generic per-param-map ``_fit``), ``CrossValidatorModel``,
``ParamGridBuilder`` — so the library's subclass is exercised against the pyspark base class."""
import numpy as np

from spark_rapids_ml_nai_amd.core._params_builtin import Param, Params, TypeConverters, keyword_only

from . import Estimator, Model
from ..sql import functions as F


class ParamGridBuilder:
    def __init__(self):
        self._param_grid = {}

    def addGrid(self, param, values):
        self._param_grid[param] = list(values)
        return self

    def build(self):
        grid = [{}]
        for k, vs in self._param_grid.items():
            grid = [{**g, k: v} for g in grid for v in vs]
        return grid


class _ValidatorParams(Params):
    estimator = Param(Params._dummy(), "estimator", "estimator to be cross-validated")
    estimatorParamMaps = Param(Params._dummy(), "estimatorParamMaps", "estimator param maps")
    evaluator = Param(Params._dummy(), "evaluator", "evaluator")
    seed = Param(Params._dummy(), "seed", "random seed.", typeConverter=TypeConverters.toInt)
    numFolds = Param(Params._dummy(), "numFolds", "number of folds", typeConverter=TypeConverters.toInt)
    foldCol = Param(Params._dummy(), "foldCol", "fold column", typeConverter=TypeConverters.toString)
    parallelism = Param(Params._dummy(), "parallelism", "threads", typeConverter=TypeConverters.toInt)
    collectSubModels = Param(Params._dummy(), "collectSubModels", "collect sub-models",
                             typeConverter=TypeConverters.toBoolean)

    def __init__(self):
        super().__init__()
        self._setDefault(numFolds=3, foldCol="", parallelism=1, collectSubModels=False, seed=7)

    def getEstimator(self):
        return self.getOrDefault(self.estimator)

    def getEstimatorParamMaps(self):
        return self.getOrDefault(self.estimatorParamMaps)

    def getEvaluator(self):
        return self.getOrDefault(self.evaluator)

    def getNumFolds(self):
        return self.getOrDefault(self.numFolds)

    def getFoldCol(self):
        return self.getOrDefault(self.foldCol)

    def getParallelism(self):
        return self.getOrDefault(self.parallelism)

    def getCollectSubModels(self):
        return self.getOrDefault(self.collectSubModels)

    def getSeed(self):
        return self.getOrDefault(self.seed)


class CrossValidator(Estimator, _ValidatorParams):
    @keyword_only
    def __init__(self, *, estimator=None, estimatorParamMaps=None, evaluator=None, numFolds=3, seed=None,
                 parallelism=1, collectSubModels=False, foldCol=""):
        super().__init__()
        self._set(**{k: v for k, v in self._input_kwargs.items() if v is not None})

    def _kFold(self, dataset):
        nFolds = self.getOrDefault(self.numFolds)
        h = 1.0 / nFolds
        randCol = self.uid + "_rand"
        df = dataset.withColumn(randCol, F.rand(self.getOrDefault(self.seed)))
        out = []
        for i in range(nFolds):
            cond = (df[randCol] >= i * h) & (df[randCol] < (i + 1) * h)
            out.append((df.filter(~cond), df.filter(cond)))
        return out

    def _fit(self, dataset):
        est, eva, epm = self.getEstimator(), self.getEvaluator(), self.getEstimatorParamMaps()
        metrics_all = []
        for train, validation in self._kFold(dataset):
            metrics_all.append([eva.evaluate(est.fit(train, pm).transform(validation, pm)) for pm in epm])
        avg = list(np.mean(metrics_all, axis=0))
        best = int(np.argmax(avg) if eva.isLargerBetter() else np.argmin(avg))
        return self._copyValues(CrossValidatorModel(est.fit(dataset, epm[best]), avg, None,
                                                    list(np.std(metrics_all, axis=0))))


class CrossValidatorModel(Model, _ValidatorParams):
    def __init__(self, bestModel, avgMetrics=None, subModels=None, stdMetrics=None):
        super().__init__()
        self.bestModel, self.avgMetrics = bestModel, list(avgMetrics or [])
        self.subModels, self.stdMetrics = subModels, list(stdMetrics or [])

    def _transform(self, dataset):
        return self.bestModel.transform(dataset)
