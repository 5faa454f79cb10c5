"""``pyspark.ml.evaluation``-compatible evaluators for the Spark-free data plane.

``RegressionEvaluator`` (rmse, mse, r2, mae, var), ``MulticlassClassificationEvaluator``
(the 14 Spark metrics) and ``BinaryClassificationEvaluator`` (areaUnderROC / areaUnderPR)
evaluate a transformed DataFrame; the CrossValidator fast path skips the transformed frame
and merges per-partition statistics computed on the device (``metrics/``).
When pyspark is installed its evaluators are accepted as well (same getters).
"""
from __future__ import annotations

from typing import Any, Optional

import numpy as np

from .core.dataframe import DataFrame, as_dataframe
from .core.params import HasLabelCol, HasPredictionCol, HasProbabilityCol, HasRawPredictionCol, Param, Params, \
    TypeConverters, keyword_only
from .metrics import ClassificationSummary, MulticlassMetrics, RegressionMetrics, RegressionSummary, binary_aupr, \
    binary_auc


def _local(dataset: Any, cols: list) -> DataFrame:
    """The evaluated columns as a local DataFrame; a Spark DataFrame is reduced to those columns
    and brought to the driver through Arrow (``toArrow`` on Spark 4, ``toPandas`` before)."""
    from .parallel.spark import is_spark_dataframe

    if is_spark_dataframe(dataset):
        sel = dataset.select(*[c for c in cols if c in dataset.columns])
        if hasattr(sel, "toArrow"):
            return DataFrame([sel.toArrow()])
        return as_dataframe(sel.toPandas())[0]
    return as_dataframe(dataset)[0]


class Evaluator(Params):
    def evaluate(self, dataset: Any, params: Optional[dict] = None) -> float:
        if params:
            return self.copy(params)._evaluate(dataset)
        return self._evaluate(dataset)

    def _evaluate(self, dataset: Any) -> float:
        raise NotImplementedError

    def isLargerBetter(self) -> bool:
        return True

    def getMetricName(self) -> str:
        return self.getOrDefault("metricName")

    def setMetricName(self, value: str) -> "Evaluator":
        return self._set(metricName=value)

    def setLabelCol(self, value: str) -> "Evaluator":
        return self._set(labelCol=value)

    def setPredictionCol(self, value: str) -> "Evaluator":
        return self._set(predictionCol=value)


class RegressionEvaluator(Evaluator, HasLabelCol, HasPredictionCol):
    metricName = Param(Params._dummy(), "metricName", "metric name in evaluation - one of: rmse, mse, r2, mae, var",
                       typeConverter=TypeConverters.toString)
    throughOrigin = Param(Params._dummy(), "throughOrigin", "whether the regression is through the origin.",
                          typeConverter=TypeConverters.toBoolean)
    weightCol = Param(Params._dummy(), "weightCol", "weight column name.", typeConverter=TypeConverters.toString)

    @keyword_only
    def __init__(self, *, predictionCol: str = "prediction", labelCol: str = "label", metricName: str = "rmse",
                 weightCol: Optional[str] = None, throughOrigin: bool = False) -> None:
        super().__init__()
        self._setDefault(metricName="rmse", throughOrigin=False, labelCol="label", predictionCol="prediction")
        self._set(**{k: v for k, v in self._input_kwargs.items() if v is not None})

    def getThroughOrigin(self) -> bool:
        return self.getOrDefault("throughOrigin")

    def isLargerBetter(self) -> bool:
        return self.getMetricName() in ("r2", "var")

    def _evaluate(self, dataset: Any) -> float:
        df = _local(dataset, [self.getOrDefault("labelCol"), self.getOrDefault("predictionCol")])
        y = df.to_numpy(self.getOrDefault("labelCol"), np.float64)
        p = df.to_numpy(self.getOrDefault("predictionCol"), np.float64)
        return RegressionMetrics(RegressionSummary.from_arrays(y, p)).evaluate(self)


class MulticlassClassificationEvaluator(Evaluator, HasLabelCol, HasPredictionCol, HasProbabilityCol):
    metricName = Param(Params._dummy(), "metricName", "metric name in evaluation", typeConverter=TypeConverters.toString)
    metricLabel = Param(Params._dummy(), "metricLabel", "The class whose metric will be computed",
                        typeConverter=TypeConverters.toFloat)
    beta = Param(Params._dummy(), "beta", "The beta value used in weightedFMeasure|fMeasureByLabel",
                 typeConverter=TypeConverters.toFloat)
    eps = Param(Params._dummy(), "eps", "log-loss clipping epsilon", typeConverter=TypeConverters.toFloat)
    weightCol = Param(Params._dummy(), "weightCol", "weight column name.", typeConverter=TypeConverters.toString)

    @keyword_only
    def __init__(self, *, predictionCol: str = "prediction", labelCol: str = "label", metricName: str = "f1",
                 weightCol: Optional[str] = None, metricLabel: float = 0.0, beta: float = 1.0,
                 probabilityCol: str = "probability", eps: float = 1e-15) -> None:
        super().__init__()
        self._setDefault(metricName="f1", metricLabel=0.0, beta=1.0, eps=1e-15, labelCol="label",
                         predictionCol="prediction", probabilityCol="probability")
        self._set(**{k: v for k, v in self._input_kwargs.items() if v is not None})

    def getMetricLabel(self) -> float:
        return self.getOrDefault("metricLabel")

    def getBeta(self) -> float:
        return self.getOrDefault("beta")

    def getEps(self) -> float:
        return self.getOrDefault("eps")

    def isLargerBetter(self) -> bool:
        return self.getMetricName() not in ("weightedFalsePositiveRate", "falsePositiveRateByLabel", "hammingLoss",
                                            "logLoss")

    def _evaluate(self, dataset: Any) -> float:
        df = _local(dataset, [self.getOrDefault(c) for c in ("labelCol", "predictionCol", "probabilityCol")])
        y = df.to_numpy(self.getOrDefault("labelCol"), np.float64)
        p = df.to_numpy(self.getOrDefault("predictionCol"), np.float64)
        prob = None
        if self.getMetricName() == "logLoss":
            prob = df.to_numpy(self.getOrDefault("probabilityCol"), np.float64)
        return MulticlassMetrics(ClassificationSummary.from_arrays(y, p, prob, self.getEps())).evaluate(self)


class BinaryClassificationEvaluator(Evaluator, HasLabelCol, HasRawPredictionCol):
    metricName = Param(Params._dummy(), "metricName", "areaUnderROC|areaUnderPR", typeConverter=TypeConverters.toString)
    numBins = Param(Params._dummy(), "numBins", "number of bins for the curves", typeConverter=TypeConverters.toInt)

    @keyword_only
    def __init__(self, *, rawPredictionCol: str = "rawPrediction", labelCol: str = "label",
                 metricName: str = "areaUnderROC", weightCol: Optional[str] = None, numBins: int = 1000) -> None:
        super().__init__()
        self._setDefault(metricName="areaUnderROC", numBins=1000, labelCol="label", rawPredictionCol="rawPrediction")
        self._set(**{k: v for k, v in self._input_kwargs.items() if v is not None and k != "weightCol"})

    def _evaluate(self, dataset: Any) -> float:
        df = _local(dataset, [self.getOrDefault("labelCol"), self.getOrDefault("rawPredictionCol")])
        y = df.to_numpy(self.getOrDefault("labelCol"), np.float64)
        rc = self.getOrDefault("rawPredictionCol")
        raw = df.to_numpy(rc, np.float64)
        score = raw[:, -1] if raw.ndim == 2 else raw
        if self.getMetricName() == "areaUnderPR":
            return binary_aupr(y, score)
        return binary_auc(y, score)
