"""Mergeable evaluation statistics computed inside the transform pass.

Reference: ``metrics/__init__.py:21-40`` (EvalMetricInfo), ``metrics/MulticlassMetrics.py``,
``metrics/RegressionMetrics.py``. Each partition (and each model of a ``_combine``d batch)
produces a small sufficient-statistics record on the device — per-class true/false positive
and label counts (+ summed log loss) for classification, [label, label-prediction, prediction]
moments for regression — which are merged on the driver and evaluated with Spark's formulas.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from enum import Enum
from typing import Any, Dict, List, Optional

import numpy as np


class transform_evaluate_metric(str, Enum):
    accuracy_like = "accuracy_like"
    log_loss = "log_loss"
    regression = "regression"


@dataclass
class EvalMetricInfo:
    eps: float = 1.0e-15
    numBins: int = 1000
    eval_metric: Optional[str] = None


# --------------------------------------------------------------------------------------
# regression
# --------------------------------------------------------------------------------------
@dataclass
class RegressionSummary:
    """Moments of [label, label - prediction, prediction] (Spark ``SummarizerBuffer`` semantics)."""

    count: int = 0
    mean: np.ndarray = field(default_factory=lambda: np.zeros(3))
    m2n: np.ndarray = field(default_factory=lambda: np.zeros(3))  # sum of squared deviations
    m2: np.ndarray = field(default_factory=lambda: np.zeros(3))  # sum of squares
    l1: np.ndarray = field(default_factory=lambda: np.zeros(3))  # sum of |x|

    @classmethod
    def from_arrays(cls, label: np.ndarray, prediction: np.ndarray) -> "RegressionSummary":
        y = np.asarray(label, dtype=np.float64)
        p = np.asarray(prediction, dtype=np.float64)
        M = np.stack([y, y - p, p])
        n = y.shape[0]
        if n == 0:
            return cls()
        mean = M.mean(1)
        return cls(n, mean, ((M - mean[:, None]) ** 2).sum(1), (M * M).sum(1), np.abs(M).sum(1))

    @classmethod
    def from_moments(cls, n: int, mom: np.ndarray) -> "RegressionSummary":
        """From the device reduction (``ops.reg_moments``): rows [sum, sum of squares, sum |x|,
        sum of squared deviations] of the columns (label, label - prediction, prediction)."""
        if n == 0:
            return cls()
        mom = np.asarray(mom, dtype=np.float64)
        return cls(int(n), mom[0] / n, mom[3].copy(), mom[1].copy(), mom[2].copy())

    def merge(self, o: "RegressionSummary") -> "RegressionSummary":
        if o.count == 0:
            return self
        if self.count == 0:
            return o
        tot = self.count + o.count
        delta = o.mean - self.mean
        mean = self.mean + delta * o.count / tot
        m2n = self.m2n + o.m2n + delta * delta * self.count * o.count / tot
        return RegressionSummary(tot, mean, m2n, self.m2 + o.m2, self.l1 + o.l1)


class RegressionMetrics:
    def __init__(self, summary: RegressionSummary) -> None:
        self.s = summary

    @property
    def _ss_err(self) -> float:
        return float(self.s.m2[1])

    @property
    def _ss_tot(self) -> float:
        return float(self.s.m2n[0])  # variance * (n-1) with unbiased variance = m2n

    @property
    def _ss_y(self) -> float:
        return float(self.s.m2[0])

    @property
    def _ss_reg(self) -> float:
        n = self.s.count
        return float(self.s.m2[2] + self.s.mean[0] ** 2 * n - 2 * self.s.mean[0] * self.s.mean[2] * n)

    @property
    def mean_squared_error(self) -> float:
        return self._ss_err / self.s.count

    @property
    def root_mean_squared_error(self) -> float:
        return math.sqrt(self.mean_squared_error)

    def r2(self, through_origin: bool = False) -> float:
        return 1 - self._ss_err / (self._ss_y if through_origin else self._ss_tot)

    @property
    def mean_absolute_error(self) -> float:
        return float(self.s.l1[1]) / self.s.count

    @property
    def explained_variance(self) -> float:
        return self._ss_reg / self.s.count

    def evaluate(self, evaluator: Any) -> float:
        name = evaluator.getMetricName()
        if name == "rmse":
            return self.root_mean_squared_error
        if name == "mse":
            return self.mean_squared_error
        if name == "r2":
            return self.r2(evaluator.getThroughOrigin())
        if name == "mae":
            return self.mean_absolute_error
        if name == "var":
            return self.explained_variance
        raise ValueError(f"Unsupported metric name, found {name}")


# --------------------------------------------------------------------------------------
# multiclass
# --------------------------------------------------------------------------------------
@dataclass
class ClassificationSummary:
    tp: Dict[float, float] = field(default_factory=dict)
    fp: Dict[float, float] = field(default_factory=dict)
    label: Dict[float, float] = field(default_factory=dict)
    count: int = 0
    log_loss_sum: float = 0.0

    @classmethod
    def from_arrays(cls, label: np.ndarray, prediction: np.ndarray, probability: Optional[np.ndarray] = None,
                    eps: float = 1e-15) -> "ClassificationSummary":
        y = np.asarray(label, dtype=np.float64)
        p = np.asarray(prediction, dtype=np.float64)
        s = cls(count=int(y.shape[0]))
        classes = np.union1d(np.unique(y), np.unique(p))
        for c in classes:
            yc = y == c
            pc = p == c
            s.tp[float(c)] = float(np.sum(yc & pc))
            s.fp[float(c)] = float(np.sum(~yc & pc))
            s.label[float(c)] = float(np.sum(yc))
        if probability is not None and len(y):
            prob = np.asarray(probability, dtype=np.float64)
            idx = y.astype(np.int64)
            pl = prob[np.arange(len(y)), np.clip(idx, 0, prob.shape[1] - 1)]
            s.log_loss_sum = float(-np.log(np.maximum(pl, eps)).sum())
        return s

    @classmethod
    def from_confusion(cls, cm: np.ndarray, count: int, log_loss_sum: float = 0.0) -> "ClassificationSummary":
        """From (label, prediction) counts (``ops.confusion_counts``): the classes present as a
        label or a prediction, like ``from_arrays``."""
        cm = np.asarray(cm, dtype=np.float64)
        rows, cols = cm.sum(1), cm.sum(0)
        s = cls(count=int(count), log_loss_sum=float(log_loss_sum))
        for c in np.nonzero((rows > 0) | (cols > 0))[0]:
            s.tp[float(c)] = float(cm[c, c])
            s.fp[float(c)] = float(cols[c] - cm[c, c])
            s.label[float(c)] = float(rows[c])
        return s

    def merge(self, o: "ClassificationSummary") -> "ClassificationSummary":
        out = ClassificationSummary(dict(self.tp), dict(self.fp), dict(self.label), self.count + o.count,
                                    self.log_loss_sum + o.log_loss_sum)
        for d_out, d_in in ((out.tp, o.tp), (out.fp, o.fp), (out.label, o.label)):
            for k, v in d_in.items():
                d_out[k] = d_out.get(k, 0.0) + v
        return out


class MulticlassMetrics:
    """Spark ``MulticlassMetrics`` formulas over merged per-class counts."""

    def __init__(self, s: ClassificationSummary) -> None:
        self.s = s

    def _labels(self) -> List[float]:
        return [k for k, v in self.s.label.items() if v > 0]

    def _precision(self, c: float) -> float:
        tp, fp = self.s.tp.get(c, 0.0), self.s.fp.get(c, 0.0)
        return 0.0 if tp + fp == 0 else tp / (tp + fp)

    def _recall(self, c: float) -> float:
        n = self.s.label.get(c, 0.0)
        return 0.0 if n == 0 else self.s.tp.get(c, 0.0) / n

    def _f_measure(self, c: float, beta: float = 1.0) -> float:
        p, r = self._precision(c), self._recall(c)
        b2 = beta * beta
        return 0.0 if p + r == 0 else (1 + b2) * p * r / (b2 * p + r)

    def false_positive_rate(self, c: float) -> float:
        neg = self.s.count - self.s.label.get(c, 0.0)
        return 0.0 if neg == 0 else self.s.fp.get(c, 0.0) / neg

    def _weighted(self, f: Any) -> float:
        return sum(f(c) * self.s.label[c] / self.s.count for c in self._labels())

    def accuracy(self) -> float:
        return sum(self.s.tp.values()) / self.s.count

    def weighted_fmeasure(self, beta: float = 1.0) -> float:
        return self._weighted(lambda c: self._f_measure(c, beta))

    def weighted_precision(self) -> float:
        return self._weighted(self._precision)

    def weighted_recall(self) -> float:
        return self._weighted(self._recall)

    def weighted_false_positive_rate(self) -> float:
        return self._weighted(self.false_positive_rate)

    def hamming_loss(self) -> float:
        return sum(self.s.fp.values()) / self.s.count

    def log_loss(self) -> float:
        return self.s.log_loss_sum / self.s.count

    def evaluate(self, evaluator: Any) -> float:
        name = evaluator.getMetricName()
        table = {
            "f1": lambda: self.weighted_fmeasure(),
            "accuracy": self.accuracy,
            "weightedPrecision": self.weighted_precision,
            "weightedRecall": self.weighted_recall,
            "weightedTruePositiveRate": self.weighted_recall,
            "weightedFalsePositiveRate": self.weighted_false_positive_rate,
            "weightedFMeasure": lambda: self.weighted_fmeasure(evaluator.getBeta()),
            "truePositiveRateByLabel": lambda: self._recall(evaluator.getMetricLabel()),
            "falsePositiveRateByLabel": lambda: self.false_positive_rate(evaluator.getMetricLabel()),
            "precisionByLabel": lambda: self._precision(evaluator.getMetricLabel()),
            "recallByLabel": lambda: self._recall(evaluator.getMetricLabel()),
            "fMeasureByLabel": lambda: self._f_measure(evaluator.getMetricLabel(), evaluator.getBeta()),
            "hammingLoss": self.hamming_loss,
            "logLoss": self.log_loss,
        }
        if name not in table:
            raise ValueError(f"Unsupported metric name, found {name}")
        return float(table[name]())

    SUPPORTED_MULTI_CLASS_METRIC_NAMES = [
        "f1", "accuracy", "weightedPrecision", "weightedRecall", "weightedTruePositiveRate",
        "weightedFalsePositiveRate", "weightedFMeasure", "truePositiveRateByLabel", "falsePositiveRateByLabel",
        "precisionByLabel", "recallByLabel", "fMeasureByLabel", "hammingLoss", "logLoss",
    ]


def binary_auc(label: np.ndarray, score: np.ndarray) -> float:
    """Area under ROC (trapezoid over distinct thresholds, ties handled like Spark)."""
    y = np.asarray(label, dtype=np.float64)
    s = np.asarray(score, dtype=np.float64)
    order = np.argsort(-s, kind="mergesort")
    s, y = s[order], y[order]
    distinct = np.r_[np.nonzero(np.diff(s))[0], len(s) - 1]
    tps = np.cumsum(y)[distinct]
    fps = np.cumsum(1 - y)[distinct]
    P, N = tps[-1] if len(tps) else 0.0, fps[-1] if len(fps) else 0.0
    if P == 0 or N == 0:
        return 0.0
    tpr = np.r_[0.0, tps / P, 1.0]
    fpr = np.r_[0.0, fps / N, 1.0]
    return float(np.trapezoid(tpr, fpr)) if hasattr(np, "trapezoid") else float(np.trapz(tpr, fpr))


def binary_aupr(label: np.ndarray, score: np.ndarray) -> float:
    y = np.asarray(label, dtype=np.float64)
    s = np.asarray(score, dtype=np.float64)
    order = np.argsort(-s, kind="mergesort")
    s, y = s[order], y[order]
    distinct = np.r_[np.nonzero(np.diff(s))[0], len(s) - 1]
    tps = np.cumsum(y)[distinct]
    fps = np.cumsum(1 - y)[distinct]
    P = tps[-1] if len(tps) else 0.0
    if P == 0:
        return 0.0
    recall = np.r_[0.0, tps / P]
    precision = np.r_[1.0, tps / np.maximum(tps + fps, 1)]
    return float(np.sum(np.diff(recall) * (precision[1:] + precision[:-1]) / 2))
