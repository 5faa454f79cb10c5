"""``Model.cpu()`` conversions to pyspark.ml models (needs pyspark + a JVM)."""
from __future__ import annotations

from typing import Any


def _require_spark() -> Any:
    try:
        from pyspark.sql import SparkSession  # type: ignore
    except Exception as e:  # noqa: BLE001
        raise ImportError("cpu() requires pyspark, which is not installed") from e
    spark = SparkSession.getActiveSession()
    if spark is None:
        raise RuntimeError("cpu() requires an active SparkSession")
    return spark


def _py2java(sc: Any, obj: Any) -> Any:
    from pyspark.ml.common import _py2java as p2j  # type: ignore

    return p2j(sc, obj)


def java_uid(sc: Any, prefix: str) -> str:
    return sc._jvm.org.apache.spark.ml.util.Identifiable.randomUID(prefix)


def to_spark_pca_model(model: Any) -> Any:
    spark = _require_spark()
    from pyspark.ml.feature import PCAModel as SparkPCAModel  # type: ignore
    from pyspark.ml.linalg import DenseMatrix, DenseVector  # type: ignore

    sc = spark.sparkContext
    pc = DenseMatrix(model.pc.numRows, model.pc.numCols, list(model.pc.values), False)
    ev = DenseVector(model.explained_variance_ratio_)
    jm = sc._jvm.org.apache.spark.ml.feature.PCAModel(java_uid(sc, "pca"), _py2java(sc, pc), _py2java(sc, ev))
    m = SparkPCAModel(jm)
    for p in ("inputCol", "outputCol"):
        if model.isDefined(p) and m.hasParam(p):
            m._set(**{p: model.getOrDefault(p)})
    return m
