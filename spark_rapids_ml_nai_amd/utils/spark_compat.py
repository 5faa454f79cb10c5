"""``Model.cpu()`` conversions to pyspark.ml models (needs pyspark + a JVM)."""
from __future__ import annotations

from typing import Any, Dict, List

import numpy as np


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


def _apply_common(src: Any, dst: Any) -> Any:
    for p in src.params:
        if src.isDefined(p) and dst.hasParam(p.name):
            try:
                dst._set(**{p.name: src.getOrDefault(p)})
            except Exception:  # noqa: BLE001 - params Spark does not type the same way are skipped
                pass
    return dst


def to_spark_linear_regression_model(model: Any) -> Any:
    """``LinearRegressionModel(uid, coefficients, intercept, scale)`` (reference ``regression.py:658-672``)."""
    spark = _require_spark()
    from pyspark.ml.linalg import DenseVector  # type: ignore
    from pyspark.ml.regression import LinearRegressionModel as SparkLRModel  # type: ignore

    sc = spark.sparkContext
    coef = DenseVector(model.coefficients.toArray())
    jm = sc._jvm.org.apache.spark.ml.regression.LinearRegressionModel(java_uid(sc, "linReg"), _py2java(sc, coef),
                                                                      float(model.intercept), float(model.scale))
    return _apply_common(model, SparkLRModel(jm))


def to_spark_kmeans_model(model: Any) -> Any:
    """mllib ``KMeansModel(centers)`` wrapped in ml ``KMeansModel`` (reference ``clustering.py:422-442``)."""
    spark = _require_spark()
    from pyspark.ml.clustering import KMeansModel as SparkKMeansModel  # type: ignore
    from pyspark.mllib.common import _py2java as mllib_py2java  # type: ignore
    from pyspark.mllib.linalg import _convert_to_vector  # type: ignore

    sc = spark.sparkContext
    centers = mllib_py2java(sc, [_convert_to_vector(list(map(float, c))) for c in model.cluster_centers_])
    jmllib = sc._jvm.org.apache.spark.mllib.clustering.KMeansModel(centers)
    jm = sc._jvm.org.apache.spark.ml.clustering.KMeansModel(java_uid(sc, "kmeans"), jmllib)
    return _apply_common(model, SparkKMeansModel(jm))


def to_spark_logistic_regression_model(model: Any) -> Any:
    """``LogisticRegressionModel(uid, coefficientMatrix, interceptVector, numClasses, isMultinomial)``."""
    spark = _require_spark()
    from pyspark.ml.classification import LogisticRegressionModel as SparkLogRegModel  # type: ignore
    from pyspark.ml.linalg import DenseMatrix, DenseVector  # type: ignore

    sc = spark.sparkContext
    cm = model.coefficientMatrix
    jcm = DenseMatrix(cm.numRows, cm.numCols, list(cm.toArray().ravel(order="F")), False)
    jiv = DenseVector(model.interceptVector.toArray())
    k = int(model.numClasses)
    jm = sc._jvm.org.apache.spark.ml.classification.LogisticRegressionModel(
        java_uid(sc, "logreg"), _py2java(sc, jcm), _py2java(sc, jiv), k, k > 2)
    return _apply_common(model, SparkLogRegModel(jm))


def _impurity_calc(sc: Any, impurity: str, stats: Any, count: int) -> Any:
    jvm = sc._jvm
    arr = sc._gateway.new_array(jvm.double, len(stats))
    for i, v in enumerate(stats):
        arr[i] = float(v)
    cls = {"gini": jvm.org.apache.spark.mllib.tree.impurity.GiniCalculator,
           "entropy": jvm.org.apache.spark.mllib.tree.impurity.EntropyCalculator,
           "variance": jvm.org.apache.spark.mllib.tree.impurity.VarianceCalculator}[impurity]
    return cls(arr, int(count))


def _java_tree(sc: Any, impurity: str, t: Any, classification: bool) -> Any:
    """Portable tree dict (feature/threshold/left/right/value/gain/count) -> Spark ``Node``, built
    bottom-up without recursion (deep trees would overflow Python's stack)."""
    jvm = sc._jvm
    n = len(t["feature"])
    order: List[int] = []
    stack = [0]
    while stack:
        i = stack.pop()
        order.append(i)
        if t["feature"][i] >= 0:
            stack.extend([t["left"][i], t["right"][i]])
    built: Dict[int, Any] = {}
    for i in reversed(order):
        v = list(t["value"][i])
        cnt = int(t["count"][i]) if "count" in t else 0
        if t["feature"][i] < 0:
            if classification:
                pred = float(int(np.argmax(v)))
                calc = _impurity_calc(sc, impurity, v, cnt)
            else:
                pred = float(v[0])
                calc = _impurity_calc(sc, "variance", [float(cnt), pred * cnt, 0.0], cnt)
            built[i] = jvm.org.apache.spark.ml.tree.LeafNode(pred, 0.0, calc)
        else:
            split = jvm.org.apache.spark.ml.tree.ContinuousSplit(int(t["feature"][i]), float(t["threshold"][i]))
            stats = v if classification else [float(cnt), 0.0, 0.0]
            calc = _impurity_calc(sc, impurity if classification else "variance", stats, cnt)
            built[i] = jvm.org.apache.spark.ml.tree.InternalNode(
                0.0, 0.0, float(t["gain"][i]) if "gain" in t else 0.0, built[t["left"][i]], built[t["right"][i]],
                split, calc)
    assert len(built) <= n
    return built[0]


def to_spark_random_forest_model(model: Any) -> Any:
    """Spark ``RandomForest{Classification,Regression}Model`` from the portable trees
    (reference ``tree.py:524-569`` + ``utils.py:330-482``)."""
    spark = _require_spark()
    sc = spark.sparkContext
    jvm = sc._jvm
    classification = bool(model._is_classification)
    impurity = model.getImpurity() if classification else "variance"
    nf = int(model.n_cols)
    if classification:
        from pyspark.ml.classification import RandomForestClassificationModel as SparkRFC  # type: ignore

        uid = java_uid(sc, "rfc")
        tcls = jvm.org.apache.spark.ml.classification.DecisionTreeClassificationModel
        k = int(model.numClasses)
        trees = [tcls(uid, _java_tree(sc, impurity, t, True), nf, k) for t in model._trees]
    else:
        from pyspark.ml.regression import RandomForestRegressionModel as SparkRFR  # type: ignore

        uid = java_uid(sc, "rfr")
        tcls = jvm.org.apache.spark.ml.regression.DecisionTreeRegressionModel
        trees = [tcls(uid, _java_tree(sc, impurity, t, False), nf) for t in model._trees]
    jarr = sc._gateway.new_array(tcls, len(trees))
    for i, tr in enumerate(trees):
        jarr[i] = tr
    if classification:
        jm = jvm.org.apache.spark.ml.classification.RandomForestClassificationModel(uid, jarr, nf, k)
        return _apply_common(model, SparkRFC(jm))
    jm = jvm.org.apache.spark.ml.regression.RandomForestRegressionModel(uid, jarr, nf)
    return _apply_common(model, SparkRFR(jm))
