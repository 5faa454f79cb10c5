"""Driver script for tests/test_spark_fake.py: runs with the fake pyspark of tests/fakespark on
sys.path (its own process, so the rest of the suite keeps the built-in Param classes)."""
import json
import sys

import numpy as np

import pyspark.ml
from pyspark.sql import SparkSession

from spark_rapids_ml_nai_amd import DataFrame as SRDF
from spark_rapids_ml_nai_amd.core import params



def main() -> None:
    out = {"pyspark_params": params.PYSPARK_PARAMS}
    spark = SparkSession(conf={"spark.sql.execution.arrow.maxRecordsPerBatch": "128"})
    rng = np.random.default_rng(0)
    m, n = 1500, 8
    X = rng.standard_normal((m, n)).astype(np.float32)
    w = np.arange(1, n + 1, dtype=np.float64)
    y = X.astype(np.float64) @ w + 0.25 + 0.01 * rng.standard_normal(m)
    yc = (X[:, 0] + 0.5 * X[:, 1] > 0).astype(np.float64)


    def sdf(X, y, vector=False, parts=2):
        t = SRDF.from_numpy(X, y, vector=vector).partitions[0]
        return spark.createDataFrame(t, num_partitions=parts)


    from spark_rapids_ml_nai_amd.classification import LogisticRegression, RandomForestClassifier  # noqa: E402
    from spark_rapids_ml_nai_amd.clustering import KMeans  # noqa: E402
    from spark_rapids_ml_nai_amd.feature import PCA  # noqa: E402
    from spark_rapids_ml_nai_amd.regression import LinearRegression  # noqa: E402

    est = LinearRegression(num_workers=2, regParam=0.0)
    out["is_pyspark_estimator"] = isinstance(est, pyspark.ml.Estimator)
    model = est.fit(sdf(X, y))
    out["is_pyspark_model"] = isinstance(model, pyspark.ml.Model)
    local = LinearRegression(num_workers=1, regParam=0.0).fit(SRDF.from_numpy(X, y))
    out["linreg_coef_maxdiff"] = float(np.abs(np.asarray(model.coef_) - np.asarray(local.coef_)).max())
    pred = model.transform(sdf(X, y)).toArrow().column("prediction").to_numpy()
    out["linreg_pred_maxdiff"] = float(np.abs(pred - local.transform(SRDF.from_numpy(X, y)).to_numpy("prediction")).max())

    # vector (VectorUDT struct) input through unwrap_udt
    mv = LinearRegression(num_workers=2, regParam=0.0).fit(sdf(X, y, vector=True))
    out["linreg_vector_coef_maxdiff"] = float(np.abs(np.asarray(mv.coef_) - np.asarray(local.coef_)).max())

    lr = LogisticRegression(num_workers=2, regParam=0.01).fit(sdf(X, yc))
    lr_local = LogisticRegression(num_workers=1, regParam=0.01).fit(SRDF.from_numpy(X, yc))
    out["logreg_coef_maxdiff"] = float(np.abs(np.asarray(lr.coef_) - np.asarray(lr_local.coef_)).max())
    tr = lr.transform(sdf(X, yc)).toArrow()
    out["logreg_columns"] = tr.schema.names
    out["logreg_acc"] = float((tr.column("prediction").to_numpy() == yc).mean())
    prob0 = tr.column("probability").to_pylist()[0]  # VectorUDT struct (type, size, indices, values)
    out["logreg_prob_rows"] = len(prob0["values"]) if isinstance(prob0, dict) else len(prob0)

    km = KMeans(k=3, seed=1, num_workers=2, maxIter=20).fit(sdf(X, None))
    out["kmeans_centers"] = len(km.clusterCenters())
    pca = PCA(k=2, num_workers=2, inputCol="features", outputCol="pca").fit(sdf(X, None))
    pca_local = PCA(k=2, num_workers=1, inputCol="features").fit(SRDF.from_numpy(X))
    comp_diff = np.abs(np.asarray(pca.components_)) - np.abs(np.asarray(pca_local.components_))
    out["pca_comp_maxdiff"] = float(np.abs(comp_diff).max())
    rf = RandomForestClassifier(numTrees=4, maxDepth=5, seed=3, num_workers=2).fit(sdf(X, yc))
    out["rf_trees"] = rf.getNumTrees

    # a pyspark Pipeline (isinstance-dispatched stages) across our estimators
    pipe = pyspark.ml.Pipeline([PCA(k=3, num_workers=2, inputCol="features", outputCol="pcs"),
                                LinearRegression(num_workers=2, featuresCol="pcs", labelCol="label")])
    pm = pipe.fit(sdf(X, y))
    res = pm.transform(sdf(X, y)).toArrow()
    out["pipeline_columns"] = res.schema.names
    print("RESULT " + json.dumps(out))
    sys.stdout.flush()


if __name__ == "__main__":  # spawned barrier tasks re-import this module
    main()
