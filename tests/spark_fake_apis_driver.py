"""Driver for tests/test_spark_fake_apis.py (fake pyspark of tests/fakespark on sys.path, own
process): the Spark-DataFrame paths of NearestNeighbors / ApproximateNearestNeighbors / DBSCAN /
UMAP / CrossValidator and the VectorUDT output typing, each compared with the in-process result."""
import json
import sys

import numpy as np

from pyspark.ml.linalg import VectorUDT
from pyspark.sql import SparkSession

from spark_rapids_ml_nai_amd import DataFrame as SRDF


def main() -> None:
    out = {}
    spark = SparkSession(conf={"spark.sql.execution.arrow.maxRecordsPerBatch": "64"})
    rng = np.random.default_rng(1)

    def sdf(X, y=None, vector=False, parts=2):
        t = SRDF.from_numpy(X, y, vector=vector).partitions[0]
        return spark.createDataFrame(t, num_partitions=parts)

    # ---- exact kNN: barrier job over items u queries, ids from monotonically_increasing_id
    from spark_rapids_ml_nai_amd.knn import ApproximateNearestNeighbors, NearestNeighbors

    items = rng.standard_normal((300, 6)).astype(np.float32)
    queries = rng.standard_normal((50, 6)).astype(np.float32)
    model = NearestNeighbors(k=4, inputCol="features", num_workers=2).fit(sdf(items, parts=3))
    item_df, query_df, knn_df = model.kneighbors(sdf(queries, parts=2))
    knn = knn_df.toArrow()
    qid = knn.column("query_unique_id").to_numpy()
    ind = np.array(knn.column("indices").to_pylist())
    dist = np.array(knn.column("distances").to_pylist())
    item_ids = item_df.toArrow().column("unique_id").to_numpy()
    query_ids = query_df.toArrow().column("unique_id").to_numpy()
    # oracle: brute force in numpy on the same id assignment
    pos_q = {int(v): i for i, v in enumerate(query_ids)}
    d2 = ((queries[:, None, :] - items[None, :, :]) ** 2).sum(-1)
    ref = np.argsort(d2, axis=1)[:, :4]
    ok = 0
    for r in range(len(qid)):
        qi = pos_q[int(qid[r])]
        ok += set(item_ids[ref[qi]].tolist()) == set(ind[r].tolist())
    out["knn_rows"] = int(len(qid))
    out["knn_sorted"] = bool(np.all(np.diff(qid) >= 0))
    out["knn_exact_frac"] = ok / max(1, len(qid))
    out["knn_dist_err"] = float(np.abs(np.sort(dist, 1) - np.sqrt(np.sort(d2, 1)[[pos_q[int(q)] for q in qid], :4])).max())
    join = model.exactNearestNeighborsJoin(sdf(queries, parts=2), distCol="d").toArrow()
    out["join_columns"] = join.schema.names
    out["join_rows"] = join.num_rows

    # ---- IVF-Flat ANN on Spark: same barrier job, recall vs exact
    ann = ApproximateNearestNeighbors(k=4, inputCol="features", num_workers=2,
                                      algoParams={"nlist": 8, "nprobe": 8}).fit(sdf(items, parts=3))
    _, _, aknn = ann.kneighbors(sdf(queries, parts=2))
    at = aknn.toArrow()
    aq = at.column("query_unique_id").to_numpy()
    aind = np.array(at.column("indices").to_pylist())
    out["ann_rows"] = int(len(aq))
    out["ann_recall_vs_exact"] = float(np.mean([len(set(a) & set(b)) / 4.0 for a, b in zip(aind, ind)]))
    out["ann_join_rows"] = ann.approxSimilarityJoin(sdf(queries, parts=2)).toArrow().num_rows

    # ---- DBSCAN on Spark: barrier job + join back on the id
    from spark_rapids_ml_nai_amd.clustering import DBSCAN

    C = np.array([[0, 0], [10, 10], [-10, 10]], np.float32)
    Xd = (C[rng.integers(0, 3, 400)] + 0.3 * rng.standard_normal((400, 2))).astype(np.float32)
    dm = DBSCAN(eps=1.0, min_samples=5, num_workers=2).fit(sdf(Xd, parts=2))
    dt = dm.transform(sdf(Xd, parts=2)).toArrow()
    local = DBSCAN(eps=1.0, min_samples=5, num_workers=1).fit(SRDF.from_numpy(Xd)).transform(SRDF.from_numpy(Xd))
    out["dbscan_columns"] = dt.schema.names
    out["dbscan_rows"] = dt.num_rows
    out["dbscan_nclusters"] = int(len(set(dt.column("prediction").to_pylist()) - {-1}))
    out["dbscan_nclusters_local"] = int(len(set(local.to_numpy("prediction").tolist()) - {-1}))

    # ---- UMAP on Spark: barrier fit (2 ranks), per-partition transform
    from spark_rapids_ml_nai_amd.umap import UMAP

    Xu = (C[rng.integers(0, 3, 300)].repeat(3, 1)[:, :6] + 0.5 * rng.standard_normal((300, 6))).astype(np.float32)
    um = UMAP(n_neighbors=10, n_epochs=60, random_state=0, num_workers=2, featuresCol="features").fit(sdf(Xu, parts=2))
    ut = um.transform(sdf(Xu, parts=2)).toArrow()
    out["umap_embedding_shape"] = list(np.asarray(um.embedding_).shape)
    out["umap_transform_columns"] = ut.schema.names
    out["umap_transform_rows"] = ut.num_rows
    # chunked path (reference tests/test_umap.py:333-377): the fit streams maxRecordsPerBatch (64)
    # row batches back, a tiny BROADCAST_LIMIT splits embedding / raw rows into several broadcasts,
    # the task closure stays small, and fit + transform equal the in-process ones
    est = UMAP(n_neighbors=10, n_epochs=60, random_state=0, num_workers=1, featuresCol="features")
    est.BROADCAST_LIMIT = 2000  # bytes: 300 x 6 fp32 raw rows -> 4 chunks, 300 x 2 embedding -> 2
    uc = est.fit(sdf(Xu, parts=1))
    local_m = UMAP(n_neighbors=10, n_epochs=60, random_state=0, featuresCol="features").fit(SRDF.from_numpy(Xu))
    out["umap_fit_batches"] = est._fit_result_batches
    out["umap_chunked_fit_equal"] = bool(np.array_equal(uc.raw_data_, Xu)) and bool(
        np.allclose(uc.embedding_, local_m.embedding_, atol=1e-5))
    n_bc0 = len(spark.sparkContext.broadcasts)
    tc = uc.transform(sdf(Xu, parts=2)).toArrow()
    out["umap_broadcasts"] = [len(uc._broadcasts[1]), len(uc._broadcasts[2])]
    out["umap_new_broadcasts"] = len(spark.sparkContext.broadcasts) - n_bc0
    out["umap_closure_bytes"] = int(uc._spark_closure_bytes)
    out["umap_raw_bytes"] = int(Xu.nbytes)
    emb_t = np.asarray(tc.column("embedding").to_pylist(), np.float32)
    uc.transform(sdf(Xu, parts=2)).toArrow()  # a second transform reuses the broadcasts
    out["umap_new_broadcasts_2nd"] = len(spark.sparkContext.broadcasts) - n_bc0
    uc.BROADCAST_LIMIT = 8 << 30  # one broadcast per array: the same transform, unchunked
    emb_1 = np.asarray(uc.transform(sdf(Xu, parts=2)).toArrow().column("embedding").to_pylist(), np.float32)
    out["umap_chunked_transform_maxdiff"] = float(np.abs(emb_t - emb_1).max())

    # ---- VectorUDT outputs: probability / rawPrediction always, PCA output mirrors a vector input
    from spark_rapids_ml_nai_amd.classification import LogisticRegression
    from spark_rapids_ml_nai_amd.feature import PCA

    Xc = rng.standard_normal((400, 5)).astype(np.float32)
    yc = (Xc[:, 0] + Xc[:, 1] > 0).astype(np.float64)
    lr = LogisticRegression(num_workers=2, regParam=0.01).fit(sdf(Xc, yc))
    tr = lr.transform(sdf(Xc, yc))
    out["lr_types"] = {f.name: type(f.dataType).__name__ for f in tr.schema.fields}
    trv = lr.transform(sdf(Xc, yc, vector=True))  # VectorUDT input: pandas-UDF path keeps every column
    out["lr_vec_types"] = {f.name: type(f.dataType).__name__ for f in trv.schema.fields}
    out["lr_vec_pred_match"] = bool(np.array_equal(trv.toArrow().column("prediction").to_numpy(),
                                                   tr.toArrow().column("prediction").to_numpy()))
    pca = PCA(k=2, num_workers=2, inputCol="features", outputCol="pcs").fit(sdf(Xc, vector=True))
    out["pca_vec_out"] = type(pca.transform(sdf(Xc, vector=True)).schema["pcs"].dataType).__name__
    out["pca_arr_out"] = type(pca.transform(sdf(Xc)).schema["pcs"].dataType).__name__
    out["vector_udt"] = VectorUDT.__name__

    # ---- CrossValidator: a pyspark CrossValidator; single-pass fast path on Spark folds vs the
    # generic pyspark loop on the same folds
    import pyspark.ml.tuning as pt

    from spark_rapids_ml_nai_amd.evaluation import MulticlassClassificationEvaluator, RegressionEvaluator
    from spark_rapids_ml_nai_amd.regression import LinearRegression
    from spark_rapids_ml_nai_amd.tuning import CrossValidator, CrossValidatorModel, ParamGridBuilder

    Xr = rng.standard_normal((600, 4)).astype(np.float32)
    yr = Xr @ np.array([1.0, -2.0, 0.5, 3.0]) + 0.1 * rng.standard_normal(600)
    lin = LinearRegression(num_workers=2)
    grid = ParamGridBuilder().addGrid(lin.regParam, [0.0, 0.5]).build()
    cv = CrossValidator(estimator=lin, estimatorParamMaps=grid, evaluator=RegressionEvaluator(), numFolds=2, seed=5)
    out["cv_is_pyspark"] = isinstance(cv, pt.CrossValidator)
    data = sdf(Xr, yr)
    cvm = cv.fit(data)
    out["cv_model_is_pyspark"] = isinstance(cvm, pt.CrossValidatorModel) and isinstance(cvm, CrossValidatorModel)
    out["cv_avg"] = [float(v) for v in cvm.avgMetrics]
    out["cv_generic_avg"] = [float(v) for v in pt.CrossValidator._fit(cv, data).avgMetrics]
    lrc = LogisticRegression(num_workers=2)
    gridc = ParamGridBuilder().addGrid(lrc.regParam, [0.01, 0.3]).build()
    for metric in ("f1", "logLoss"):
        ev = MulticlassClassificationEvaluator(metricName=metric)
        cvc = CrossValidator(estimator=lrc, estimatorParamMaps=gridc, evaluator=ev, numFolds=2, seed=3)
        dc = sdf(Xc, yc)
        out["cvc_%s" % metric] = [float(v) for v in cvc.fit(dc).avgMetrics]
        out["cvc_%s_generic" % metric] = [float(v) for v in pt.CrossValidator._fit(cvc, dc).avgMetrics]
    print("RESULT " + json.dumps(out))
    sys.stdout.flush()


if __name__ == "__main__":  # spawned barrier tasks re-import this module
    main()
