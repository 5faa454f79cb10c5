"""Driver of tests/test_spmd_matrix.py: every public entry point on the SAME global data, either
as ONE process (``--single``: the whole dataset, one rank) or as one rank of a torchrun (SPMD)
world, where each rank holds only its own, deliberately uneven, row shard of every frame.

Every rank writes what it sees (its model attributes, the rows its transforms / searches return)
to ``<out>/rank<r>.npz``; the test compares the SPMD ranks, concatenated in rank order, with the
single-process run. CPU ranks on gloo: the collectives are the ones RCCL runs on MI355X ranks.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

N, D, NQ = 1200, 8, 300


def shard_bounds(total: int, world: int) -> np.ndarray:
    """Uneven shards (rank r gets a share proportional to r + 2) so offset bugs cannot hide."""
    w = np.arange(2, world + 2, dtype=np.float64)
    return np.concatenate([[0], np.round(np.cumsum(w) / w.sum() * total)]).astype(np.int64)


def global_data() -> dict:
    rng = np.random.default_rng(2024)
    C = rng.uniform(-12, 12, (5, D))
    lab = rng.integers(0, 5, N)
    Xb = (C[lab] + 0.7 * rng.standard_normal((N, D))).astype(np.float32)
    Q = (C[rng.integers(0, 5, NQ)] + 0.9 * rng.standard_normal((NQ, D))).astype(np.float32)
    Xr = rng.standard_normal((N, D)).astype(np.float32)
    yr = (Xr @ rng.uniform(-3, 3, D) + 0.5 + 0.1 * rng.standard_normal(N)).astype(np.float64)
    yc = (Xr[:, 0] - 2 * Xr[:, 1] + 0.5 * rng.standard_normal(N) > 0).astype(np.float64)
    ym = np.argmax(Xr[:, :3] + 0.3 * rng.standard_normal((N, 3)), 1).astype(np.float64)
    # sparse copy of Xr: ~70 % of the entries zeroed, so LogisticRegression takes the CSR path
    Xs = np.where(rng.random((N, D)) < 0.7, 0.0, Xr).astype(np.float32)
    return dict(Xb=Xb, Q=Q, Xr=Xr, yr=yr, yc=yc, ym=ym, lab=lab.astype(np.float64), Xs=Xs)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--single", action="store_true")
    args = ap.parse_args()
    os.environ["SRML_FORCE_CPU"] = "1"
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    if args.single:
        rank, world = 0, 1
    else:
        dist.init_process_group("gloo", init_method="env://")
        rank, world = dist.get_rank(), dist.get_world_size()
    g = global_data()
    qb = shard_bounds(NQ, world)
    rb = shard_bounds(N, world)
    lo, hi = int(rb[rank]), int(rb[rank + 1])
    qlo, qhi = int(qb[rank]), int(qb[rank + 1])

    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.classification import LogisticRegression, RandomForestClassifier
    from spark_rapids_ml_nai_amd.clustering import DBSCAN, KMeans
    from spark_rapids_ml_nai_amd.feature import PCA
    from spark_rapids_ml_nai_amd.knn import ApproximateNearestNeighbors, NearestNeighbors
    from spark_rapids_ml_nai_amd.regression import LinearRegression, RandomForestRegressor
    from spark_rapids_ml_nai_amd.umap import UMAP

    nw = dict(num_workers=1) if args.single else {}
    out = {"rows": np.array([lo, hi]), "qrows": np.array([qlo, qhi])}

    def frame(X, y=None):
        return DataFrame.from_numpy(X[lo:hi], None if y is None else y[lo:hi], num_partitions=2)

    # ---- PCA
    pm = PCA(k=3, inputCol="features", outputCol="pca", **nw).fit(frame(g["Xr"]))
    out["pca_components"] = np.asarray(pm.components_)
    out["pca_evr"] = np.asarray(pm.explained_variance_ratio_)
    out["pca_transform"] = pm.transform(frame(g["Xr"])).to_numpy("pca")
    # ---- KMeans (well-separated blobs, k = true centre count)
    km = KMeans(k=5, seed=3, maxIter=30, **nw).setFeaturesCol("features").fit(frame(g["Xb"]))
    out["kmeans_centers"] = np.asarray(km.cluster_centers_)
    out["kmeans_pred"] = km.transform(frame(g["Xb"])).to_numpy("prediction")
    # ---- linear family
    for name, kw in (("ols", {}), ("ridge", dict(regParam=0.1)), ("enet", dict(regParam=0.05, elasticNetParam=0.5))):
        lm = LinearRegression(**kw, **nw).fit(frame(g["Xr"], g["yr"]))
        out[name + "_coef"] = np.asarray(lm.coef_, np.float64).ravel()
        out[name + "_intercept"] = np.asarray(lm.intercept_, np.float64).ravel()
        out[name + "_pred"] = lm.transform(frame(g["Xr"], g["yr"])).to_numpy("prediction")
    # ---- logistic (binary + multinomial)
    for name, y in (("logreg", g["yc"]), ("logreg_multi", g["ym"])):
        lg = LogisticRegression(regParam=0.01, maxIter=50, **nw).fit(frame(g["Xr"], y))
        out[name + "_objective"] = np.array([lg.objective])
        out[name + "_coef"] = np.asarray(lg.coef_, np.float64)
        t = lg.transform(frame(g["Xr"], y))
        out[name + "_pred"] = t.to_numpy("prediction")
        out[name + "_prob"] = t.to_numpy("probability")
    # ---- random forests (trees split over ranks, reference semantics)
    rfc = RandomForestClassifier(numTrees=12, maxDepth=6, seed=1, **nw).fit(frame(g["Xr"], g["yc"]))
    out["rfc_pred"] = rfc.transform(frame(g["Xr"], g["yc"])).to_numpy("prediction")
    out["rfc_trees"] = np.array([rfc.getNumTrees])
    rfr = RandomForestRegressor(numTrees=12, maxDepth=6, seed=1, **nw).fit(frame(g["Xr"], g["yr"]))
    out["rfr_pred"] = rfr.transform(frame(g["Xr"], g["yr"])).to_numpy("prediction")
    # ---- exact kNN: items = this rank's blob rows, queries = this rank's query rows
    items = DataFrame.from_numpy(g["Xb"][lo:hi], num_partitions=2)
    queries = DataFrame.from_numpy(g["Q"][qlo:qhi], num_partitions=2)
    nn = NearestNeighbors(k=6, inputCol="features", **nw).fit(items)
    item_df, query_df, knn_df = nn.kneighbors(queries)
    out["knn_item_ids"] = item_df.to_numpy("unique_id")
    out["knn_query_ids"] = query_df.to_numpy("unique_id")
    out["knn_qid"] = knn_df.to_numpy("query_unique_id")
    out["knn_ind"] = np.stack([np.asarray(v) for v in knn_df.toPandas()["indices"]])
    out["knn_dist"] = np.stack([np.asarray(v) for v in knn_df.toPandas()["distances"]])
    join = nn.exactNearestNeighborsJoin(queries, distCol="d")
    out["join_rows"] = np.array([join.count()])
    # ---- IVF-Flat ANN with nprobe = nlist (exhaustive: exact results) and its join
    ann = ApproximateNearestNeighbors(k=6, algoParams={"nlist": 4, "nprobe": 4}, inputCol="features", **nw).fit(items)
    _, _, aknn = ann.kneighbors(queries)
    out["ann_qid"] = aknn.to_numpy("query_unique_id")
    out["ann_ind"] = np.stack([np.asarray(v) for v in aknn.toPandas()["indices"]])
    out["ann_join_rows"] = np.array([ann.approxSimilarityJoin(queries).count()])
    # ---- DBSCAN: labels of this rank's rows
    db = DBSCAN(eps=1.6, min_samples=6, **nw).fit(frame(g["Xb"]))
    out["dbscan_labels"] = db.transform(frame(g["Xb"])).to_numpy("prediction")
    # ---- UMAP fit + transform of this rank's rows
    um = UMAP(n_neighbors=10, n_epochs=80, random_state=0, **nw).setFeaturesCol("features").fit(frame(g["Xb"]))
    out["umap_transform"] = um.transform(frame(g["Xb"])).to_numpy("embedding")
    out["umap_embedding_rows"] = np.array([np.asarray(um.embedding_).shape[0]])
    # ---- CrossValidator fast path (LinearRegression, 2 param maps)
    from spark_rapids_ml_nai_amd.evaluation import RegressionEvaluator
    from spark_rapids_ml_nai_amd.tuning import CrossValidator, ParamGridBuilder

    lin = LinearRegression(**nw)
    grid = ParamGridBuilder().addGrid(lin.regParam, [0.0, 5.0]).build()
    cvm = CrossValidator(estimator=lin, estimatorParamMaps=grid, evaluator=RegressionEvaluator(), numFolds=2,
                         seed=5).fit(frame(g["Xr"], g["yr"]))
    out["cv_avg"] = np.asarray(cvm.avgMetrics, np.float64)
    out["cv_best_coef"] = np.asarray(cvm.bestModel.coef_, np.float64).ravel()

    # ---- sparse (CSR) LogisticRegression on VectorUDT rows
    import scipy.sparse as sps

    sdf = DataFrame.from_numpy(sps.csr_matrix(g["Xs"][lo:hi]), g["yc"][lo:hi], num_partitions=2)
    ls = LogisticRegression(regParam=0.01, maxIter=50, **nw).fit(sdf)
    out["logreg_sparse_objective"] = np.array([ls.objective])
    out["logreg_sparse_coef"] = np.asarray(ls.coef_, np.float64)
    out["logreg_sparse_pred"] = ls.transform(sdf).to_numpy("prediction")
    # ---- data-parallel random forest: every rank grows the SAME trees from globally reduced
    # histograms, so every rank's model predicts the whole dataset identically
    rdp = RandomForestClassifier(numTrees=6, maxDepth=6, seed=1, split_mode="data_parallel", **nw).fit(
        frame(g["Xr"], g["yc"]))
    out["rfdp_pred_all"] = rdp.transform(DataFrame.from_numpy(g["Xr"])).to_numpy("prediction")
    # ---- supervised UMAP (categorical target intersection)
    us = UMAP(n_neighbors=10, n_epochs=80, random_state=0, labelCol="label", **nw).setFeaturesCol("features").fit(
        frame(g["Xb"], g["lab"]))
    out["umap_sup_transform"] = us.transform(frame(g["Xb"])).to_numpy("embedding")
    # ---- fp64 inputs (float32_inputs=False): PCA and OLS on the fp64 data
    Xr64 = g["Xr"].astype(np.float64)
    p64 = PCA(k=3, inputCol="features", float32_inputs=False, **nw).fit(frame(Xr64))
    out["pca64_components"] = np.asarray(p64.components_)
    l64 = LinearRegression(float32_inputs=False, **nw).fit(frame(Xr64, g["yr"]))
    out["ols64_coef"] = np.asarray(l64.coef_, np.float64).ravel()
    # ---- save -> load round trips from every rank to ONE shared path per model (rank-0 writes)
    from spark_rapids_ml_nai_amd.classification import LogisticRegressionModel
    from spark_rapids_ml_nai_amd.clustering import KMeansModel
    from spark_rapids_ml_nai_amd.feature import PCAModel
    from spark_rapids_ml_nai_amd.regression import RandomForestRegressionModel

    mdir = os.path.join(args.out, "models")
    rt = []
    for tag, mdl, cls, X, colname in (("pca", pm, PCAModel, g["Xr"], "pca"), ("kmeans", km, KMeansModel, g["Xb"],
                                                                                "prediction"),
                                      ("logreg", lg, LogisticRegressionModel, g["Xr"], "prediction"),
                                      ("rfr", rfr, RandomForestRegressionModel, g["Xr"], "prediction")):
        p = os.path.join(mdir, tag)
        mdl.write().overwrite().save(p)
        back = cls.load(p)
        a = mdl.transform(frame(X)).to_numpy(colname)
        b = back.transform(frame(X)).to_numpy(colname)
        rt.append(float(np.max(np.abs(np.asarray(a, np.float64) - np.asarray(b, np.float64)))))
    out["roundtrip_maxdiff"] = np.array(rt)

    os.makedirs(args.out, exist_ok=True)
    np.savez(os.path.join(args.out, "rank%d.npz" % rank), **out)
    if not args.single:
        dist.barrier()
        dist.destroy_process_group()
    print("SPMD-MATRIX-OK rank %d/%d" % (rank, world), flush=True)


if __name__ == "__main__":
    main()
