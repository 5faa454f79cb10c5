"""Writes the example notebooks in notebooks/ (the reference ships one notebook per algorithm,
notebooks/*.ipynb). Each notebook is a list of markdown / code cells; tests/test_notebooks.py
executes every code cell (CPU path in CI, the HIP kernels on a GPU box).

    python tools/make_notebooks.py
"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "notebooks")

SETUP = """import numpy as np
from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.ops import native
print("MI355X HIP kernels available:", native.available())"""

NOTEBOOKS = {
    "kmeans": [
        ("md", "# KMeans\nk-means‖ (default) or random init, Lloyd iterations on the split-bf16 MFMA distance "
               "kernel with a fused arg-min (`pkg/models/kmeans.py`). Same API as `pyspark.ml.clustering.KMeans`."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import make_blobs
X, y = make_blobs(n_samples=20000, n_features=16, centers=8, random_state=0)
df = DataFrame.from_numpy(X.astype(np.float32), num_partitions=2)
from spark_rapids_ml_nai_amd.clustering import KMeans
km = KMeans(k=8, maxIter=20, seed=1).setFeaturesCol("features")
model = km.fit(df)
print("iterations:", model._model_attributes.get("n_iter"))
print("centres:", np.round(np.asarray(model.clusterCenters())[:3], 2))"""),
        ("code", """out = model.transform(df)
pred = out.to_numpy("prediction")
from sklearn.metrics import adjusted_rand_score
print("ARI vs generating blobs:", round(adjusted_rand_score(y, pred), 4))
assert adjusted_rand_score(y, pred) > 0.9"""),
    ],
    "pca": [
        ("md", "# PCA\nStreamed moments + MFMA SYRK covariance, device top-k eigensolver, sign-fixed components "
               "(`pkg/models/pca.py`). Spark semantics: `transform` projects the uncentred rows."),
        ("code", SETUP),
        ("code", """rng = np.random.default_rng(0)
X = rng.standard_normal((5000, 40)) @ rng.standard_normal((40, 40))
df = DataFrame.from_numpy(X.astype(np.float32))
from spark_rapids_ml_nai_amd.feature import PCA
model = PCA(k=3, inputCol="features", outputCol="pca").fit(df)
print("explained variance:", np.round(model.explainedVariance.toArray(), 4))
from sklearn.decomposition import PCA as SkPCA
sk = SkPCA(3).fit(X)
assert np.allclose(np.abs(model.components_), np.abs(sk.components_), atol=1e-3)
print(model.transform(df).select("pca").limit(2).collect())"""),
    ],
    "linear-regression": [
        ("md", "# LinearRegression\nOLS / Ridge / Lasso / ElasticNet from one pass of sufficient statistics "
               "(SYRK Gram + Xᵀy), device Cholesky or block coordinate descent (`pkg/models/linear.py`)."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import make_regression
X, y = make_regression(n_samples=20000, n_features=30, noise=5.0, random_state=0)
df = DataFrame.from_numpy(X.astype(np.float32), y.astype(np.float32), num_partitions=2)
from spark_rapids_ml_nai_amd.regression import LinearRegression
for reg, l1 in [(0.0, 0.0), (0.1, 0.0), (0.1, 0.5)]:
    m = LinearRegression(regParam=reg, elasticNetParam=l1, standardization=False).fit(df)
    print(reg, l1, "intercept", round(m.intercept, 4), "coef[:3]", np.round(m.coefficients.toArray()[:3], 3))"""),
        ("code", """from spark_rapids_ml_nai_amd.evaluation import RegressionEvaluator
pred = m.transform(df)
print("RMSE:", RegressionEvaluator(metricName="rmse").evaluate(pred))"""),
    ],
    "logistic-regression": [
        ("md", "# LogisticRegression\nOne fused loss+gradient pass per evaluation; the L-BFGS / OWL-QN step runs "
               "on the device (`pkg/models/qn.py`). Binomial and multinomial, L1 / L2 / ElasticNet."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import make_classification
X, y = make_classification(n_samples=20000, n_features=20, n_informative=10, random_state=0)
df = DataFrame.from_numpy(X.astype(np.float32), y.astype(np.float32), num_partitions=2)
from spark_rapids_ml_nai_amd.classification import LogisticRegression
model = LogisticRegression(regParam=0.001, maxIter=100).fit(df)
print("iterations:", model.num_iters, "objective:", round(model.objective, 6))
out = model.transform(df)
acc = float((out.to_numpy("prediction") == y).mean())
print("train accuracy:", round(acc, 4))
assert acc > 0.7"""),
        ("code", """X3, y3 = make_classification(n_samples=9000, n_features=12, n_informative=8, n_classes=3, random_state=1)
df3 = DataFrame.from_numpy(X3.astype(np.float32), y3.astype(np.float32))
m3 = LogisticRegression(regParam=0.01, maxIter=100).fit(df3)
print("multinomial coefficient matrix:", m3.coefficientMatrix.toArray().shape)"""),
    ],
    "random-forest": [
        ("md", "# RandomForestClassifier / RandomForestRegressor\nQuantised features, LDS-privatised level-wise "
               "histograms, device split search and routing; inference with rows staged in LDS (`pkg/models/forest.py`)."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import make_classification
X, y = make_classification(n_samples=20000, n_features=20, n_informative=8, random_state=0)
df = DataFrame.from_numpy(X.astype(np.float32), y.astype(np.float32), num_partitions=2)
from spark_rapids_ml_nai_amd.classification import RandomForestClassifier
model = RandomForestClassifier(numTrees=20, maxDepth=8, seed=1).fit(df)
out = model.transform(df)
acc = float((out.to_numpy("prediction") == y).mean())
print("trees:", model.getNumTrees, "nodes:", model.totalNumNodes, "train accuracy:", round(acc, 4))
print("top features:", np.argsort(-model.featureImportances.toArray())[:5])
assert acc > 0.85"""),
        ("code", """from spark_rapids_ml_nai_amd.regression import RandomForestRegressor
from sklearn.datasets import make_regression
Xr, yr = make_regression(n_samples=10000, n_features=10, noise=1.0, random_state=0)
dfr = DataFrame.from_numpy(Xr.astype(np.float32), yr.astype(np.float32))
mr = RandomForestRegressor(numTrees=10, maxDepth=6, seed=1).fit(dfr)
print("regressor trees:", mr.getNumTrees)"""),
    ],
    "knn": [
        ("md", "# NearestNeighbors (exact)\nFused MFMA distance tiles + LDS top-k (k ≤ 64) or distance chunks + "
               "radix select (k ≤ 1024); queries ride a point-to-point ring across ranks (`pkg/models/knn.py`)."),
        ("code", SETUP),
        ("code", """rng = np.random.default_rng(0)
items = rng.standard_normal((20000, 16)).astype(np.float32)
queries = items[:200] + 0.01
from spark_rapids_ml_nai_amd.knn import NearestNeighbors
nn = NearestNeighbors(k=5, inputCol="features", num_workers=2)
model = nn.fit(DataFrame.from_numpy(items, num_partitions=2))
_, _, knn_df = model.kneighbors(DataFrame.from_numpy(queries))
rows = knn_df.collect()
print(rows[0])
assert rows[0].indices[0] == rows[0].query_unique_id"""),
    ],
    "approx-nearest-neighbors": [
        ("md", "# ApproximateNearestNeighbors (IVF-Flat)\nk-means coarse quantiser, contiguous inverted lists, "
               "probe-scan kernel (`pkg/models/knn.py`)."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import make_blobs
X, _ = make_blobs(n_samples=20000, n_features=16, centers=20, random_state=0)
X = X.astype(np.float32)
from spark_rapids_ml_nai_amd.knn import ApproximateNearestNeighbors
ann = ApproximateNearestNeighbors(k=10, algoParams={"nlist": 32, "nprobe": 8}, inputCol="features")
model = ann.fit(DataFrame.from_numpy(X))
_, _, knn_df = model.kneighbors(DataFrame.from_numpy(X[:500]))
from sklearn.neighbors import NearestNeighbors as SkNN
_, exact = SkNN(n_neighbors=10).fit(X).kneighbors(X[:500])
got = np.stack([np.asarray(r.indices) for r in sorted(knn_df.collect(), key=lambda r: r.query_unique_id)])
recall = np.mean([len(set(a) & set(b)) / 10 for a, b in zip(got, exact)])
print("recall@10:", round(recall, 4))
assert recall > 0.9"""),
    ],
    "dbscan": [
        ("md", "# DBSCAN\nε-degree and core-link sweeps over 128×128 distance tiles, device union-find "
               "(`pkg/models/dbscan.py`); no N×N matrix."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import make_blobs
X, _ = make_blobs(n_samples=5000, n_features=4, centers=5, cluster_std=0.5, random_state=0)
from spark_rapids_ml_nai_amd.clustering import DBSCAN
model = DBSCAN(eps=0.5, min_samples=5).fit(DataFrame.from_numpy(X.astype(np.float32)))
labels = model.transform(DataFrame.from_numpy(X.astype(np.float32))).to_numpy("prediction")
from sklearn.cluster import DBSCAN as SkDBSCAN
from sklearn.metrics import adjusted_rand_score
ref = SkDBSCAN(eps=0.5, min_samples=5).fit_predict(X)
print("clusters:", len(set(labels) - {-1}), "ARI vs sklearn:", round(adjusted_rand_score(ref, labels), 4))
assert adjusted_rand_score(ref, labels) > 0.99"""),
    ],
    "umap": [
        ("md", "# UMAP\nkNN graph, fused smooth-kNN / membership and fuzzy-union kernels, device spectral init, "
               "edge-parallel SGD epochs (`pkg/models/umap.py`). Quality gate: trustworthiness."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import load_digits
from sklearn.manifold import trustworthiness
X, y = load_digits(return_X_y=True)
from spark_rapids_ml_nai_amd.umap import UMAP
umap = UMAP(n_neighbors=15, random_state=1, featuresCol="features")
model = umap.fit(DataFrame.from_numpy(X.astype(np.float32)))
emb = model.embedding_
tw = trustworthiness(X, emb, n_neighbors=15)
print("embedding:", emb.shape, "trustworthiness:", round(tw, 4))
assert tw > 0.9"""),
    ],
    "cv-rf-regressor": [
        ("md", "# CrossValidator over a RandomForestRegressor grid\nSingle-pass `fitMultiple` per fold and a "
               "one-pass transform/evaluate (`pkg/tuning.py`)."),
        ("code", SETUP),
        ("code", """from sklearn.datasets import make_regression
X, y = make_regression(n_samples=6000, n_features=10, noise=2.0, random_state=0)
df = DataFrame.from_numpy(X.astype(np.float32), y.astype(np.float32))
from spark_rapids_ml_nai_amd.regression import RandomForestRegressor
from spark_rapids_ml_nai_amd.tuning import CrossValidator, ParamGridBuilder
from spark_rapids_ml_nai_amd.evaluation import RegressionEvaluator
rf = RandomForestRegressor(seed=1)
grid = ParamGridBuilder().addGrid(rf.maxDepth, [3, 6]).addGrid(rf.numTrees, [5, 10]).build()
cv = CrossValidator(estimator=rf, estimatorParamMaps=grid, evaluator=RegressionEvaluator(), numFolds=3, seed=1)
cvm = cv.fit(df)
print("avg RMSE per grid point:", np.round(cvm.avgMetrics, 3))
print("best maxDepth:", cvm.bestModel.getOrDefault("maxDepth"))"""),
    ],
}


def _cell(kind: str, text: str) -> dict:
    lines = text.split("\n")
    src = [ln + "\n" for ln in lines[:-1]] + [lines[-1]]
    if kind == "md":
        return {"cell_type": "markdown", "metadata": {}, "source": src}
    return {"cell_type": "code", "execution_count": None, "metadata": {}, "outputs": [], "source": src}


def main() -> None:
    os.makedirs(OUT, exist_ok=True)
    for name, cells in NOTEBOOKS.items():
        nb = {"cells": [_cell(k, t) for k, t in cells],
              "metadata": {"kernelspec": {"display_name": "Python 3", "language": "python", "name": "python3"},
                           "language_info": {"name": "python"}},
              "nbformat": 4, "nbformat_minor": 5}
        with open(os.path.join(OUT, name + ".ipynb"), "w") as fh:
            json.dump(nb, fh, indent=1)
            fh.write("\n")
    print("wrote %d notebooks to %s" % (len(NOTEBOOKS), OUT))


if __name__ == "__main__":
    main()
