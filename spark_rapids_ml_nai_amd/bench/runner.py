"""Per-algorithm benchmark runner (reference ``python/benchmark/benchmark_runner.py`` +
``benchmark/base.py`` + ``bench_*.py``).

    python -m spark_rapids_ml_nai_amd.bench.runner <algorithm> --train_path DATA [--transform_path DATA]
        [--num_gpus N] [--num_runs R] [--report_path out.csv] [--cpu] [--<estimator param> VALUE ...]

Algorithms: approximate_nearest_neighbors, dbscan, kmeans, knn, linear_regression, pca,
random_forest_classifier, random_forest_regressor, logistic_regression, umap.

Every run times fit, transform and total wall clock and computes the reference's quality metric
(KMeans inertia, PCA orthonormality + projected variance, LinReg RMSE, LogReg log-loss / AUC /
accuracy, RF accuracy or RMSE, UMAP trustworthiness, DBSCAN silhouette, ANN average recall vs
exact kNN). ``--cpu`` runs the scikit-learn equivalent instead (the reference's CPU baseline is
pyspark.ml, which is not part of this image). Unknown ``--name value`` options become estimator
parameters (the reference derives them from the estimator signature).
"""
from __future__ import annotations

import argparse
import ast
import csv
import json
import os
import sys
import time
import warnings
from typing import Any, Callable, Dict, List, Optional, Tuple

import numpy as np

from ..core.dataframe import DataFrame

warnings.filterwarnings("ignore")


def _literal(v: str) -> Any:
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return {"true": True, "false": False, "none": None}.get(v.lower(), v)


def with_benchmark(phrase: str, fn: Callable[[], Any]) -> Tuple[Any, float]:
    t0 = time.perf_counter()
    res = fn()
    dt = time.perf_counter() - t0
    print("-" * 100)
    print("%s takes %.3f seconds" % (phrase, dt))
    return res, dt


# ------------------------------------------------------------------------------------------
# data helpers
# ------------------------------------------------------------------------------------------
def _features(df: DataFrame, col: Optional[str]) -> np.ndarray:
    from ..core.base import _dense_from_df

    if col is not None:
        return _dense_from_df(df, col, None, np.float32)
    cols = [c for c in df.columns if c.startswith("c") and c[1:].isdigit()]
    return _dense_from_df(df, None, cols, np.float32)


def _feature_kwargs(df: DataFrame, col: Optional[str], key: str = "featuresCol") -> Dict[str, Any]:
    if col is not None:
        return {key: col}
    return {key: [c for c in df.columns if c.startswith("c") and c[1:].isdigit()]}


def _sample(X: np.ndarray, k: int, seed: int = 0) -> np.ndarray:
    if X.shape[0] <= k:
        return np.arange(X.shape[0])
    return np.random.default_rng(seed).choice(X.shape[0], k, replace=False)


# ------------------------------------------------------------------------------------------
# algorithms: (fit+transform on our estimators, sklearn baseline, score)
# ------------------------------------------------------------------------------------------
class Bench:
    name = ""
    supervised = False

    def __init__(self, args: argparse.Namespace, params: Dict[str, Any]) -> None:
        self.args = args
        self.params = params

    def estimator(self, train: DataFrame) -> Any:
        raise NotImplementedError

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        return {}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        raise NotImplementedError


class KMeansBench(Bench):
    name = "kmeans"

    def estimator(self, train: DataFrame) -> Any:
        from ..clustering import KMeans

        return KMeans(num_workers=self.args.num_gpus, **_feature_kwargs(train, self.args.feature_col), **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        C = np.asarray(model.cluster_centers_, dtype=np.float64)
        d = ((X[:, None, :] - C[None]) ** 2).sum(-1) if X.shape[0] * C.shape[0] < 5e7 else None
        if d is None:
            import torch

            from .. import ops

            Xt = torch.from_numpy(X)
            lab, dist = ops.nearest_centroid(Xt, torch.from_numpy(C).float())
            return {"inertia": float(dist.double().sum())}
        return {"inertia": float(d.min(1).sum())}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.cluster import KMeans as SK

        k = int(self.params.get("k", 2))
        m = SK(n_clusters=k, max_iter=int(self.params.get("maxIter", 20)), n_init=1,
               init="random" if self.params.get("initMode") == "random" else "k-means++").fit(X)
        return m, m.predict(Xt)


class PCABench(Bench):
    name = "pca"

    def estimator(self, train: DataFrame) -> Any:
        from ..feature import PCA

        kw = _feature_kwargs(train, self.args.feature_col, "inputCol")
        return PCA(num_workers=self.args.num_gpus, outputCol="pca_features", **kw, **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        pc = np.asarray(model.components_, dtype=np.float64)
        ortho = float(np.abs(pc @ pc.T - np.eye(pc.shape[0])).max())
        idx = _sample(X, 100000)
        Xs = X[idx] - X[idx].mean(0)
        proj = Xs @ pc.T
        return {"orthonormality_err": ortho, "projected_variance": float(proj.var(0).sum())}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.decomposition import PCA as SK

        m = SK(n_components=int(self.params.get("k", 3)), svd_solver="full").fit(X)
        return m, m.transform(Xt)


class LinearRegressionBench(Bench):
    name = "linear_regression"
    supervised = True

    def estimator(self, train: DataFrame) -> Any:
        from ..regression import LinearRegression

        return LinearRegression(num_workers=self.args.num_gpus, labelCol=self.args.label_col,
                                **_feature_kwargs(train, self.args.feature_col), **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        pred = out.to_numpy(model.getPredictionCol()) if out is not None else None
        if pred is None or y is None:
            return {}
        return {"rmse": float(np.sqrt(np.mean((pred - y) ** 2)))}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.linear_model import ElasticNet, LinearRegression as SK, Ridge

        reg = float(self.params.get("regParam", 0.0))
        en = float(self.params.get("elasticNetParam", 0.0))
        if reg == 0:
            m = SK().fit(X, y)
        elif en == 0:
            m = Ridge(alpha=reg * X.shape[0]).fit(X, y)
        else:
            m = ElasticNet(alpha=reg, l1_ratio=en, max_iter=int(self.params.get("maxIter", 100))).fit(X, y)
        return m, m.predict(Xt)


class LogisticRegressionBench(Bench):
    name = "logistic_regression"
    supervised = True

    def estimator(self, train: DataFrame) -> Any:
        from ..classification import LogisticRegression

        return LogisticRegression(num_workers=self.args.num_gpus, labelCol=self.args.label_col,
                                  **_feature_kwargs(train, self.args.feature_col), **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        if out is None or y is None:
            return {}
        from ..metrics import binary_auc

        pred = out.to_numpy(model.getPredictionCol())
        prob = out.to_numpy(model.getProbabilityCol())
        p1 = np.clip(prob[:, -1] if prob.ndim == 2 else prob, 1e-15, 1 - 1e-15)
        res = {"accuracy": float((pred == y).mean())}
        if prob.ndim == 2 and prob.shape[1] == 2:
            res["log_loss"] = float(-np.mean(y * np.log(p1) + (1 - y) * np.log(1 - p1)))
            res["auc"] = float(binary_auc(y, p1))
        return res

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.linear_model import LogisticRegression as SK

        reg = float(self.params.get("regParam", 0.0))
        m = SK(C=1.0 / max(reg * X.shape[0], 1e-12), max_iter=int(self.params.get("maxIter", 100))).fit(X, y)
        return m, m.predict(Xt)


class RandomForestClassifierBench(Bench):
    name = "random_forest_classifier"
    supervised = True

    def estimator(self, train: DataFrame) -> Any:
        from ..classification import RandomForestClassifier

        return RandomForestClassifier(num_workers=self.args.num_gpus, labelCol=self.args.label_col,
                                      **_feature_kwargs(train, self.args.feature_col), **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        if out is None or y is None:
            return {}
        return {"accuracy": float((out.to_numpy(model.getPredictionCol()) == y).mean())}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.ensemble import RandomForestClassifier as SK

        m = SK(n_estimators=int(self.params.get("numTrees", 20)), max_depth=int(self.params.get("maxDepth", 5)),
               n_jobs=-1).fit(X, y)
        return m, m.predict(Xt)


class RandomForestRegressorBench(RandomForestClassifierBench):
    name = "random_forest_regressor"

    def estimator(self, train: DataFrame) -> Any:
        from ..regression import RandomForestRegressor

        return RandomForestRegressor(num_workers=self.args.num_gpus, labelCol=self.args.label_col,
                                     **_feature_kwargs(train, self.args.feature_col), **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        if out is None or y is None:
            return {}
        return {"rmse": float(np.sqrt(np.mean((out.to_numpy(model.getPredictionCol()) - y) ** 2)))}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.ensemble import RandomForestRegressor as SK

        m = SK(n_estimators=int(self.params.get("numTrees", 20)), max_depth=int(self.params.get("maxDepth", 5)),
               n_jobs=-1).fit(X, y)
        return m, m.predict(Xt)


class UMAPBench(Bench):
    name = "umap"

    def estimator(self, train: DataFrame) -> Any:
        from ..umap import UMAP

        return UMAP(num_workers=self.args.num_gpus, **_feature_kwargs(train, self.args.feature_col), **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        from sklearn.manifold import trustworthiness

        emb = out.to_numpy(model.getOutputCol()) if out is not None else np.asarray(model.embedding_)
        idx = _sample(X, 5000)
        return {"trustworthiness": float(trustworthiness(X[idx], emb[idx], n_neighbors=15))}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        raise RuntimeError("umap-learn is not installed in this image")


class DBSCANBench(Bench):
    name = "dbscan"

    def estimator(self, train: DataFrame) -> Any:
        from ..clustering import DBSCAN

        return DBSCAN(num_workers=self.args.num_gpus, **_feature_kwargs(train, self.args.feature_col), **self.params)

    def score(self, model: Any, out: Optional[DataFrame], X: np.ndarray, y: Optional[np.ndarray]) -> Dict[str, float]:
        from sklearn.metrics import silhouette_score

        lab = out.to_numpy(model.getPredictionCol())
        idx = _sample(X, 10000)
        if len(set(lab[idx].tolist())) < 2:
            return {"n_clusters": int(lab.max() + 1)}
        return {"silhouette": float(silhouette_score(X[idx], lab[idx])), "n_clusters": int(lab.max() + 1)}

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.cluster import DBSCAN as SK

        m = SK(eps=float(self.params.get("eps", 0.5)), min_samples=int(self.params.get("min_samples", 5))).fit(X)
        return m, m.labels_


class KNNBench(Bench):
    name = "knn"

    def estimator(self, train: DataFrame) -> Any:
        from ..knn import NearestNeighbors

        return NearestNeighbors(num_workers=self.args.num_gpus,
                                **_feature_kwargs(train, self.args.feature_col, "inputCol"), **self.params)

    def cpu(self, X: np.ndarray, y: Optional[np.ndarray], Xt: np.ndarray) -> Tuple[Any, Any]:
        from sklearn.neighbors import NearestNeighbors as SK

        m = SK(n_neighbors=int(self.params.get("k", 5)), algorithm="brute").fit(X)
        return m, m.kneighbors(Xt)


class ANNBench(KNNBench):
    name = "approximate_nearest_neighbors"

    def estimator(self, train: DataFrame) -> Any:
        from ..knn import ApproximateNearestNeighbors

        return ApproximateNearestNeighbors(num_workers=self.args.num_gpus,
                                           **_feature_kwargs(train, self.args.feature_col, "inputCol"),
                                           **self.params)


BENCHMARKS = {b.name: b for b in (ANNBench, DBSCANBench, KMeansBench, KNNBench, LinearRegressionBench, PCABench,
                                  RandomForestClassifierBench, RandomForestRegressorBench, LogisticRegressionBench,
                                  UMAPBench)}


def _parse(argv: List[str]) -> Tuple[argparse.Namespace, Dict[str, Any]]:
    p = argparse.ArgumentParser(prog="runner", description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    p.add_argument("algorithm", choices=sorted(BENCHMARKS))
    p.add_argument("--train_path", required=True)
    p.add_argument("--transform_path", default=None)
    p.add_argument("--num_gpus", type=int, default=1)
    p.add_argument("--num_runs", type=int, default=1)
    p.add_argument("--report_path", default="")
    p.add_argument("--cpu", action="store_true", help="scikit-learn baseline instead of the GPU estimators")
    p.add_argument("--feature_col", default="feature_array")
    p.add_argument("--label_col", default="label")
    p.add_argument("--no_quality", action="store_true")
    p.add_argument("--verbose", action="store_true")
    args, rest = p.parse_known_args(argv)
    params: Dict[str, Any] = {}
    i = 0
    while i < len(rest):
        tok = rest[i]
        if not tok.startswith("--"):
            raise SystemExit("unexpected argument %r" % tok)
        key = tok[2:]
        if "=" in key:
            key, val = key.split("=", 1)
            i += 1
        elif i + 1 < len(rest) and not rest[i + 1].startswith("--"):
            val = rest[i + 1]
            i += 2
        else:
            val, i = "true", i + 1
        params[key] = _literal(val)
    if args.feature_col in ("", "none", "None"):
        args.feature_col = None
    return args, params


def run(argv: List[str]) -> List[Dict[str, Any]]:
    args, params = _parse(argv)
    bench = BENCHMARKS[args.algorithm](args, params)
    train = DataFrame.read_parquet(args.train_path)
    test = DataFrame.read_parquet(args.transform_path) if args.transform_path else train
    if args.feature_col is not None and args.feature_col not in train.columns:
        args.feature_col = None
    rows = []
    for r in range(args.num_runs):
        res: Dict[str, Any] = {"algorithm": args.algorithm, "run": r, "num_gpus": args.num_gpus,
                               "mode": "cpu-sklearn" if args.cpu else "gpu", "params": json.dumps(params)}
        t0 = time.perf_counter()
        X = _features(test, args.feature_col)
        y = test.to_numpy(args.label_col) if args.label_col in test.columns else None
        if args.cpu:
            Xtr = _features(train, args.feature_col)
            ytr = train.to_numpy(args.label_col) if args.label_col in train.columns else None
            (_, _), fit_t = with_benchmark("CPU fit+predict", lambda: bench.cpu(Xtr, ytr, X))
            res.update(fit=fit_t, transform=0.0)
        else:
            est = bench.estimator(train)
            model, fit_t = with_benchmark("fit", lambda: est.fit(train))
            out = None
            tr_t = 0.0
            if args.algorithm in ("knn", "approximate_nearest_neighbors"):
                (_, _, knn_df), tr_t = with_benchmark("kneighbors", lambda: model.kneighbors(test))
                if args.algorithm == "approximate_nearest_neighbors" and not args.no_quality:
                    res.update(_ann_recall(train, test, knn_df, args, params))
            else:
                out, tr_t = with_benchmark("transform", lambda: model.transform(test))
                if not args.no_quality:
                    res.update(bench.score(model, out, X, y))
            res.update(fit=fit_t, transform=tr_t)
        res["total"] = time.perf_counter() - t0
        print(res)
        rows.append(res)
    if args.report_path:
        new = not os.path.exists(args.report_path)
        keys = sorted({k for r in rows for k in r})
        with open(args.report_path, "a", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            if new:
                w.writeheader()
            for r in rows:
                w.writerow(r)
    return rows


def _ann_recall(train: DataFrame, test: DataFrame, knn_df: DataFrame, args: argparse.Namespace,
                params: Dict[str, Any]) -> Dict[str, float]:
    """Average recall of the approximate neighbours vs exact kNN on a query sample (reference
    ``bench_approximate_nearest_neighbors.py:223-274``)."""
    from ..knn import NearestNeighbors

    k = int(params.get("k", 5))
    kd = knn_df.toPandas()
    sample = kd.head(1000)
    qids = set(sample.iloc[:, 0].tolist())
    id_col = "unique_id"
    q_with = test.with_row_id(id_col) if id_col not in test.columns else test
    qmask = np.isin(q_with.to_numpy(id_col), list(qids))
    q_sub = q_with.filter(qmask)
    nn = NearestNeighbors(k=k, idCol=id_col, **_feature_kwargs(train, args.feature_col, "inputCol"))
    items = train.with_row_id(id_col) if id_col not in train.columns else train
    _, _, exact = nn.fit(items).kneighbors(q_sub)
    ex = {r[0]: set(r[1]) for r in exact.toPandas().itertuples(index=False)}
    rec = [len(set(r[1]) & ex[r[0]]) / float(k) for r in sample.itertuples(index=False) if r[0] in ex]
    return {"avg_recall": float(np.mean(rec)) if rec else float("nan")}


def main() -> int:
    run(sys.argv[1:])
    return 0


if __name__ == "__main__":
    sys.exit(main())
