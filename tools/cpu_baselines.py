"""Same-host CPU denominators for the BASELINE.json north-star configs (BASELINE.md asks for the
Spark-ML CPU time on the same host; pyspark / a JVM are not in this image, so scikit-learn on the
host's CPU cores stands in, clearly labelled). Each config runs at a reduced row count on the same
generator family and is extrapolated linearly in rows (and in trees for the forest): one JSON line
per config with the measured seconds, the scale factor and the extrapolated full-size seconds.

    python tools/cpu_baselines.py [--configs pca,kmeans,logreg,rf] [--threads 16]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="pca,kmeans,logreg,rf")
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    os.environ.setdefault("OMP_NUM_THREADS", str(a.threads))
    import numpy as np
    import torch

    torch.set_num_threads(a.threads)
    from spark_rapids_ml_nai_amd.bench import datagen

    cpu = torch.device("cpu")
    for name in a.configs.split(","):
        rec = {"config": name, "threads": a.threads, "impl": "scikit-learn " + __import__("sklearn").__version__}
        if name == "pca":
            from sklearn.decomposition import PCA

            X = datagen.low_rank_matrix(10_000, 128, cpu, seed=7000).numpy()
            t0 = time.perf_counter()
            PCA(n_components=3, svd_solver="full").fit(X)
            rec.update(rows=10_000, full_rows=10_000, scale=1.0, fit_s=time.perf_counter() - t0)
        elif name == "kmeans":
            from sklearn.cluster import KMeans

            m = 10_000_000
            X = datagen.uniform(m, 64, cpu, seed=7000).numpy()
            t0 = time.perf_counter()
            KMeans(n_clusters=20, max_iter=20, tol=0.0, n_init=1, init="random", random_state=1,
                   algorithm="lloyd").fit(X)
            rec.update(rows=m, full_rows=100_000_000, scale=10.0, fit_s=time.perf_counter() - t0)
        elif name == "logreg":
            from sklearn.linear_model import LogisticRegression

            m = 2_000_000
            X, y = datagen.classification(m, 256, cpu, seed=7000, n_informative=128, n_redundant=64)
            X, y = X.numpy(), y.numpy()
            t0 = time.perf_counter()
            LogisticRegression(C=1.0 / (1e-5 * m), max_iter=100, tol=1e-6, solver="lbfgs").fit(X, y)
            rec.update(rows=m, full_rows=200_000_000, scale=100.0, fit_s=time.perf_counter() - t0)
        elif name == "rf":
            from sklearn.ensemble import RandomForestClassifier

            m, trees = 1_000_000, 10
            X, y = datagen.classification(m, 64, cpu, seed=7000, n_informative=32, n_redundant=16)
            X, y = X.numpy(), y.numpy()
            t0 = time.perf_counter()
            RandomForestClassifier(n_estimators=trees, max_depth=16, n_jobs=a.threads, random_state=1).fit(X, y)
            # rows x trees (sklearn sorts exact thresholds: n log n per node level; linear is a floor)
            rec.update(rows=m, full_rows=50_000_000, trees=trees, full_trees=100, scale=50.0 * 10.0,
                       fit_s=time.perf_counter() - t0)
        else:
            raise ValueError(name)
        rec["fit_s"] = round(rec["fit_s"], 3)
        rec["extrapolated_full_s"] = round(rec["fit_s"] * rec["scale"], 1)
        print(json.dumps(rec), flush=True)
        del rec
        np.random.seed(0)


if __name__ == "__main__":
    main()
