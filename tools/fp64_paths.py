"""float32_inputs=False paths on the device, for a rocprofv3 check that only srml_* kernels (no
library GEMMs: Cijk_* / rocblas_*) run (VERDICT r1 task 4).

    rocprofv3 --kernel-trace --stats -d gpurun_out/fp64 -o fp64 -- python3 tools/fp64_paths.py
    python tools/fp64_paths.py --check gpurun_out/fp64/.../fp64_kernel_stats.csv

Fits PCA / LinearRegression (OLS + ridge) / KMeans / LogisticRegression in fp64 and runs exact
kNN with k=200 (radix-select path) on a 200k x 500 dataset; prints one line per step.
"""
import argparse
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(rows: int, cols: int) -> None:
    import numpy as np
    import torch

    from spark_rapids_ml_nai_amd import DataFrame, ops
    from spark_rapids_ml_nai_amd.classification import LogisticRegression
    from spark_rapids_ml_nai_amd.clustering import KMeans
    from spark_rapids_ml_nai_amd.feature import PCA
    from spark_rapids_ml_nai_amd.regression import LinearRegression

    rng = np.random.default_rng(0)
    X = rng.standard_normal((rows, cols))
    w = rng.standard_normal(cols)
    y = X @ w + 0.1 * rng.standard_normal(rows)
    yc = (y > 0).astype(np.float64)
    df = DataFrame.from_numpy(X, y)
    dfc = DataFrame.from_numpy(X, yc)
    steps = [
        ("pca", lambda: PCA(k=8, inputCol="features", float32_inputs=False).fit(df)),
        ("linreg_ols", lambda: LinearRegression(float32_inputs=False).fit(df)),
        ("linreg_ridge", lambda: LinearRegression(regParam=1e-3, float32_inputs=False).fit(df)),
        ("kmeans", lambda: KMeans(k=100, maxIter=10, float32_inputs=False, seed=1).fit(df)),
        ("logreg", lambda: LogisticRegression(maxIter=30, regParam=1e-4, float32_inputs=False).fit(dfc)),
    ]
    for name, fn in steps:
        t0 = time.perf_counter()
        m = fn()
        torch.cuda.synchronize()
        print("%-14s %.4f s  %s" % (name, time.perf_counter() - t0, type(m).__name__), flush=True)
    dev = torch.device("cuda", 0)
    Q = torch.from_numpy(X[:2000]).float().to(dev)
    I = torch.from_numpy(X).float().to(dev)
    t0 = time.perf_counter()
    d, i = ops.knn(Q, I, 200)
    torch.cuda.synchronize()
    print("%-14s %.4f s  %s" % ("knn_k200", time.perf_counter() - t0, tuple(d.shape)), flush=True)


def check(path: str) -> int:
    bad = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            n = r["Name"]
            if n.startswith("Cijk_") or "rocblas" in n.lower() or "hipblaslt" in n.lower():
                bad.append(n)
    for n in bad:
        print("LIBRARY KERNEL:", n[:140])
    print("library kernels: %d" % len(bad))
    return 1 if bad else 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=200_000)
    ap.add_argument("--cols", type=int, default=500)
    ap.add_argument("--check", default=None)
    a = ap.parse_args()
    if a.check:
        sys.exit(check(a.check))
    run(a.rows, a.cols)
