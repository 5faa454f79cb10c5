"""The reference's UMAP notebook data points (BASELINE.md secondary table), re-measured:

* "blobs": 100k x 3000 blobs, fit on a 50 % sample (sample_fraction=0.5), transform all 100k rows
  (reference notebooks/umap.ipynb cells 38-45: GPU fit 24.94 s / transform 13.75 s);
* "mnist_shape": 52.5k x 784 train / 17.5k test synthetic blobs of MNIST's shape (the dataset itself
  is not available offline; reference cells 15/20: GPU fit 16.40 s / transform 13.21 s).

Prints one JSON line per case with fit / transform seconds and trustworthiness (k=15) on a
2000-row subsample of the transformed rows.
    python tools/umap_notebook.py [--cases blobs,mnist_shape]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
from sklearn.datasets import make_blobs  # noqa: E402
from sklearn.manifold import trustworthiness  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.umap import UMAP  # noqa: E402

REF = {"blobs": {"fit_s": 24.94, "transform_s": 13.75}, "mnist_shape": {"fit_s": 16.40, "transform_s": 13.21}}


def run(case: str) -> dict:
    if case == "blobs":
        X, _ = make_blobs(100_000, 3000, centers=10, cluster_std=1.0, random_state=0)
        train, test, frac = X, X, 0.5
    else:
        X, _ = make_blobs(70_000, 784, centers=10, cluster_std=4.0, random_state=0)
        X = np.abs(X)  # non-negative like pixel intensities
        train, test, frac = X[:52_500], X[52_500:], 1.0
    train = train.astype(np.float32)
    test = test.astype(np.float32)
    dtr, dte = DataFrame.from_numpy(train), DataFrame.from_numpy(test)
    est = UMAP(n_neighbors=15, n_components=2, random_state=1, sample_fraction=frac, featuresCol="features")
    t0 = time.perf_counter()
    model = est.fit(dtr)
    torch.cuda.synchronize() if torch.cuda.is_available() else None
    fit_s = time.perf_counter() - t0
    t0 = time.perf_counter()
    emb = model.transform(dte).to_numpy("embedding")
    transform_s = time.perf_counter() - t0
    rng = np.random.default_rng(0)
    sel = rng.choice(test.shape[0], size=min(2000, test.shape[0]), replace=False)
    tw = float(trustworthiness(test[sel], emb[sel], n_neighbors=15))
    return {"case": case, "rows_fit": int(train.shape[0] * frac), "rows_transform": int(test.shape[0]),
            "cols": int(train.shape[1]), "fit_s": round(fit_s, 3), "transform_s": round(transform_s, 3),
            "trustworthiness_k15": round(tw, 4), "ref_gpu": REF[case]}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="blobs,mnist_shape")
    a = ap.parse_args()
    for c in a.cases.split(","):
        print(json.dumps(run(c)), flush=True)


if __name__ == "__main__":
    main()
