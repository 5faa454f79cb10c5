"""UMAP layout epochs alone at a north-star-like graph (IVF kNN of blobs, list order, fuzzy union):

    python tools/umap_epoch_bench.py [--rows 4000000] [--epochs 20]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--cols", type=int, default=128)
    ap.add_argument("--epochs", type=int, default=20)
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models import umap as U
    from spark_rapids_ml_nai_amd.models.knn_graph import build_knn_graph

    dev = torch.device("cuda", 0)
    X, _ = datagen.blobs(a.rows, a.cols, dev, seed=7000, centers=20)
    dist, idx, order = build_knn_graph(X, 15, "ivf", None, 1, None, list_order=U.LIST_ORDER)
    del X
    _, _, w = ops.umap_smooth_knn(dist, idx, 15.0, local_connectivity=1.0, self_rows=True)
    rows, cols, vals = ops.umap_fuzzy_union_knn(idx, w, 1.0)
    N = dist.shape[0]
    a_, b_ = U.find_ab_params(1.0, 0.1)
    print("edges %d" % rows.numel(), flush=True)
    for rep in range(2):
        emb = torch.rand(N, 2, device=dev) * 10
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        U.optimize_layout(emb, emb, rows, cols, vals, a.epochs, a_, b_, 1.0, 1.0, 5.0, True, 3, pull=U.PULL)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print("epochs %d: %.4f s (%.2f ms/epoch)" % (a.epochs, dt, 1e3 * dt / a.epochs), flush=True)


if __name__ == "__main__":
    main()
