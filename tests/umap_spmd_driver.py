"""Driver of tests/test_umap_spmd.py: ONE distributed UMAP fit (IVF graph + row-partitioned
spectral init + edge-parallel epochs) on the same global data, either single-process or as one
rank of a torchrun world (every rank holds the whole matrix, as the fit's all-gather leaves it).
Writes <out>/rank<r>.npz with the embedding and this rank's per-phase row counts."""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def data(n: int = 6000, d: int = 32) -> np.ndarray:
    from sklearn.datasets import make_classification

    X, _ = make_classification(n_samples=n, n_features=d, n_informative=12, n_redundant=8, n_classes=4,
                               n_clusters_per_class=2, random_state=3)
    return X.astype(np.float32)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--single", action="store_true")
    a = ap.parse_args()
    os.environ["SRML_FORCE_CPU"] = "1"
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    ctx = None
    rank = 0
    if not a.single:
        dist.init_process_group("gloo", init_method="env://")
        from spark_rapids_ml_nai_amd.parallel.context import spmd_context

        ctx = spmd_context()
        rank = ctx.rank
    from spark_rapids_ml_nai_amd.models import umap as U

    X = torch.from_numpy(data())
    params = {"n_neighbors": 12, "n_components": 2, "random_state": 5, "n_epochs": 120, "build_algo": "nn_descent",
              "build_kwds": {"nlist": 24, "nprobe": 8, "nnd_iters": 1}}
    emb = U.umap_fit(X, params, ctx=ctx)
    os.makedirs(a.out, exist_ok=True)
    np.savez(os.path.join(a.out, "rank%d.npz" % rank), emb=emb, phases=json.dumps(U.LAST_PHASES))
    if ctx is not None:
        dist.barrier()
        dist.destroy_process_group()
    print("UMAP-SPMD-OK", rank, json.dumps(U.LAST_PHASES), flush=True)


if __name__ == "__main__":
    main()
