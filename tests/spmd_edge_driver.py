"""Driver of tests/test_spmd_edges.py: SPMD (torchrun) launch-mode edges beyond fit / transform.

``--mode saves``: every rank fits the same model and calls ``write().overwrite().save(path)`` on ONE
shared path ``--reps`` times, then loads it back; each rank records how many saves raised and
whether every reload predicts like the fitted model (rank-0-only writes, atomic rename).

``--mode empty``: rank ``--empty-rank`` holds no rows; every rank fits each estimator and records
the error message it got and how long it took to get it (the ranks must agree, quickly).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--mode", choices=("saves", "empty"), required=True)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--empty-rank", type=int, default=1)
    args = ap.parse_args()
    os.environ["SRML_FORCE_CPU"] = "1"
    import torch
    import torch.distributed as dist

    torch.set_num_threads(1)
    dist.init_process_group("gloo", init_method="env://")
    rank, world = dist.get_rank(), dist.get_world_size()
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.classification import LogisticRegression, RandomForestClassifier
    from spark_rapids_ml_nai_amd.clustering import KMeans
    from spark_rapids_ml_nai_amd.feature import PCA
    from spark_rapids_ml_nai_amd.regression import LinearRegression, LinearRegressionModel

    rng = np.random.default_rng(7)
    N, D = 600, 6
    X = rng.standard_normal((N, D)).astype(np.float32)
    y = (X @ rng.uniform(-2, 2, D) + 0.3).astype(np.float64)
    yc = (X[:, 0] > 0).astype(np.float64)
    bounds = np.linspace(0, N, world + 1).astype(int)
    lo, hi = int(bounds[rank]), int(bounds[rank + 1])
    out = {"rank": rank, "world": world}
    if args.mode == "saves":
        path = os.path.join(args.out, "shared_model")
        model = LinearRegression(regParam=0.1).fit(DataFrame.from_numpy(X[lo:hi], y[lo:hi]))
        ref = model.transform(DataFrame.from_numpy(X)).to_numpy("prediction")
        save_errors, load_ok = [], 0
        for i in range(args.reps):
            try:
                model.write().overwrite().save(path)
            except Exception as e:  # noqa: BLE001
                save_errors.append(repr(e)[:300])
            try:
                m2 = LinearRegressionModel.load(path)
                p2 = m2.transform(DataFrame.from_numpy(X)).to_numpy("prediction")
                load_ok += int(np.allclose(p2, ref, rtol=1e-6, atol=1e-6))
            except Exception as e:  # noqa: BLE001
                save_errors.append("load: " + repr(e)[:300])
        # not-overwrite on an existing path: the same IOError on every rank
        try:
            model.write().save(path)
            out["exists_error"] = None
        except Exception as e:  # noqa: BLE001
            out["exists_error"] = type(e).__name__ + ": " + str(e)
        out.update(save_errors=save_errors, load_ok=load_ok, reps=args.reps,
                   leftovers=sorted(f for f in os.listdir(args.out) if f.startswith(".shared_model")))
    else:
        if rank == args.empty_rank:
            lo = hi = 0
        fits = {
            "PCA": lambda: PCA(k=2, inputCol="features").fit(DataFrame.from_numpy(X[lo:hi])),
            "KMeans": lambda: KMeans(k=3, seed=1).fit(DataFrame.from_numpy(X[lo:hi])),
            "LinearRegression": lambda: LinearRegression().fit(DataFrame.from_numpy(X[lo:hi], y[lo:hi])),
            "LogisticRegression": lambda: LogisticRegression(maxIter=5).fit(DataFrame.from_numpy(X[lo:hi], yc[lo:hi])),
            "RandomForestClassifier": lambda: RandomForestClassifier(numTrees=4, maxDepth=3).fit(
                DataFrame.from_numpy(X[lo:hi], yc[lo:hi])),
        }
        res = {}
        for name, fn in fits.items():
            t0 = time.perf_counter()
            try:
                fn()
                msg = None
            except Exception as e:  # noqa: BLE001
                msg = str(e)
            res[name] = {"error": msg, "seconds": round(time.perf_counter() - t0, 3)}
        out["fits"] = res
    with open(os.path.join(args.out, "rank%d.json" % rank), "w") as f:
        json.dump(out, f)
    dist.barrier()
    dist.destroy_process_group()
    print("SPMD-EDGE-OK rank %d/%d" % (rank, world), flush=True)


if __name__ == "__main__":
    main()
