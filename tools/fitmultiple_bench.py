"""Hyper-parameter batching benchmark: a LogisticRegression grid fitted one setting at a time vs
batched (``logistic_fit_multi``: shared passes over X + one batched optimiser launch).

    python tools/fitmultiple_bench.py [--rows 1000000 --cols 3000 --grid 4 --iters 100]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=3000)
    ap.add_argument("--grid", type=int, default=4)
    ap.add_argument("--iters", type=int, default=100)
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models.logistic import logistic_fit, logistic_fit_multi, logistic_stats
    from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

    dev = torch.device("cuda", 0)
    X, y = datagen.classification(a.rows, a.cols, dev, seed=5)
    X = X.float().contiguous()
    y = y.float().contiguous()
    ctx = WorkerContext.single(dev)
    stats = logistic_stats(X, y, a.rows, ctx, False)
    regs = [10.0 ** (-5 + i) for i in range(a.grid)]
    settings = [dict(reg=r, l1_ratio=0.0, fit_intercept=True, standardization=False, max_iter=a.iters, tol=1e-30)
                for r in regs]
    logistic_fit_multi(X[:20000], y[:20000], 20000, ctx, settings[:2])  # warm up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    one = [logistic_fit(X, y, a.rows, ctx, s["reg"], 0.0, True, False, a.iters, 1e-30, stats=stats) for s in settings]
    torch.cuda.synchronize()
    t_seq = time.perf_counter() - t0
    t0 = time.perf_counter()
    bat = logistic_fit_multi(X, y, a.rows, ctx, settings, stats=stats)
    torch.cuda.synchronize()
    t_bat = time.perf_counter() - t0
    dobj = max(abs(p["objective"] - q["objective"]) for p, q in zip(one, bat))
    print(json.dumps({"rows": a.rows, "cols": a.cols, "grid": a.grid, "max_iter": a.iters,
                      "sequential_s": round(t_seq, 4), "batched_s": round(t_bat, 4),
                      "speedup": round(t_seq / t_bat, 2), "max_objective_diff": dobj,
                      "evals": [q["_solver"]["n_evals"] for q in bat]}))


if __name__ == "__main__":
    main()
