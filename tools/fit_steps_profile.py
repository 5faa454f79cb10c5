"""cProfile each of several back-to-back fits of one headline workload (host-side view of
step-to-step variance). python tools/fit_steps_profile.py linear_regression --steps 3"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.bench.suite import make_shard, registry


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("algo")
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=3000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--top", type=int, default=12)
    a = ap.parse_args()
    dev = torch.device("cuda")
    wl = registry()[a.algo]
    Xh, yh = make_shard(wl.data, a.rows, a.cols, dev, 0, a.rows)
    df = DataFrame.from_numpy(Xh, yh if wl.label else None)
    est = wl.make_estimator()
    est.fit(df)
    torch.cuda.synchronize()
    model = None
    for s in range(a.steps):
        pr = cProfile.Profile()
        t0 = time.perf_counter()
        pr.enable()
        model = est.fit(df)
        pr.disable()
        torch.cuda.synchronize()
        print(f"step {s}: {time.perf_counter() - t0:.4f} s")
        out = io.StringIO()
        pstats.Stats(pr, stream=out).sort_stats("tottime").print_stats(a.top)
        print("\n".join(l[:160] for l in out.getvalue().splitlines()[6:6 + a.top + 2]))


if __name__ == "__main__":
    main()
