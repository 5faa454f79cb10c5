"""cProfile one headline fit on the GPU (host-side overhead hunting).

    python tools/fit_profile.py linear_regression [--rows 1000000 --cols 3000]
"""
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
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    dev = torch.device("cuda")
    wl = registry()[a.algo]
    Xh, yh = make_shard(wl.data, a.rows, a.cols, dev, 0, a.rows)
    df = DataFrame.from_numpy(Xh, yh if wl.label else None)
    est = wl.make_estimator()
    est.fit(df)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    est.fit(df)
    torch.cuda.synchronize()
    pr.disable()
    print("fit wall %.4f s" % (time.perf_counter() - t0))
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(a.top)
    print(s.getvalue())
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
