"""cProfile of one north-star fit (host-side time between kernels).
python tools/fit_host_profile.py --config logreg --scale 0.5"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
import northstar as ns  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="logreg")
ap.add_argument("--scale", type=float, default=0.5)
a = ap.parse_args()
rows, cols, gen = ns.CONFIGS[a.config]
rows = int(rows * a.scale)
dev = torch.device("cuda")
Xh, yh = ns._shard(gen, rows, cols, dev, 0)
df = DataFrame.from_numpy(Xh, yh)
est = ns._estimator(a.config, 1)
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
est.fit(df)
torch.cuda.synchronize()
pr.disable()
print("fit %.3f s" % (time.perf_counter() - t0))
pstats.Stats(pr).sort_stats("cumulative").print_stats(30)
