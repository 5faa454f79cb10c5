"""Host-side (Python) profile of the per-rank random-forest fits (tools/rf_rank_proxy.py shapes):
where the level loop spends CPU time between kernels. python tools/rf_host_profile.py"""
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.bench.suite import make_shard  # noqa: E402
from spark_rapids_ml_nai_amd.classification import RandomForestClassifier  # noqa: E402
from spark_rapids_ml_nai_amd.regression import RandomForestRegressor  # noqa: E402

dev = torch.device("cuda")
for name, fam, mk in [("rfc7", "classification",
                       lambda: RandomForestClassifier(numTrees=7, maxBins=128, maxDepth=13, seed=1)),
                      ("rfr4", "regression", lambda: RandomForestRegressor(numTrees=4, maxBins=128, maxDepth=6, seed=1))]:
    Xh, yh = make_shard(fam, 125000, 3000, dev, 0, 1000000)
    df = DataFrame.from_numpy(Xh, yh)
    est = mk()
    est.fit(df)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    for _ in range(3):
        est.fit(df)
    torch.cuda.synchronize()
    pr.disable()
    print(name, "3 fits %.4f s" % (time.perf_counter() - t0))
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)
