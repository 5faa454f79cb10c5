"""Where a KMeans transform's time goes at 1M x 3000 (one MI355X): the bench's pinned shard, a
short fit, then model.transform + count under cProfile next to a bare pinned H2D of the rows."""
import cProfile
import os
import io
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.bench.suite import make_shard
from spark_rapids_ml_nai_amd.clustering import KMeans

m = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
dev = torch.device("cuda:0")
Xh, _ = make_shard("uniform", m, 3000, dev, 0, m)
df = DataFrame.from_numpy(Xh, None)
model = KMeans(k=1000, maxIter=2, seed=1).fit(df)
t = torch.from_numpy(Xh)
for _ in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = t.to(dev, non_blocking=True)
    torch.cuda.synchronize()
    print("bare H2D %.4f s (%.1f GB/s)" % (time.perf_counter() - t0, t.numel() * 4 / (time.perf_counter() - t0) / 1e9))
    del d
for i in range(3):
    pr = cProfile.Profile() if i == 2 else None
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if pr:
        pr.enable()
    out = model.transform(df)
    n = out.count()
    if pr:
        pr.disable()
    print("transform %.4f s rows %d" % (time.perf_counter() - t0, n))
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
print(s.getvalue())
