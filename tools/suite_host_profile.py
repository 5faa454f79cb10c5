"""Host-side profile of the bench suite's fits at a row count (default the 125k per-rank shard):
per workload, one warm-up fit, then a cProfile'd fit — wall time and the top host functions by
own time (where a fit waits on the device shows as synchronize / item / copy)."""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.bench.suite import make_shard, registry  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 125000
algos = sys.argv[2].split(",") if len(sys.argv) > 2 else None
dev = torch.device("cuda", 0)
reg = registry()
for name, wl in reg.items():
    if algos and name not in algos:
        continue
    Xh, yh = make_shard(wl.data, rows, 3000, dev, 0, rows)
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
    dt = time.perf_counter() - t0
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(12)
    lines = [ln for ln in s.getvalue().splitlines() if ln.strip() and ("/" in ln or "{" in ln)]
    print("=== %s fit %.4f s" % (name, dt))
    for ln in lines[:12]:
        print("   " + ln.strip()[:150])
    del df, Xh, yh
