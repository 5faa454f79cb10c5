"""Per-rank work of an N-GPU strong-scaling run of the headline suite, on ONE GPU: each workload is
fitted on rank 0's row shard (rows / N) with rank 0's share of the random-forest trees
(ceil(numTrees / N), reference tree.py:270-281 split), collectives excluded. Prints wall time per
fit (median of --reps) so fixed per-rank costs can be found before the driver's 8-GPU run.

    python tools/rank_proxy.py --world 8 [--algos all] [--reps 3]
"""
import argparse
import json
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.bench.suite import SPARK_CPU_S, make_shard, model_evidence, registry  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=3000)
    ap.add_argument("--algos", default="all")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    reg = registry()
    names = list(SPARK_CPU_S) if a.algos == "all" else a.algos.split(",")
    m_local = int(np.linspace(0, a.rows, a.world + 1).astype(np.int64)[1])
    out = {}
    for name in names:
        wl = reg[name]
        Xh, yh = make_shard(wl.data, m_local, a.cols, dev, 0, a.rows)
        df = DataFrame.from_numpy(Xh, yh if wl.label else None)
        est = wl.make_estimator()
        if name.startswith("random_forest"):
            est.setNumTrees(int(math.ceil(est.getNumTrees() / a.world)))
        est.fit(df)
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            model = est.fit(df)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name] = {"fit_s": round(float(np.median(ts)), 4), "evidence": model_evidence(name, model)}
        print(name, out[name], flush=True)
        del df, Xh, yh
        torch.cuda.empty_cache()
    print(json.dumps({"world": a.world, "rows_per_rank": m_local, "suite_s": round(sum(v["fit_s"] for v in out.values()), 4),
                      "workloads": out}))


if __name__ == "__main__":
    main()
