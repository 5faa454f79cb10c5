"""Per-level host timing of one RandomForest fit at the bench shape (SRML_RF_LEVEL_LOG): for every
level, the segments / candidates / splits and the seconds spent building work items on the host,
launching, waiting for the split records, deciding splits and waiting for the child bounds."""
import json
import os
import sys
import time

os.environ["SRML_RF_LEVEL_LOG"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.bench.suite import make_shard, registry  # noqa: E402
from spark_rapids_ml_nai_amd.models import forest  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
name = sys.argv[2] if len(sys.argv) > 2 else "random_forest_classifier"
dev = torch.device("cuda", 0)
if name == "northstar_rf":  # BASELINE.json config 4 shape: 64 features, 100 trees, depth 16
    from spark_rapids_ml_nai_amd.classification import RandomForestClassifier

    Xh, yh = make_shard("classification", rows, 64, dev, 0, rows)
    est = RandomForestClassifier(numTrees=100, maxDepth=16, maxBins=128, seed=1, featuresCol="features",
                                 labelCol="label", split_mode="data_parallel")
else:
    wl = registry()[name]
    Xh, yh = make_shard(wl.data, rows, 3000, dev, 0, rows)
    est = wl.make_estimator()
df = DataFrame.from_numpy(Xh, yh)
est.fit(df)
torch.cuda.synchronize()
t0 = time.perf_counter()
est.fit(df)
torch.cuda.synchronize()
print(json.dumps({"workload": name, "rows": rows, "fit_s": round(time.perf_counter() - t0, 4)}))
keys = ["items_host", "hist_split_launch", "split_sync", "decide_host", "route_launch", "end_sync"]
tot = {k: 0.0 for k in keys}
for rec in forest.LAST_LEVELS:
    print(json.dumps(rec))
    for k in keys:
        tot[k] += rec.get(k, 0.0)
print(json.dumps({"total": {k: round(v, 4) for k, v in tot.items()}}))
