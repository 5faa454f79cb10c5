"""Where the LogisticRegression evaluations go: the bench's 1M x 3000 classification shard fitted
with maxIter = 5, 10, 20, ... (everything else as the bench): iterations, evaluations, objective
and solver status per cap, on the device solver and the fp64-evaluation path."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.bench.suite import make_shard  # noqa: E402
from spark_rapids_ml_nai_amd.classification import LogisticRegression  # noqa: E402

m = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
dev = torch.device("cuda:0")
Xh, yh = make_shard("classification", m, 3000, dev, 0, 1_000_000)
df = DataFrame.from_numpy(Xh, yh)
for f32 in (True, False):
    for cap in (5, 10, 20, 30, 40, 60, 200):
        est = LogisticRegression(standardization=False, maxIter=cap, tol=1e-30, regParam=1e-5, float32_inputs=f32)
        mdl = est.fit(df)
        info = getattr(mdl, "_solver_info", {}) or {}
        print(json.dumps({"rows": m, "float32_inputs": f32, "maxIter": cap, "iters": int(mdl.num_iters),
                          "objective": float(mdl.objective),
                          **{k: info.get(k) for k in ("n_evals", "n_margin_only", "status", "path")}}),
              flush=True)
