import sys, time, os
sys.path.insert(0, os.getcwd())
import torch
from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.bench.suite import make_shard
from spark_rapids_ml_nai_amd.classification import RandomForestClassifier
from spark_rapids_ml_nai_amd.regression import RandomForestRegressor
dev = torch.device("cuda")
for name, fam, mk in [("rfc7", "classification",
                        lambda: RandomForestClassifier(numTrees=7, maxBins=128, maxDepth=13, seed=1)),
                      ("rfr4", "regression", lambda: RandomForestRegressor(numTrees=4, maxBins=128, maxDepth=6, seed=1))]:
    Xh, yh = make_shard(fam, 125000, 3000, dev, 0, 1000000)
    df = DataFrame.from_numpy(Xh, yh)
    est = mk()
    est.fit(df); torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter(); est.fit(df); torch.cuda.synchronize(); ts.append(time.perf_counter() - t0)
    print(name, [round(t, 4) for t in ts])
