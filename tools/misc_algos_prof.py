"""Fit / query the secondary estimators once at moderate sizes (for rocprofv3 --stats passes):
DBSCAN 50k x 32 blobs, exact kNN 200k items x 20k queries x 128, IVF-Flat ANN same shapes."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from sklearn.datasets import make_blobs
from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.clustering import DBSCAN
from spark_rapids_ml_nai_amd.knn import ApproximateNearestNeighbors, NearestNeighbors


def t(label, fn):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter(); fn(); torch.cuda.synchronize()
    print(f"{label}: {time.perf_counter() - t0:.3f} s", flush=True)


Xd, _ = make_blobs(50_000, 32, centers=20, cluster_std=1.0, random_state=0)
dfd = DataFrame.from_numpy(Xd.astype(np.float32))
t("dbscan 50k x 32", lambda: DBSCAN(eps=3.0, min_samples=10).fit(dfd).transform(dfd).to_numpy("prediction"))
Xi, _ = make_blobs(200_000, 128, centers=50, random_state=1)
Xq = Xi[:20_000] + 0.01
dfi, dfq = DataFrame.from_numpy(Xi.astype(np.float32)), DataFrame.from_numpy(Xq.astype(np.float32))
t("knn exact 200k x 20k x 128 k=10", lambda: NearestNeighbors(k=10, inputCol="features").fit(dfi).kneighbors(dfq))
t("ann ivfflat 200k x 20k x 128 k=10", lambda: ApproximateNearestNeighbors(k=10, inputCol="features",
  algoParams={"nlist": 256, "nprobe": 16}).fit(dfi).kneighbors(dfq))
