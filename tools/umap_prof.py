import sys, os, time
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from sklearn.datasets import make_blobs
from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.umap import UMAP
X, _ = make_blobs(100_000, 3000, centers=10, cluster_std=1.0, random_state=0)
X = X.astype(np.float32)
df = DataFrame.from_numpy(X)
est = UMAP(n_neighbors=15, n_components=2, random_state=1, sample_fraction=0.5, featuresCol="features")
est.fit(df); torch.cuda.synchronize()
t0 = time.perf_counter(); m = est.fit(df); torch.cuda.synchronize(); print("fit", time.perf_counter() - t0)
t0 = time.perf_counter(); e = m.transform(df).to_numpy("embedding"); print("transform", time.perf_counter() - t0)
