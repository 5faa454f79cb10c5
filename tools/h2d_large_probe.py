"""H2D of a large pinned shard through the package's ingest (is it DMA'd at PCIe rate?).
python tools/h2d_large_probe.py --gb 100"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spark_rapids_ml_nai_amd.ops import ingest  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--gb", type=float, default=100.0)
a = ap.parse_args()
dev = torch.device("cuda")
n = 256
m = int(a.gb * 1e9 / (4 * n))
t0 = time.perf_counter()
h = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
print("pinned alloc %.2f s" % (time.perf_counter() - t0), "is_pinned", h.is_pinned(), flush=True)
X = h.numpy()
print("numpy view pinned:", ingest.is_pinned(X), flush=True)
for _ in range(2):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = ingest.host_to_device(X, dev, torch.float32)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("host_to_device %.1f GB in %.2f s = %.1f GB/s" % (m * n * 4 / 1e9, dt, m * n * 4 / 1e9 / dt), flush=True)
    del d
    torch.cuda.empty_cache()

# the same shard through the Arrow-backed DataFrame (the estimators' route)
from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.core.dataframe import array_column_to_dense  # noqa: E402

t0 = time.perf_counter()
df = DataFrame.from_numpy(X)
print("from_numpy %.2f s" % (time.perf_counter() - t0), flush=True)
t0 = time.perf_counter()
tab = df.partitions[0] if hasattr(df, "partitions") else None
Xa = array_column_to_dense(tab.column("features")) if tab is not None else df.to_numpy("features")
print("arrow view %.2f s, same buffer: %s, pinned: %s, contiguous: %s" % (
    time.perf_counter() - t0, Xa.ctypes.data == X.ctypes.data, ingest.is_pinned(Xa), Xa.flags["C_CONTIGUOUS"]),
    flush=True)
torch.cuda.synchronize()
t0 = time.perf_counter()
d = ingest.host_to_device(Xa, dev, torch.float32)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print("arrow-route host_to_device %.1f GB/s" % (m * n * 4 / 1e9 / dt), flush=True)
