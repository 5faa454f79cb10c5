"""Which step makes a 100 GB pinned H2D slow: raw tensor, numpy view, Arrow view (read-only)?"""
import os
import sys
import time
import warnings

sys.path.insert(0, os.getcwd())
import numpy as np  # noqa: E402
import torch  # noqa: E402

from spark_rapids_ml_nai_amd import DataFrame  # noqa: E402
from spark_rapids_ml_nai_amd.core.dataframe import array_column_to_dense  # noqa: E402

warnings.simplefilter("ignore")
dev = torch.device("cuda")
gb = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
n = 256
m = int(gb * 1e9 / (4 * n))
h = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
X = h.numpy()
Xa = array_column_to_dense(DataFrame.from_numpy(X).partitions[0].column("features"))
print("writeable:", X.flags["WRITEABLE"], Xa.flags["WRITEABLE"], "same ptr:", X.ctypes.data == Xa.ctypes.data,
      flush=True)


def run(name, t):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d = t.to(dev, non_blocking=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%-28s pinned=%s  call %.2f s  total %.2f s  %.1f GB/s" % (name, t.is_pinned(), t1 - t0, t2 - t0,
                                                                    gb / (t2 - t0)), flush=True)
    del d
    torch.cuda.empty_cache()


run("warmup torch pinned", h)
run("torch pinned", h)
run("from_numpy(numpy view)", torch.from_numpy(X))
run("from_numpy(arrow view)", torch.from_numpy(Xa))
run("torch pinned again", h)
