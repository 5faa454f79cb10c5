"""Small-k Lloyd step at the BASELINE KMeans shape (100M x 64 fp32, k = 20) on one MI355X: ms per
fused step for the MFMA kernel (lloyd.hip: with per-row labels / distances, and without them as the
Lloyd loop runs it) and the VALU kernel, the HBM rate (X read once per
step), and the device-resident 20-iteration loop (step + update, no host sync). One JSON line."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spark_rapids_ml_nai_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
m = int(os.environ.get("ROWS", "100000000"))
n, k = 64, 20
g = torch.Generator(device=dev)
g.manual_seed(0)
X = torch.rand(m, n, device=dev, generator=g)
C = X[:k].clone()
out = {"rows": m, "cols": n, "k": k, "bytes_per_step": m * n * 4}


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


buf = torch.zeros(k * n + k + 1, dtype=torch.float64, device=dev)
lab = torch.empty(m, dtype=torch.int32, device=dev)
dist = torch.empty(m, dtype=torch.float32, device=dev)
for kern in ("mfma", "valu"):
    os.environ["SRML_LLOYD_KERNEL"] = kern
    ms = timeit(lambda: (buf.zero_(), ops.kmeans_lloyd_small(X, C, out=buf, labels=lab, dist=dist)))
    out[kern + "_step_ms"] = round(ms, 3)
    out[kern + "_TBps"] = round(m * n * 4 / ms / 1e9, 2)
    ms = timeit(lambda: ops.kmeans_lloyd_small(X, C, with_sums=False, labels=lab, dist=dist))
    out[kern + "_search_ms"] = round(ms, 3)
os.environ["SRML_LLOYD_KERNEL"] = "mfma"
ms = timeit(lambda: (buf.zero_(), ops.kmeans_lloyd_small(X, C, out=buf, rows_out=False)))
out["norows_step_ms"] = round(ms, 3)
out["norows_TBps"] = round(m * n * 4 / ms / 1e9, 2)
from spark_rapids_ml_nai_amd.models.kmeans import _lloyd_small_loop  # noqa: E402
from spark_rapids_ml_nai_amd.parallel.context import WorkerContext  # noqa: E402

ctx = WorkerContext.single(dev)
_lloyd_small_loop(X, C.double(), ctx, k, 2, 0.0)
torch.cuda.synchronize()
t = time.perf_counter()
_, it, inertia = _lloyd_small_loop(X, C.double(), ctx, k, 20, 0.0)
torch.cuda.synchronize()
dt = time.perf_counter() - t
out.update(loop_iters=it, loop_s=round(dt, 4), loop_ms_per_iter=round(dt / max(it, 1) * 1e3, 3), inertia=inertia)
print(json.dumps(out))
