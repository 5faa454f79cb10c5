"""Microbench of the fused small-k Lloyd step at 10M x 64 (fp32): with sums (k = 20) and the
search alone (k = 20, 41), against the MFMA search (SRML_KMEANS_SMALL=0). Prints ms per call."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from spark_rapids_ml_nai_amd import ops  # noqa: E402

dev = torch.device("cuda:0")
m, n = 10_000_000, 64
X = torch.rand(m, n, device=dev)
tag = "mfma" if os.environ.get("SRML_KMEANS_SMALL") == "0" else "small"


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


for k in (20, 41):
    C = torch.rand(k, n, device=dev)
    if k <= 32 and tag != "mfma":
        print("%-6s k=%d fused step  %.3f ms" % (tag, k, timeit(lambda: ops.kmeans_lloyd_small(X, C))))
    print("%-6s k=%d search only %.3f ms" % (tag, k, timeit(lambda: ops.nearest_centroid(X, C))))
