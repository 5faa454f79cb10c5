"""First-use H2D of a large pinned buffer: torch copy of a from_numpy tensor vs a direct
hipMemcpyAsync (srml_memcpy_h2d_async) on the same pointer."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch  # noqa: E402

from spark_rapids_ml_nai_amd.ops import native  # noqa: E402

dev = torch.device("cuda")
gb = float(sys.argv[1]) if len(sys.argv) > 1 else 100.0
mode = sys.argv[2] if len(sys.argv) > 2 else "native"
n = 256
m = int(gb * 1e9 / (4 * n))
h = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
X = h.numpy()
out = torch.empty((m, n), dtype=torch.float32, device=dev)
torch.cuda.synchronize()
for i in range(2):
    t0 = time.perf_counter()
    if mode == "native":
        native.call("srml_memcpy_h2d_async", out.data_ptr(), X.ctypes.data, m * n * 4, native.stream(dev))
    else:
        out.copy_(torch.from_numpy(X), non_blocking=True)
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("%s use %d: call %.2f s total %.2f s %.1f GB/s" % (mode, i, t1 - t0, t2 - t0, gb / (t2 - t0)), flush=True)
