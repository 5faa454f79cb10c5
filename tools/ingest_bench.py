"""Host -> device ingest of a Spark-like batch stream (pageable Arrow buffers of N-row batches).

    python tools/ingest_bench.py [--rows 1000000 --cols 3000 --batch 20000]

Modes: ``pinned`` (one page-locked buffer: the headline bench's input), ``staged`` (threaded
pageable -> pinned ring -> DMA, ops/ingest.py), ``register`` (hipHostRegister each batch buffer in
place, DMA, unregister). Prints GB/s per mode.
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=3000)
    ap.add_argument("--batch", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd.ops import ingest

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rng = np.random.default_rng(0)
    parts = [rng.random((min(a.batch, a.rows - r), a.cols), dtype=np.float32) for r in range(0, a.rows, a.batch)]
    nbytes = sum(p.nbytes for p in parts)
    pinned = torch.empty((a.rows, a.cols), dtype=torch.float32, pin_memory=True)
    off = 0
    for p in parts:
        pinned[off: off + p.shape[0]].numpy()[:] = p
        off += p.shape[0]

    def run(name, fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            t0 = time.perf_counter()
            out = fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            del out
        t = min(ts)
        print(f"{name:10s} {t * 1e3:8.1f} ms  {nbytes / t / 1e9:6.1f} GB/s", flush=True)

    run("pinned", lambda: pinned.to(dev, non_blocking=True))
    for th in (1, 4, 8, 16):
        os.environ["SRML_INGEST_THREADS"] = str(th)
        run(f"staged{th}", lambda: ingest.parts_to_device(parts, dev, torch.float32))
    run("register", lambda: ingest.parts_to_device(parts, dev, torch.float32, mode="register"))


if __name__ == "__main__":
    main()
