"""Phase breakdown of one UMAP fit (north-star shape at a scale): cProfile of the host side with
device synchronisation at phase boundaries.

    python tools/umap_phases.py [--rows 2000000] [--cols 128]
"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--cols", type=int, default=128)
    ap.add_argument("--no-profile", action="store_true", help="skip cProfile (kernel-trace runs)")
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models import umap as U

    dev = torch.device("cuda", 0)
    X, _ = datagen.blobs(a.rows, a.cols, dev, seed=7000, centers=20)
    torch.cuda.synchronize()
    params = {"n_neighbors": 15, "n_components": 2, "random_state": 1}
    U.umap_fit(X[:20000].contiguous(), params)  # warm up kernels / libraries
    torch.cuda.synchronize()
    time.sleep(1.5)  # an idle marker before the timed fit (tools/trace_summary.py TRACE_AFTER_GAP_MS)
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    if not a.no_profile:
        pr.enable()
    U.umap_fit(X, params)
    torch.cuda.synchronize()
    if not a.no_profile:
        pr.disable()
    print("fit %.3f s" % (time.perf_counter() - t0), flush=True)
    print("phases", U.LAST_PHASES, flush=True)
    if not a.no_profile:
        pstats.Stats(pr).sort_stats("cumulative").print_stats(35)


if __name__ == "__main__":
    main()
