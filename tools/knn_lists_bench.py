"""IVF all-points kNN tile kernel alone (fp16 centred), for PMC passes:

    python tools/knn_lists_bench.py [--rows 4000000] [--mode f16|f32]
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=4_000_000)
    ap.add_argument("--cols", type=int, default=128)
    ap.add_argument("--k", type=int, default=19)
    ap.add_argument("--mode", default="f16")
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models import knn_graph as KG

    dev = torch.device("cuda", 0)
    X, _ = datagen.blobs(a.rows, a.cols, dev, seed=7000, centers=20)
    N = X.shape[0]
    nlist = max(1, int(round(N / KG.IVF_LIST_ROWS)))
    C = KG.train_quantizer(X, nlist, 0)
    lab = ops.nearest_list(X, C, ops.quantizer_planes(X) if nlist > 256 else None)
    order, off, _ = ops.label_sort(lab, nlist)
    counts = off[1:] - off[:-1]
    Xs = X.index_select(0, order.long()).contiguous()
    del X
    xn = ops.row_sqnorm(Xs)
    cn = torch.where(counts > 0, ops.row_sqnorm(C), torch.full((nlist,), float("inf"), device=dev))
    _, probes = ops.knn(C, C, KG.IVF_NPROBE, inorm=cn, qnorm=torch.zeros(nlist, device=dev))
    probes = torch.where((probes >= 0) & torch.isfinite(cn[probes.clamp_min(0)]), probes, torch.full_like(probes, -1))
    tq, tl = KG.ivf_tiles(counts, off)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ops.knn_lists(Xs, xn, off, probes.int(), tq, tl, a.k, centroids=C if a.mode == "f16" else None)
        torch.cuda.synchronize()
        print("%s knn_lists %.4f s" % (a.mode, time.perf_counter() - t0), flush=True)


if __name__ == "__main__":
    main()
