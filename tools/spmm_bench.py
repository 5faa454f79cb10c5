"""CSR SpMM of the UMAP spectral init alone (normalised fuzzy graph of a 4M-row IVF kNN graph,
16 dense columns):

    python tools/spmm_bench.py [--rows 4000000] [--reps 20]
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
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--k", type=int, default=16)
    a = ap.parse_args()
    from spark_rapids_ml_nai_amd import ops
    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.core.base import CSR
    from spark_rapids_ml_nai_amd.models import umap as U
    from spark_rapids_ml_nai_amd.models.knn_graph import build_knn_graph

    dev = torch.device("cuda", 0)
    X, _ = datagen.blobs(a.rows, a.cols, dev, seed=7000, centers=20)
    dist, idx, order = build_knn_graph(X, 15, "ivf", None, 1, None, list_order=U.LIST_ORDER)
    del X
    _, _, w = ops.umap_smooth_knn(dist, idx, 15.0, local_connectivity=1.0, self_rows=True)
    rows, cols, vals = ops.umap_fuzzy_union_knn(idx, w, 1.0)
    n = dist.shape[0]
    r64 = rows.long()
    indptr = torch.searchsorted(r64.contiguous(), torch.arange(n + 1, device=dev, dtype=torch.int64))
    M = CSR(indptr=indptr, indices=cols.to(torch.int32).contiguous(), data=vals.float().contiguous(), shape=(n, n))
    Y = torch.randn(n, a.k, device=dev)
    print("rows %d nnz %d" % (n, rows.numel()), flush=True)
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            Z = ops.csr_spmm(M, Y)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / a.reps
        print("spmm %.3f ms (%.1f GB/s of index+value+W-row traffic)" % (
            1e3 * dt, (rows.numel() * (8 + 4 * a.k) + n * 4 * a.k) / dt / 1e9), flush=True)
    del Z


if __name__ == "__main__":
    main()
