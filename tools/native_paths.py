"""The formerly host-looped / library-op device paths, run back to back for a
rocprofv3 kernel trace whose check lists every kernel that is neither an in-tree ``srml`` kernel
nor torch glue (fills / copies / elementwise casts / concatenation / indexing): sorts, top-k,
library GEMMs, sparse-library or reduction kernels would show up there.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/np -o np -- python3 tools/native_paths.py
    python tools/native_paths.py --check gpurun_out/np/.../np_kernel_stats.csv
"""
import argparse
import csv
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GLUE = ("elementwise", "fill", "Fill", "copy", "Copy", "CatArray", "index", "Index", "gather", "scatter",
        "arange", "distribution", "unrolled_elementwise", "vectorized", "__amd_rocclr")
LIBRARY = ("sort", "Sort", "topk", "TopK", "radix", "Cijk_", "rocblas", "hipblas", "gemm", "Gemm", "sparse",
           "Sparse", "reduce_kernel", "scan", "Scan", "bitonic", "cub", "cdist", "unique")
# --set r5 counts only library COMPUTE (GEMMs, sorts, top-k, sparse, unique, cdist, scans); torch's
# small-vector reductions (.all() / norms / sums), nonzero compaction (rocprim partition) and
# searchsorted are listed separately as glue
LIBRARY_R5 = ("sort", "Sort", "topk", "TopK", "Cijk_", "rocblas", "hipblas", "gemm", "Gemm", "sparse", "Sparse",
              "bitonic", "cdist", "unique", "scan_kernel", "ScanOp", "cumsum")


def run_r5() -> None:
    """Round-5 set: fp64 multinomial LogReg (K = 3 and the wide K = 20),
    DBSCAN (label compaction), supervised UMAP on the device spectral path (categorical
    intersection, sorted spectral input), the min-norm solve of singular normal equations past
    n = 4096, and a k > 64 kNN on 1500-dimensional rows (refine-sort beyond 1024 columns)."""
    import numpy as np
    import torch

    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.classification import LogisticRegression
    from spark_rapids_ml_nai_amd.clustering import DBSCAN
    from spark_rapids_ml_nai_amd.knn import NearestNeighbors
    from spark_rapids_ml_nai_amd.models import linear
    from spark_rapids_ml_nai_amd.umap import UMAP

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(5)
    steps = []
    Xf = rng.standard_normal((20000, 300))
    for K in (3, 20):
        yk = rng.integers(0, K, 20000).astype(np.float64)
        steps.append(("logreg_f64_multinomial_k%d" % K, lambda yk=yk: LogisticRegression(
            maxIter=10, regParam=1e-3, float32_inputs=False).fit(DataFrame.from_numpy(Xf, yk))))
    Xd = np.concatenate([rng.standard_normal((2000, 16)) * 0.05 + c for c in rng.standard_normal((10, 16)) * 3])
    steps.append(("dbscan", lambda: DBSCAN(eps=0.5, min_samples=5, featuresCol="features").fit(
        DataFrame.from_numpy(Xd.astype(np.float32))).transform(DataFrame.from_numpy(Xd.astype(np.float32)))))
    Xu = np.concatenate([rng.standard_normal((1000, 32)) + c for c in rng.standard_normal((5, 32)) * 4])
    yu = np.repeat(np.arange(5), 1000).astype(np.float64)
    yu[::7] = -1.0
    steps.append(("umap_supervised", lambda: UMAP(n_neighbors=15, random_state=1, featuresCol="features",
                                                   labelCol="label").fit(DataFrame.from_numpy(Xu.astype(np.float32), yu))))
    # the singular normal equations are formed on the host: the trace should show the solve only
    Xs = rng.standard_normal((6000, 4000))
    Xs = np.concatenate([Xs, 2.0 * Xs[:, :300]], 1)
    A = torch.from_numpy(Xs.T @ Xs / 6000.0).to(dev)
    bs = torch.from_numpy(Xs.T @ rng.standard_normal(6000) / 6000.0).to(dev)
    steps.append(("min_norm_n4300", lambda: linear._min_norm_solve(A, bs)))
    Xk = rng.standard_normal((20000, 1500)).astype(np.float32)
    steps.append(("knn_k100_n1500", lambda: NearestNeighbors(k=100, inputCol="features").fit(
        DataFrame.from_numpy(Xk)).kneighbors(DataFrame.from_numpy(Xk[:300]))))
    for name, fn in steps:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        print("%-28s %.4f s" % (name, time.perf_counter() - t0), flush=True)


def run() -> None:
    import numpy as np
    import torch

    from spark_rapids_ml_nai_amd import DataFrame, ops
    from spark_rapids_ml_nai_amd.classification import LogisticRegression
    from spark_rapids_ml_nai_amd.knn import ApproximateNearestNeighbors, NearestNeighbors

    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(0)
    steps = []
    X = rng.standard_normal((30000, 784)).astype(np.float32)
    items = DataFrame.from_numpy(X)
    queries = DataFrame.from_numpy(X[:500])
    steps.append(("ivf_n784_k100", lambda: ApproximateNearestNeighbors(
        k=100, inputCol="features", algoParams={"nlist": 32, "nprobe": 4}).fit(items).kneighbors(queries)))
    Xs = rng.standard_normal((40000, 32)).astype(np.float32)
    steps.append(("knn_k2000", lambda: NearestNeighbors(k=2000, inputCol="features").fit(
        DataFrame.from_numpy(Xs)).kneighbors(DataFrame.from_numpy(Xs[:200]))))
    Xl = rng.standard_normal((400, 20000))
    yl = (Xl[:, 0] > 0).astype(np.float64)
    steps.append(("logreg_fp64_n20000", lambda: LogisticRegression(maxIter=10, regParam=1e-3,
                                                                   float32_inputs=False).fit(
        DataFrame.from_numpy(Xl, yl))))
    Xm = torch.randn(20000, 128, device=dev)
    ym = (torch.rand(20000, device=dev) > 0.5).float()
    WB = torch.randn(20, 129, dtype=torch.float64, device=dev) * 0.1
    steps.append(("logreg_multi_m20", lambda: ops.logistic_loss_grad_multi(
        Xm, ym, WB, torch.zeros(20, 130, dtype=torch.float64, device=dev))))
    import scipy.sparse as sp

    A = sp.random(20000, 500, density=0.02, random_state=1, format="csr", dtype=np.float32)
    yk = rng.integers(0, 20, 20000).astype(np.float64)
    steps.append(("csr_logreg_k20", lambda: LogisticRegression(maxIter=10, regParam=1e-3).fit(
        DataFrame.from_numpy(A, yk))))
    for name, fn in steps:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        print("%-20s %.4f s" % (name, time.perf_counter() - t0), flush=True)


def check(path: str, lib_terms: tuple = LIBRARY) -> int:
    lib, glue, srml = [], [], []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            nm = r["Name"]
            if "srml" in nm or any(t in nm for t in ("_kernel<", "_kernel(")) and "at::native" not in nm:
                srml.append(nm)
            elif any(t in nm for t in lib_terms) and "searchsorted" not in nm:
                lib.append((nm[:110], r["Calls"]))
            else:
                glue.append((nm[:110], r["Calls"]))
    print("in-tree kernels: %d, torch glue kernels: %d, library compute kernels: %d" % (len(srml), len(glue), len(lib)))
    for nm, c in lib:
        print("  LIBRARY %s x%s" % (nm, c))
    for nm, c in glue:
        print("  glue    %s x%s" % (nm, c))
    return 1 if lib else 0


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--check", default="")
    ap.add_argument("--set", default="r3", choices=("r3", "r5"))
    a = ap.parse_args()
    if a.check:
        sys.exit(check(a.check, LIBRARY_R5 if a.set == "r5" else LIBRARY))
    run_r5() if a.set == "r5" else run()
