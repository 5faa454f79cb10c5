"""Micro-benchmark of the hot HIP kernels at the headline shapes (1M x 3000 fp32)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from spark_rapids_ml_nai_amd import ops


def timeit(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1_000_000)
    ap.add_argument("--n", type=int, default=3000)
    ap.add_argument("--k", type=int, default=1000)
    ap.add_argument("--q", type=int, default=10000)
    ap.add_argument("--only", type=str, default="")
    a = ap.parse_args()
    dev = torch.device("cuda")
    g = torch.Generator(device=dev).manual_seed(0)
    X = torch.randn(a.m, a.n, device=dev, generator=g)
    res = {}
    gb = a.m * a.n * 4 / 1e9
    sel = set(a.only.split(",")) if a.only else None

    def want(name):
        return sel is None or name in sel

    if want("col_moments"):
        t = timeit(lambda: ops.col_moments(X))
        res["col_moments"] = {"ms": t, "TB/s": gb / t}
    if want("gram"):
        mu = X.mean(0).double()
        t = timeit(lambda: ops.gram(X, mu), 3)
        res["gram"] = {"ms": t, "TFLOP/s(sym)": a.m * a.n * a.n / t / 1e9}
    if want("xtv"):
        y = torch.randn(a.m, device=dev)
        t = timeit(lambda: ops.xtv(X, y))
        res["xtv"] = {"ms": t, "TB/s": gb / t}
    if want("logreg"):
        y = (torch.rand(a.m, device=dev) > 0.5).float()
        w = torch.randn(a.n, device=dev, dtype=torch.float64) * 0.01
        t = timeit(lambda: ops.logreg_binary_loss_grad(X, y, w, 0.1))
        res["logreg"] = {"ms": t, "TB/s": gb / t}
    if want("xw"):
        W = torch.randn(a.n, 3, device=dev)
        t = timeit(lambda: ops.xw(X, W))
        res["xw_k3"] = {"ms": t, "TB/s": gb / t}
    if want("nearest"):
        C = torch.randn(a.k, a.n, device=dev, generator=g)
        xn = ops.row_sqnorm(X)
        t = timeit(lambda: ops.nearest_centroid(X, C, xn), 3)
        res["nearest_centroid"] = {"ms": t, "TFLOP/s": 2 * a.m * a.k * a.n / t / 1e9}
    if want("nearest_split"):
        C = torch.randn(a.k, a.n, device=dev, generator=g)
        xn = ops.row_sqnorm(X)
        tiled = os.environ.get("SRML_SPLIT_TILED", "1") == "1"
        t0 = timeit(lambda: ops.split_bf16x3(X, tiled=tiled), 2)
        P = ops.split_bf16x3(X, tiled=tiled)
        t = timeit(lambda: ops.nearest_centroid_split(P, a.m, C, xn), 3)
        res["nearest_centroid_split"] = {"ms": t, "split_X_ms": t0,
                                         "TFLOP/s(fp32-equiv)": 2 * a.m * a.k * a.n / t / 1e9,
                                         "TFLOP/s(bf16 issued)": 12 * a.m * a.k * a.n / t / 1e9}
        del P
    if want("nearest_certified"):  # the Lloyd search: centred planes, certified 3-product pass
        C = torch.randn(a.k, a.n, device=dev, generator=g) * 0.05 + X[:1]
        mu = X.double().mean(0).float()
        xn = ops.row_sqnorm(X, mu)
        P = ops.split_bf16x3(X, tiled=True, mu=mu)
        t = timeit(lambda: ops.nearest_centroid_split(P, a.m, C, xn, X=X, mu=mu), 3)
        st = ops._CERTIFY_STATS
        res["nearest_centroid_certified"] = {"ms": t, "refined_frac": st["refined"] / max(1, st["rows"]),
                                             "TFLOP/s(bf16 issued)": 6 * a.m * a.k * a.n / t / 1e9}
        del P
    if want("nearest_f16"):  # the Lloyd search on the fp16 certified filter (one product)
        C = X[torch.randperm(a.m, device=dev, generator=g)[: a.k]].clone()  # random-row centres
        mu = X.double().mean(0).float()
        F = ops.F16Planes(X, mu)
        st0 = dict(ops._CERTIFY_STATS)
        t = timeit(lambda: ops.nearest_centroid_f16(F, C), 3)
        st = ops._CERTIFY_STATS
        res["nearest_centroid_f16"] = {"ms": t, "refined_frac": (st["refined"] - st0["refined"]) /
                                       max(1, st["rows"] - st0["rows"]),
                                       "TFLOP/s(f16 issued)": 2 * a.m * a.k * a.n / t / 1e9}
        del F
    if want("hgemm"):  # library fp16 GEMM of the filter's shape (rows x centres x 3008): attainable MFMA rate
        A = X[:, :].half()
        kp = 3008 if a.n == 3000 else a.n
        A = torch.nn.functional.pad(A, (0, kp - a.n))
        B = A[torch.randperm(a.m, device=dev, generator=g)[: a.k]].clone()
        t = timeit(lambda: torch.mm(A, B.T), 3)
        res["hgemm_f16_out_f16"] = {"ms": t, "TFLOP/s": 2 * a.m * a.k * kp / t / 1e9}
        B2 = B[:, :].contiguous()
        t = timeit(lambda: torch.mm(B2, A.T), 3)
        res["hgemm_f16_transposed"] = {"ms": t, "TFLOP/s": 2 * a.m * a.k * kp / t / 1e9}
        del A, B, B2
    if want("kpp"):  # greedy k-means++ over the k-means|| candidates (one block, k sequential steps)
        for nc in (4001, 8000):
            gk = torch.Generator().manual_seed(nc)
            Cc = torch.randn(nc, 32, generator=gk, dtype=torch.float64)
            G = (Cc @ Cc.T).to(dev)
            w = torch.randint(1, 50, (nc,), generator=gk).double().to(dev)
            t = timeit(lambda: ops.kmeanspp_gram(G, w, a.k, 1234), 3)
            res[f"kmeanspp_gram_nc{nc}"] = {"ms": t, "us_per_centre": 1e3 * t / a.k}
    if want("sums"):
        lab = torch.randint(0, a.k, (a.m,), device=dev, dtype=torch.int32)
        t = timeit(lambda: ops.cluster_sums(X, lab, a.k), 3)
        res["cluster_sums"] = {"ms": t, "TB/s": gb / t}
    if want("rowsq"):
        t = timeit(lambda: ops.row_sqnorm(X))
        res["row_sqnorm"] = {"ms": t, "TB/s": gb / t}
    if want("h2d"):
        h = torch.empty(a.m, a.n, pin_memory=True)
        t = timeit(lambda: h.to(dev, non_blocking=True), 3)
        res["h2d_pinned"] = {"ms": t, "GB/s": gb / t * 1000}
    if want("knn"):
        Q = X[: a.q].clone()
        xn = ops.row_sqnorm(X)
        t = timeit(lambda: ops.knn(Q, X, 10, inorm=xn), 3)
        res["knn_k10"] = {"ms": t, "TFLOP/s": 2 * a.q * a.m * a.n / t / 1e9}
    if want("ivf"):
        from spark_rapids_ml_nai_amd.models.knn import build_ivf

        ids = torch.arange(a.m, device=dev)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        index = build_ivf(X, ids, 1024, seed=1, iters=10)
        torch.cuda.synchronize()
        res["ivf_build_nlist1024"] = {"ms": (time.perf_counter() - t0) * 1e3}
        Q = X[: a.q].clone()
        qn = ops.row_sqnorm(Q)

        def _search():
            _, probes = ops.knn(Q, index.centroids, 20, inorm=index.cnorm, qnorm=qn)
            return ops.ivf_search(Q, probes.int(), index.list_off, index.items, index.inorm, index.ids, 10, qnorm=qn)

        t = timeit(_search, 3)
        scanned = a.q * 20 * (a.m / 1024) * a.n * 4 / 1e9
        res["ivf_search_nprobe20"] = {"ms": t, "scan_TB/s": scanned / t}
    if want("dbscan"):
        from spark_rapids_ml_nai_amd.models.dbscan import dbscan_fit_predict
        from spark_rapids_ml_nai_amd.parallel.context import WorkerContext

        Nd, nd = 200_000, 64
        C = torch.randn(50, nd, device=dev, generator=g) * 8
        Xd = C[torch.randint(0, 50, (Nd,), device=dev, generator=g)] + torch.randn(Nd, nd, device=dev, generator=g)
        xn = ops.row_sqnorm(Xd)
        T = ops.dbscan_num_tiles(Nd)
        t = timeit(lambda: ops.dbscan_degree(Xd, xn, 100.0, 0, T), 2)
        res["dbscan_degree_200k_x64"] = {"ms": t, "TFLOP/s(sym)": Nd * Nd * nd / t / 1e9}
        ctx = WorkerContext.single(dev)
        t = timeit(lambda: dbscan_fit_predict(Xd, ctx, 10.0, 5), 2)
        res["dbscan_fit_200k_x64"] = {"ms": t}
    if want("umap"):
        # reference notebook config: blobs 100k x 3000, fit on a 50% sample (GPU 24.94 s there)
        from spark_rapids_ml_nai_amd.models.umap import umap_fit, umap_transform

        Nu, nu = 100_000, 3000
        C = torch.randn(10, nu, device=dev, generator=g) * 4
        Xu = C[torch.randint(0, 10, (Nu,), device=dev, generator=g)] + torch.randn(Nu, nu, device=dev, generator=g)
        Xs = Xu[torch.randperm(Nu, device=dev, generator=g)[: Nu // 2]].contiguous()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        emb = umap_fit(Xs, dict(n_neighbors=15, n_components=2, random_state=1))
        torch.cuda.synchronize()
        res["umap_fit_50k_x3000"] = {"ms": (time.perf_counter() - t0) * 1e3}
        t0 = time.perf_counter()
        umap_transform(Xu, Xs, torch.from_numpy(emb).to(dev), dict(n_neighbors=15, random_state=1))
        torch.cuda.synchronize()
        res["umap_transform_100k_x3000"] = {"ms": (time.perf_counter() - t0) * 1e3}
    if want("quantize"):  # RF binning of the whole shard: 127 quantile edges per feature
        e = torch.sort(torch.randn(a.n, 127, device=dev, generator=g), dim=1).values.contiguous()
        t = timeit(lambda: ops.rf_quantize(X, e), 3)
        res["rf_quantize"] = {"ms": t, "TB/s(read X)": gb / t}
    if want("rfhist"):
        # root level of a regression tree at the headline shape: in-bag rows x 1000 sampled features
        import numpy as np

        n_, m_ = a.n, a.m
        del X
        torch.cuda.empty_cache()
        bins = torch.randint(0, 128, (n_, m_), device=dev, dtype=torch.uint8, generator=g)
        w = torch.poisson(torch.ones(m_, device=dev), generator=g).clamp_max(255).to(torch.uint8)
        idx = torch.nonzero(w).view(-1).int()
        y = torch.randn(m_, device=dev, generator=g)
        nf = max(1, n_ // 3)
        feats = torch.randperm(n_, device=dev, generator=g)[:nf].int().view(1, -1).contiguous()
        rows = idx.shape[0]
        for reg, S, nm in ((True, 2, "rf_hist_reg_root"), (False, 3, "rf_hist_clf3_root")):
            fb = ops.rf_hist_fb(128, S, reg)
            nfc = (nf + fb - 1) // fb
            rpi = int(min(65536, max(4096, rows * nfc // 8192)))
            rpi = (rpi + 511) // 512 * 512
            it = []
            for r0 in range(0, rows, rpi):
                for fc in range(nfc):
                    it.append((0, r0, min(rows, r0 + rpi), fc))
            items = torch.tensor(np.array(it, dtype=np.int32), device=dev)
            yy = y if reg else torch.randint(0, 3, (m_,), device=dev, generator=g).float()
            t = timeit(lambda: ops.rf_hist(bins, idx, yy, w, items, feats, 1, 128, S, reg), 3)
            res[nm] = {"ms": t, "Gpairs/s": rows * nf / t / 1e6}
    print(json.dumps({k: {kk: round(vv, 3) for kk, vv in v.items()} for k, v in res.items()}))


if __name__ == "__main__":
    main()
