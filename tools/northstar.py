"""North-star configurations of BASELINE.json, measured through the public estimator API.

    python tools/northstar.py [--configs kmeans,logreg,rf,umap,pca] [--scale 1.0] [--out file.jsonl]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/northstar.py ...

Configs (BASELINE.json "configs"): PCA k=3 on 10k x 128; KMeans k=20 on 100M x 64; binary L2
LogisticRegression on 200M x 256; RandomForestClassifier 100 trees depth 16 on 50M x 64
(data-parallel histogram all-reduce); UMAP n_neighbors=15 d=2 on 20M x 128 (IVF kNN graph,
edge-parallel SGD). ``--scale`` multiplies every row count (a 1-GPU box cannot hold the
200M x 256 shard in pinned host memory next to its device copy). Rows are split over the
ranks (strong scaling); synthetic data generated on the device of each rank, handed to the
estimator as pinned host Arrow-backed DataFrames, so each timed fit includes H2D ingest.
One JSON line per config on rank 0 (fit seconds = max over ranks).
"""
import argparse
import json
import os
import sys
import time
import traceback

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (rows, cols, generator)
    "pca": (10_000, 128, "low_rank"),
    # uniform rows: 20 blobs would converge exactly (zero centre shift) after 2 iterations, and the
    # tol-0 config exists to time all 20 Lloyd / centroid-all-reduce iterations
    "kmeans": (100_000_000, 64, "uniform"),
    "logreg": (200_000_000, 256, "classification"),
    "rf": (50_000_000, 64, "classification"),
    "umap": (20_000_000, 128, "blobs"),
    # the same fit on non-blob rows: the reference-faithful classification generator (2 clusters
    # per class with random covariances, redundant mixes, shuffled columns)
    "umap_cls": (20_000_000, 128, "classification"),
}


def _estimator(name: str, world: int):
    if name == "pca":
        from spark_rapids_ml_nai_amd.feature import PCA

        return PCA(k=3, inputCol="features")
    if name == "kmeans":
        from spark_rapids_ml_nai_amd.clustering import KMeans

        # tol 0 (-> float32 tiny, the reference's mapping): all maxIter Lloyd iterations run, so the
        # timed fit is the Lloyd / centroid-all-reduce loop this config exists to stress
        return KMeans(k=20, maxIter=20, tol=0.0, seed=1, featuresCol="features")
    if name == "logreg":
        from spark_rapids_ml_nai_amd.classification import LogisticRegression

        return LogisticRegression(regParam=1e-5, maxIter=100, tol=1e-6, standardization=False,
                                  featuresCol="features", labelCol="label")
    if name == "rf":
        from spark_rapids_ml_nai_amd.classification import RandomForestClassifier

        # data-parallel histogram mode (north-star config 4): every level's histograms are
        # all-reduced; SRML_NS_RF_MODE=ensemble gives the reference's tree-split ensemble instead
        return RandomForestClassifier(numTrees=100, maxDepth=16, maxBins=128, seed=1, featuresCol="features",
                                      labelCol="label", split_mode=os.environ.get("SRML_NS_RF_MODE", "data_parallel"))
    if name.startswith("umap"):
        from spark_rapids_ml_nai_amd.umap import UMAP

        return UMAP(n_neighbors=15, n_components=2, random_state=1, featuresCol="features")
    raise ValueError(name)


CHUNK_BYTES = 16 << 30  # device generation in row chunks of <= 16 GB straight into the pinned shard


def _shard(gen: str, m: int, n: int, device, rank: int):
    from spark_rapids_ml_nai_amd.bench import datagen

    seed = 7000 + rank
    y = None
    step = max(1, CHUNK_BYTES // (4 * n))
    if gen in ("blobs", "classification") and m > step and device.type == "cuda":
        # large shards (the 200M x 256 LogisticRegression): the generators' class centres / mixing
        # matrices come from fixed seeds, so chunks with their own row seeds draw from the same
        # distribution; the device never holds more than one chunk plus its temporaries
        Xh = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
        yh = np.empty(m, dtype=np.float64)
        for c, r0 in enumerate(range(0, m, step)):
            mc = min(step, m - r0)
            if gen == "blobs":
                Xc, yc = datagen.blobs(mc, n, device, seed=seed * 1000 + c, centers=20)
            else:
                Xc, yc = datagen.classification(mc, n, device, seed=seed * 1000 + c, n_informative=n // 2,
                                                n_redundant=n // 4)
            Xh[r0: r0 + mc].copy_(Xc)
            yh[r0: r0 + mc] = yc.cpu().numpy()
            del Xc, yc
        torch.cuda.empty_cache()
        return Xh.numpy(), (yh if gen == "classification" else None)
    if gen == "uniform" and m > step and device.type == "cuda":
        Xh = torch.empty((m, n), dtype=torch.float32, pin_memory=True)
        for c, r0 in enumerate(range(0, m, step)):
            mc = min(step, m - r0)
            Xh[r0: r0 + mc].copy_(datagen.uniform(mc, n, device, seed=seed * 1000 + c))
        torch.cuda.empty_cache()
        return Xh.numpy(), None
    if gen == "uniform":
        X = datagen.uniform(m, n, device, seed=seed)
    elif gen == "low_rank":
        X = datagen.low_rank_matrix(m, n, device, seed=seed)
    elif gen == "blobs":
        X, _ = datagen.blobs(m, n, device, seed=seed, centers=20)
    elif gen == "classification":
        X, y = datagen.classification(m, n, device, seed=seed, n_informative=n // 2, n_redundant=n // 4)
    else:
        raise ValueError(gen)
    Xh = datagen.to_pinned_numpy(X)
    yh = y.cpu().numpy().astype(np.float64) if y is not None else None
    del X, y
    if device.type == "cuda":
        torch.cuda.empty_cache()
    return Xh, yh


def trustworthiness(X: torch.Tensor, E: torch.Tensor, k: int = 15, chunk: int = 1024) -> float:
    """sklearn.manifold.trustworthiness on the device (exact ranks, chunked rows): 1 - 2 / (n k
    (2n - 3k - 1)) * sum_i sum_{j in kNN_E(i) \\ kNN_X(i)} (rank_X(i, j) - k)."""
    n = X.shape[0]
    X = X.float()
    E = E.float()
    xn = (X * X).sum(1)
    en = (E * E).sum(1)
    pen = 0.0
    ar = torch.arange(n, device=X.device)
    for r0 in range(0, n, chunk):
        r1 = min(n, r0 + chunk)
        dx = xn[r0:r1, None] + xn[None, :] - 2.0 * X[r0:r1] @ X.T
        de = en[r0:r1, None] + en[None, :] - 2.0 * E[r0:r1] @ E.T
        rows = ar[r0:r1]
        dx[torch.arange(r1 - r0), rows] = float("inf")  # self excluded (rank 0 in sklearn)
        de[torch.arange(r1 - r0), rows] = float("inf")
        order = torch.argsort(dx, 1)
        rank_x = torch.empty_like(order)
        rank_x.scatter_(1, order, ar.view(1, -1).expand(r1 - r0, -1) + 1)  # 1-based ranks
        nn_e = torch.topk(de, k, 1, largest=False).indices
        rk = rank_x.gather(1, nn_e)
        pen += float((rk - k).clamp_min(0).sum().item())
    return 1.0 - 2.0 / (n * k * (2.0 * n - 3.0 * k - 1.0)) * pen


def _umap_quality(model, Xh, device, sample: int = 20_000, small_fit: bool = True) -> dict:
    """Trustworthiness of the fitted embedding on a row sample, and of a UMAP fitted on that sample
    alone (the reference's "single-GPU" comparison, tests/test_umap.py:146,377: gap <= 0.15).
    Multi-rank jobs skip the sample fit: one rank fitting alone inside the job's process group
    would wait on collectives the other ranks never join."""
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.umap import UMAP

    n = Xh.shape[0]
    idx = np.sort(np.random.default_rng(0).choice(n, size=min(sample, n), replace=False))
    Xs = torch.from_numpy(np.ascontiguousarray(Xh[idx])).to(device)
    Es = torch.from_numpy(np.asarray(model.embedding_)[idx]).to(device)
    t_big = trustworthiness(Xs, Es)
    if not small_fit:
        return {"trust_sample": int(idx.size), "trustworthiness": round(t_big, 5)}
    small = UMAP(n_neighbors=15, n_components=2, random_state=1, featuresCol="features").fit(
        DataFrame.from_numpy(np.ascontiguousarray(Xh[idx])))
    t_small = trustworthiness(Xs, torch.from_numpy(np.asarray(small.embedding_)).to(device))
    return {"trust_sample": int(idx.size), "trustworthiness": round(t_big, 5),
            "trustworthiness_small_fit": round(t_small, 5), "trust_gap": round(t_small - t_big, 5)}


def _ivf_recall(Xh, device, sample: int = 2000, k: int = 15) -> dict:
    """Recall@15 of the all-points IVF graph the UMAP fit builds (same builder and defaults), over
    ALL fitted rows: a query sample's graph rows against their exact neighbours among all N rows."""
    from spark_rapids_ml_nai_amd.models.knn_graph import IVF_PROBE, IVF_QPROBES, knn_graph, knn_graph_ivf

    X = torch.from_numpy(Xh).to(device).float()
    n = X.shape[0]
    q = torch.from_numpy(np.sort(np.random.default_rng(1).choice(n, size=min(sample, n), replace=False))).to(device)
    _, gi = knn_graph_ivf(X, k, seed=1)
    gi = gi.index_select(0, q).cpu().numpy()
    _, ei = knn_graph(X.index_select(0, q), X, k)
    ei = ei.cpu().numpy()
    del X
    torch.cuda.empty_cache()
    hit = np.mean([len(set(a.tolist()) & set(b.tolist())) / float(k) for a, b in zip(gi, ei)])
    return {"ivf_recall_queries": int(q.numel()), "ivf_recall_at_15": round(float(hit), 5),
            "ivf_probe": IVF_PROBE, "ivf_qprobes": IVF_QPROBES}


def main() -> None:
    if os.environ.get("SRML_NS_STACKDUMP"):  # periodic all-thread stacks (diagnosing a stuck rank)
        import faulthandler

        faulthandler.dump_traceback_later(int(os.environ["SRML_NS_STACKDUMP"]), repeat=True)
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="pca,kmeans,logreg,rf,umap")
    ap.add_argument("--scale", type=float, default=1.0)
    ap.add_argument("--warmup", type=int, default=0)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available()
    ndev = torch.cuda.device_count() if use_gpu else 0
    device = torch.device("cuda", local_rank % max(1, ndev)) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    if world > 1:
        from datetime import timedelta

        # SRML_NS_BACKEND=gloo: several ranks sharing ONE GPU (the development box), so the
        # multi-rank paths (data-parallel RF histogram all-reduce, ...) run and are timed there
        backend = os.environ.get("SRML_NS_BACKEND", "nccl" if use_gpu else "gloo")
        dist.init_process_group(backend, timeout=timedelta(minutes=30),
                                **({"device_id": device} if use_gpu and backend == "nccl" else {}))
    from spark_rapids_ml_nai_amd import DataFrame

    for name in a.configs.split(","):
        rows, cols, gen = CONFIGS[name]
        rows = max(1000, int(rows * a.scale)) if name != "pca" else rows
        b = np.linspace(0, rows, world + 1).astype(np.int64)
        m_local = int(b[rank + 1] - b[rank])
        rec = {"config": name, "rows": rows, "cols": cols, "n_gpus": world, "scale": a.scale,
               "backend": dist.get_backend() if world > 1 else None, "devices": ndev}
        try:
            t0 = time.perf_counter()
            Xh, yh = _shard(gen, m_local, cols, device, rank)
            rec["gen_s"] = round(time.perf_counter() - t0, 3)
            df = DataFrame.from_numpy(Xh, yh)
            est = _estimator(name, world)
            est.num_workers = world
            for _ in range(a.warmup):
                est.fit(df)
            if use_gpu:
                torch.cuda.synchronize()
            if world > 1:
                dist.barrier()
            t0 = time.perf_counter()
            model = est.fit(df)
            if use_gpu:
                torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([dt], dtype=torch.float64, device=device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dt = float(t.item())
            rec["fit_s"] = round(dt, 3)
            rec["rows_per_s"] = round(rows / dt, 1)
            ma = getattr(model, "_model_attributes", {}) or {}
            rec["phases"] = {k: round(v, 4) for k, v in getattr(model, "_fit_timings", {}).items()}
            rs = getattr(model, "_rank_stats", None)
            if rs:
                rec["ranks"] = rs
            if name == "kmeans":
                rec["iters"] = int(ma.get("n_iter", getattr(model, "num_iters", -1)) or -1)
                ph = ma.get("phase_s")
                if ph:
                    rec["phase_s"] = {"prep": ph[0], "init": ph[1], "lloyd": ph[2]}
                    rec["lloyd_s_per_iter"] = round(ph[2] / max(1, rec["iters"]), 5)
            if name == "logreg":
                rec["iters"] = int(getattr(model, "num_iters", -1))
            if name == "rf":
                rec["total_nodes"] = int(model.totalNumNodes)
                rec["split_mode"] = os.environ.get("SRML_NS_RF_MODE", "data_parallel")
                if rank == 0:  # held-out accuracy: fresh rows of the same family
                    Xq, yq = _shard(gen, 200_000, cols, device, 10_000 + rank)
                    pred = model.transform(DataFrame.from_numpy(Xq, yq)).to_numpy("prediction")
                    rec["holdout_accuracy"] = round(float((pred == yq).mean()), 5)
                    del Xq, yq
            if name.startswith("umap"):
                emb = np.asarray(model.embedding_)
                rec["finite"] = bool(np.isfinite(emb).all())
                from spark_rapids_ml_nai_amd.models import umap as _U

                # this rank's per-phase rows / seconds of the timed fit (before the quality fit)
                rec["umap_phases"] = json.loads(json.dumps(_U.LAST_PHASES))
                if rank == 0:
                    rec.update(_umap_quality(model, Xh, device, small_fit=world == 1))
                    rec.update(_ivf_recall(Xh, device))
            del model, df, Xh, yh
        except Exception as e:  # noqa: BLE001
            rec["error"] = repr(e)[:500]
            print("rank %d failed:" % rank, flush=True)
            traceback.print_exc()
        if use_gpu:
            torch.cuda.empty_cache()
        if rank == 0:
            line = json.dumps(rec)
            print(line, flush=True)
            if a.out:
                with open(a.out, "a") as f:
                    f.write(line + "\n")
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
