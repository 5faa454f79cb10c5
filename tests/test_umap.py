"""UMAP (reference tests/test_umap.py): quality gate = trustworthiness (sklearn) — the reference
allows a gap <= 0.15 vs single-GPU cuML; umap-learn reaches ~0.98 on digits, we require >= 0.9."""
import warnings

import numpy as np
import pytest
from sklearn.datasets import load_digits, make_blobs
from sklearn.manifold import trustworthiness

from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.umap import UMAP, UMAPModel

warnings.filterwarnings("ignore")


def _digits(n=1200):
    X, y = load_digits(return_X_y=True)
    return X[:n].astype(np.float32), y[:n]


def test_params():
    u = UMAP()
    assert u.cuml_params["n_neighbors"] == 15 and u.cuml_params["n_components"] == 2
    assert u.getOutputCol() == "embedding"
    u2 = UMAP(n_neighbors=10, min_dist=0.2, random_state=3)
    assert u2.cuml_params["n_neighbors"] == 10 and u2.cuml_params["min_dist"] == 0.2
    assert u2.cuml_params["random_state"] == 3


def test_find_ab_params():
    from spark_rapids_ml_nai_amd.models.umap import find_ab_params

    a, b = find_ab_params(1.0, 0.1)
    assert abs(a - 1.577) < 0.01 and abs(b - 0.895) < 0.01


@pytest.mark.parametrize("init", ["spectral", "random"])
def test_umap_fit_transform_trustworthiness(init, tmp_path):
    X, y = _digits()
    df = DataFrame.from_numpy(X, num_partitions=2)
    model = UMAP(n_neighbors=15, random_state=1, init=init).setFeaturesCol("features").fit(df)
    emb = np.asarray(model.embedding)
    assert emb.shape == (len(X), 2)
    assert trustworthiness(X, emb, n_neighbors=15) > 0.9
    out = model.transform(df)
    assert out.columns == ["features", "embedding"]
    e2 = out.to_numpy("embedding")
    assert e2.shape == (len(X), 2) and np.isfinite(e2).all()
    assert trustworthiness(X, e2, n_neighbors=15) > 0.85
    # persistence (npy side files)
    path = str(tmp_path / "umap")
    model.write().overwrite().save(path)
    m2 = UMAPModel.load(path)
    assert np.allclose(m2.embedding_, model.embedding_)
    assert np.allclose(m2.raw_data_, model.raw_data_)
    assert m2.getOrDefault("n_neighbors") == 15


def test_umap_supervised_separates_classes():
    X, y = make_blobs(800, 10, centers=4, cluster_std=4.0, random_state=0)
    X = X.astype(np.float32)
    df = DataFrame.from_numpy(X, y.astype(np.float64))
    model = UMAP(random_state=2, labelCol="label").fit(df)
    emb = model.embedding_
    cent = np.stack([emb[y == c].mean(0) for c in range(4)])
    within = np.mean([np.linalg.norm(emb[y == c] - cent[c], axis=1).mean() for c in range(4)])
    between = np.mean([np.linalg.norm(cent[i] - cent[j]) for i in range(4) for j in range(i + 1, 4)])
    assert between > 2 * within


def test_umap_sample_fraction_and_cosine():
    X, _ = _digits(800)
    df = DataFrame.from_numpy(X)
    model = UMAP(sample_fraction=0.5, metric="cosine", random_state=4, n_components=3).fit(df)
    assert 300 < model.embedding_.shape[0] < 500
    assert model.embedding_.shape[1] == 3
    out = model.transform(df).to_numpy("embedding")
    assert out.shape == (800, 3)


def test_query_probing_and_nn_descent_recall():
    """Per-query IVF probing beats list probing at the same probe count on rows whose neighbours
    straddle lists, and build_algo='nn_descent' (the per-query graph + NN-descent rounds) raises
    the recall further; the graphs stay sorted, exact and duplicate-free."""
    import torch

    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.models.knn_graph import build_knn_graph, knn_graph_brute

    X, _ = datagen.classification(12000, 32, torch.device("cpu"), seed=3, n_informative=12, n_redundant=8)
    X = X.float().contiguous()
    _, ie = knn_graph_brute(X, 10)

    def rec(idx):
        return np.mean([len(set(a) & set(b)) / 10.0 for a, b in zip(idx.numpy(), ie.numpy())])

    r = {}
    for name, algo, kw in (("list", "ivf", {"nprobe": 2, "probe": "list", "nlist": 24}),
                           ("query", "ivf", {"nprobe": 2, "probe": "query", "nlist": 24}),
                           ("nnd", "nn_descent", {"nprobe": 2, "probe": "query", "nlist": 24, "nnd_iters": 2})):
        d, i = build_knn_graph(X, 10, algo, kw, seed=1)
        assert torch.all(d[:, 1:] >= d[:, :-1] - 1e-6)
        assert all(len(set(row)) == 10 for row in i[:500].tolist())
        ref = ((X[i.clamp_min(0)] - X.unsqueeze(1)) ** 2).sum(-1).sqrt()
        assert torch.allclose(d, ref, atol=1e-3)
        r[name] = rec(i)
    assert r["query"] > r["list"] + 0.05 and r["nnd"] > r["query"], r


def test_ivf_knn_graph_recall():
    """IVF-list all-points graph (UMAP build_algo='ivf') vs the exact graph: recall >= 0.9."""
    import torch

    from spark_rapids_ml_nai_amd.models.knn_graph import knn_graph_brute, knn_graph_ivf

    X, _ = make_blobs(4000, 16, centers=12, cluster_std=3.0, random_state=3)
    Xt = torch.from_numpy(X.astype(np.float32))
    de, ie = knn_graph_brute(Xt, 10)
    da, ia = knn_graph_ivf(Xt, 10, nlist=16, nprobe=6, seed=1)
    assert ia.shape == (4000, 10) and (ia[:, 0] == torch.arange(4000)).float().mean() > 0.99
    hit = np.mean([len(set(a) & set(b)) / 10.0 for a, b in zip(ia.numpy(), ie.numpy())])
    assert hit >= 0.9
    assert torch.all(da[:, 1:] >= da[:, :-1] - 1e-6)
    # distances are exact for the selected neighbours
    sel = Xt[ia.clamp_min(0)]
    ref = ((sel - Xt.unsqueeze(1)) ** 2).sum(-1).sqrt()
    assert torch.allclose(da, ref, atol=1e-3)


def test_umap_ivf_graph_trustworthiness():
    X, _ = _digits()
    df = DataFrame.from_numpy(X)
    model = UMAP(random_state=1, build_algo="ivf", build_kwds={"nlist": 8, "nprobe": 4}).fit(df)
    assert model.getOrDefault("build_algo") == "ivf"
    assert trustworthiness(X, model.embedding_, n_neighbors=15) > 0.9


@pytest.mark.dist
def test_umap_two_ranks(monkeypatch):
    """Distributed fit (replicated rows, tile-parallel graph, edge-parallel SGD with a delta
    all-reduce per epoch) on 2 gloo ranks reaches the single-rank quality."""
    monkeypatch.setenv("SRML_FORCE_CPU", "1")
    X, _ = _digits(900)
    df = DataFrame.from_numpy(X, num_partitions=2)
    for algo in ("brute_force_knn", "ivf"):
        m2 = UMAP(random_state=5, num_workers=2, n_epochs=200, build_algo=algo,
                  build_kwds={"nlist": 8, "nprobe": 4}).fit(df)
        assert m2.embedding_.shape == (900, 2) and m2.raw_data_.shape == X.shape
        assert trustworthiness(X, m2.embedding_, n_neighbors=15) > 0.88


def test_umap_multi_column_input():
    X, _ = make_blobs(300, 3, centers=3, random_state=5)
    import pandas as pd

    df = DataFrame.from_pandas(pd.DataFrame({"a": X[:, 0], "b": X[:, 1], "c": X[:, 2]}))
    model = UMAP(random_state=0).setFeaturesCols(["a", "b", "c"]).fit(df)
    out = model.transform(df)
    assert out.columns == ["features", "embedding"]


def test_ivf_graph_list_order_maps_back():
    """knn_graph_ivf(list_order=True) is the same graph relabelled: row i is original row order[i]
    and its neighbours are list positions (CPU)."""
    import numpy as np
    import torch

    from spark_rapids_ml_nai_amd.models.knn_graph import knn_graph_ivf

    g = np.random.default_rng(3)
    X = torch.from_numpy(np.concatenate([g.normal(c, 1.0, (300, 8)) for c in range(6)]).astype(np.float32))
    d0, i0 = knn_graph_ivf(X, 7, nlist=12, nprobe=4, seed=2)
    d1, i1, order = knn_graph_ivf(X, 7, nlist=12, nprobe=4, seed=2, list_order=True)
    assert sorted(order.tolist()) == list(range(X.shape[0]))
    back = torch.where(i1 >= 0, order[i1.clamp_min(0)], torch.full_like(i1, -1))
    torch.testing.assert_close(d1, d0[order])
    assert torch.equal(back, i0[order])


def test_umap_spmd_two_ranks_every_rank_gets_a_model(tmp_path):
    """torchrun (SPMD) UMAP on 2 gloo ranks: every rank builds its model (rank 1 used to get
    (None, None) back from the worker and fail in _make_model, leaving rank 0 in a collective)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = tmp_path / "ns.jsonl"
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29634", os.path.join(root, "tools", "northstar.py"),
           "--configs", "umap", "--scale", "0.0001", "--out", str(out)]
    r = subprocess.run(cmd, env=env, cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    rec = json.loads(out.read_text().strip().splitlines()[-1])
    assert "error" not in rec and rec["n_gpus"] == 2 and rec["finite"], rec
    assert rec["trustworthiness"] > 0.9, rec


def test_broadcast_chunks_cache_keeps_both_arrays_of_a_model():
    """The executor-side cache holds a model's embedding AND raw rows together (the second array
    must not evict the first), and only another model's arrays are evicted."""
    import numpy as np

    from spark_rapids_ml_nai_amd.umap import _BroadcastChunks

    class _B:
        def __init__(self, v):
            self.value = v
            self.reads = 0

    class _SC:
        def broadcast(self, v):
            return _B(v)

    class _Spark:
        sparkContext = _SC()

    _BroadcastChunks._cache.clear()
    emb, raw = np.arange(12, dtype=np.float32).reshape(6, 2), np.ones((6, 4), np.float32)
    e = _BroadcastChunks(_Spark(), emb, 16, "m1", "e")
    r = _BroadcastChunks(_Spark(), raw, 16, "m1", "r")
    assert len(e) == 3 and len(r) == 6
    a0, b0 = e.value(), r.value()
    assert e.value() is a0 and r.value() is b0  # cache hits for both arrays
    np.testing.assert_array_equal(a0, emb)
    other = _BroadcastChunks(_Spark(), emb, 1 << 20, "m2", "e")
    other.value()
    assert set(_BroadcastChunks._cache) == {("m2", "e")}
    _BroadcastChunks._cache.clear()
