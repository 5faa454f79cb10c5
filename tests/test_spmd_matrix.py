"""SPMD (torchrun) correctness matrix: every public entry point run with 2 and 4 gloo ranks, each
rank holding only an uneven shard of every frame, against ONE process on the concatenated data.

This is the launch mode of ``bench.py --gpus N``, ``tools/northstar.py`` and the 8-GPU runs.
Gates: exact-search results (kNN, exhaustive IVF, DBSCAN labels) must be identical; ids global
and unique; every rank gets back exactly its own query / row count. Fitted models use the
reference's multi-GPU vs single-GPU tolerances (PCA / KMeans 1e-3, tests/test_pca.py:344-349,
tests/test_kmeans.py:274; RF accuracy gap < 0.07 / R^2 < 0.09, tests/test_random_forest.py:401,491).
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "spmd_matrix_driver.py")
pytestmark = [pytest.mark.dist]
WORLDS = [2, 4, 8]

sys.path.insert(0, os.path.join(ROOT, "tests"))
from spmd_matrix_driver import global_data  # noqa: E402


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env() -> dict:
    env = dict(os.environ, SRML_FORCE_CPU="1", OMP_NUM_THREADS="1", PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "SRML_NUM_WORKERS"):
        env.pop(k, None)
    return env


def _load(d: str, world: int) -> list:
    return [dict(np.load(os.path.join(d, "rank%d.npz" % r))) for r in range(world)]


@pytest.fixture(scope="module")
def runs(tmp_path_factory):
    res = {}
    d = str(tmp_path_factory.mktemp("single"))
    r = subprocess.run([sys.executable, DRIVER, "--single", "--out", d], env=_env(), capture_output=True,
                       text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    res[1] = _load(d, 1)
    for w in WORLDS:
        d = str(tmp_path_factory.mktemp("w%d" % w))
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % w,
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), DRIVER, "--out", d]
        r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=900, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-4000:]
        res[w] = _load(d, w)
    return res


def _cat(ranks: list, key: str) -> np.ndarray:
    return np.concatenate([r[key] for r in ranks])




@pytest.mark.parametrize("w", WORLDS)
def test_every_rank_gets_its_own_rows(runs, w):
    g = global_data()
    ranks = runs[w]
    for r in ranks:
        lo, hi = r["rows"]
        qlo, qhi = r["qrows"]
        for key in ("pca_transform", "kmeans_pred", "ols_pred", "logreg_pred", "rfc_pred", "dbscan_labels",
                    "umap_transform"):
            assert r[key].shape[0] == hi - lo, (key, r[key].shape, lo, hi)
        assert r["knn_qid"].shape[0] == qhi - qlo and r["ann_qid"].shape[0] == qhi - qlo
    assert _cat(ranks, "dbscan_labels").shape[0] == g["Xb"].shape[0]


@pytest.mark.parametrize("w", WORLDS)
def test_ids_are_global_and_unique(runs, w):
    single, ranks = runs[1][0], runs[w]
    np.testing.assert_array_equal(_cat(ranks, "knn_item_ids"), single["knn_item_ids"])
    np.testing.assert_array_equal(_cat(ranks, "knn_query_ids"), single["knn_query_ids"])
    qid = _cat(ranks, "knn_qid")
    assert len(np.unique(qid)) == len(qid)
    for r in ranks:  # each rank answers exactly its own queries
        np.testing.assert_array_equal(np.sort(r["knn_qid"]), np.sort(r["knn_query_ids"]))


@pytest.mark.parametrize("w", WORLDS)
def test_exact_knn_and_ann_match_single(runs, w):
    single, ranks = runs[1][0], runs[w]
    qid = _cat(ranks, "knn_qid")
    o, os_ = np.argsort(qid), np.argsort(single["knn_qid"])
    np.testing.assert_array_equal(_cat(ranks, "knn_ind")[o], single["knn_ind"][os_])
    np.testing.assert_allclose(_cat(ranks, "knn_dist")[o], single["knn_dist"][os_], rtol=1e-5, atol=1e-5)
    # exhaustive IVF (nprobe = nlist) returns the exact neighbours on any number of ranks
    aq = _cat(ranks, "ann_qid")
    np.testing.assert_array_equal(_cat(ranks, "ann_ind")[np.argsort(aq)], single["knn_ind"][os_])
    assert sum(int(r["join_rows"][0]) for r in ranks) == int(single["join_rows"][0]) == 300 * 6
    assert sum(int(r["ann_join_rows"][0]) for r in ranks) == int(single["ann_join_rows"][0])


@pytest.mark.parametrize("w", WORLDS)
def test_dbscan_labels_match_single(runs, w):
    single, ranks = runs[1][0], runs[w]
    np.testing.assert_array_equal(_cat(ranks, "dbscan_labels"), single["dbscan_labels"])
    assert len(set(single["dbscan_labels"].tolist()) - {-1}) == 5


@pytest.mark.parametrize("w", WORLDS)
def test_dp_models_match_single(runs, w):
    single, ranks = runs[1][0], runs[w]
    for r in ranks:
        np.testing.assert_allclose(np.abs(r["pca_components"]), np.abs(single["pca_components"]), atol=1e-3)
        np.testing.assert_allclose(r["pca_evr"], single["pca_evr"], atol=1e-3)
        np.testing.assert_allclose(np.sort(r["kmeans_centers"], 0), np.sort(single["kmeans_centers"], 0), atol=1e-3)
        for name in ("ols", "ridge", "enet"):
            c1 = single[name + "_coef"]
            np.testing.assert_allclose(r[name + "_coef"], c1, rtol=1e-4, atol=1e-4 * np.abs(c1).max())
            np.testing.assert_allclose(r[name + "_intercept"], single[name + "_intercept"], atol=1e-3)
        for name in ("logreg", "logreg_multi"):
            o1 = float(single[name + "_objective"][0])
            assert abs(float(r[name + "_objective"][0]) - o1) <= 1e-5 * abs(o1) + 1e-8
    np.testing.assert_allclose(np.abs(_cat(ranks, "pca_transform")), np.abs(single["pca_transform"]), atol=1e-3)
    np.testing.assert_allclose(_cat(ranks, "ols_pred"), single["ols_pred"], rtol=1e-4, atol=1e-3)
    assert (_cat(ranks, "logreg_pred") == single["logreg_pred"]).mean() > 0.995
    assert (_cat(ranks, "logreg_multi_pred") == single["logreg_multi_pred"]).mean() > 0.99
    # KMeans labels agree up to a relabelling of the clusters
    a, b = _cat(ranks, "kmeans_pred").astype(int), single["kmeans_pred"].astype(int)
    pairs = set(zip(a.tolist(), b.tolist()))
    assert len(pairs) == len(set(a.tolist())) == len(set(b.tolist()))


@pytest.mark.parametrize("w", WORLDS)
def test_forests_cv_and_umap(runs, w):
    g = global_data()
    single, ranks = runs[1][0], runs[w]
    assert all(int(r["rfc_trees"][0]) == 12 for r in ranks)
    acc = lambda p: (p == g["yc"]).mean()  # noqa: E731
    assert abs(acc(_cat(ranks, "rfc_pred")) - acc(single["rfc_pred"])) < 0.07
    r2 = lambda p: 1 - np.mean((p - g["yr"]) ** 2) / np.var(g["yr"])  # noqa: E731
    # ensemble mode (reference semantics) grows each rank's trees on its local rows only: at 8 ranks
    # a tree sees ~150 of the 1200 rows, so the R^2 gap widens beyond the reference's 2-worker gate
    assert abs(r2(_cat(ranks, "rfr_pred")) - r2(single["rfr_pred"])) < (0.09 if w <= 4 else 0.2)
    # CrossValidator: every rank sees the same metrics and best model; close to the 1-rank run
    for r in ranks:
        np.testing.assert_allclose(r["cv_avg"], ranks[0]["cv_avg"], rtol=1e-9)
        assert int(np.argmin(r["cv_avg"])) == int(np.argmin(single["cv_avg"]))
        np.testing.assert_allclose(r["cv_best_coef"], single["cv_best_coef"], rtol=1e-3, atol=1e-3)
    np.testing.assert_allclose(ranks[0]["cv_avg"], single["cv_avg"], rtol=0.2)
    # UMAP: the fit sees every rank's rows; transform of the concatenated shards keeps quality
    from sklearn.manifold import trustworthiness

    assert all(int(r["umap_embedding_rows"][0]) == g["Xb"].shape[0] for r in ranks)
    emb = _cat(ranks, "umap_transform")
    assert np.isfinite(emb).all()
    t_w = trustworthiness(g["Xb"], emb, n_neighbors=10)
    t_1 = trustworthiness(g["Xb"], single["umap_transform"], n_neighbors=10)
    assert t_w > t_1 - 0.02, (t_w, t_1)


@pytest.mark.parametrize("w", WORLDS)
def test_sparse_logreg_matches_single(runs, w):
    single, ranks = runs[1][0], runs[w]
    o1 = float(single["logreg_sparse_objective"][0])
    for r in ranks:
        assert abs(float(r["logreg_sparse_objective"][0]) - o1) <= 1e-5 * abs(o1) + 1e-8
        np.testing.assert_allclose(r["logreg_sparse_coef"], single["logreg_sparse_coef"], rtol=1e-3, atol=1e-3)
    assert (_cat(ranks, "logreg_sparse_pred") == single["logreg_sparse_pred"]).mean() > 0.995


@pytest.mark.parametrize("w", WORLDS)
def test_data_parallel_forest_is_one_model(runs, w):
    g = global_data()
    single, ranks = runs[1][0], runs[w]
    for r in ranks[1:]:  # the same trees on every rank
        np.testing.assert_array_equal(r["rfdp_pred_all"], ranks[0]["rfdp_pred_all"])
    acc = lambda p: (p == g["yc"]).mean()  # noqa: E731
    assert abs(acc(ranks[0]["rfdp_pred_all"]) - acc(single["rfdp_pred_all"])) < 0.07


@pytest.mark.parametrize("w", WORLDS)
def test_supervised_umap_and_fp64(runs, w):
    from sklearn.manifold import trustworthiness

    g = global_data()
    single, ranks = runs[1][0], runs[w]
    emb = _cat(ranks, "umap_sup_transform")
    assert emb.shape == (g["Xb"].shape[0], 2) and np.isfinite(emb).all()
    t_w = trustworthiness(g["Xb"], emb, n_neighbors=10)
    t_1 = trustworthiness(g["Xb"], single["umap_sup_transform"], n_neighbors=10)
    assert t_w > t_1 - 0.03, (t_w, t_1)
    for r in ranks:
        np.testing.assert_allclose(np.abs(r["pca64_components"]), np.abs(single["pca64_components"]), atol=1e-6)
        c1 = single["ols64_coef"]
        np.testing.assert_allclose(r["ols64_coef"], c1, rtol=1e-7, atol=1e-8 * np.abs(c1).max())


@pytest.mark.parametrize("w", WORLDS)
def test_save_load_round_trip_on_every_rank(runs, w):
    for r in runs[w]:
        assert r["roundtrip_maxdiff"].shape == (4,)
        assert float(r["roundtrip_maxdiff"].max()) <= 1e-6, r["roundtrip_maxdiff"]
