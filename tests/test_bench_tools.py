"""Benchmark tooling (reference python/benchmark/test_gen_data.py + benchmark runner smoke)."""
import os
import warnings

import numpy as np
import pytest

from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.bench import gen_data, runner

warnings.filterwarnings("ignore")


@pytest.mark.parametrize("kind", gen_data.TYPES)
@pytest.mark.parametrize("feature_type", ["array", "vector", "multi_cols"])
def test_gen_data(tmp_path, kind, feature_type):
    out = str(tmp_path / kind)
    counts = gen_data.generate([kind, "--num_rows", "500", "--num_cols", "6", "--feature_type", feature_type,
                                "--output_num_files", "3", "--output_dir", out, "--device", "cpu"])
    assert counts[out] == 500
    df = DataFrame.read_parquet(out)
    assert df.getNumPartitions() == 3 and df.count() == 500
    if kind == "sparse_regression" or feature_type == "vector":
        assert df.is_vector("feature_array")
    elif feature_type == "array":
        assert df.to_numpy("feature_array").shape == (500, 6)
    else:
        assert [c for c in df.columns if c != "label"] == ["c%d" % i for i in range(6)]
    if kind in ("blobs", "regression", "classification", "sparse_regression"):
        assert "label" in df.columns


def test_gen_data_train_fraction_and_determinism(tmp_path):
    a = str(tmp_path / "a")
    b = str(tmp_path / "b")
    for o in (a, b):
        gen_data.generate(["regression", "--num_rows", "400", "--num_cols", "4", "--feature_type", "array",
                           "--output_num_files", "2", "--output_dir", o, "--train_fraction", "0.75", "--device", "cpu"])
    ta = DataFrame.read_parquet(os.path.join(a, "train"))
    tb = DataFrame.read_parquet(os.path.join(b, "train"))
    ea = DataFrame.read_parquet(os.path.join(a, "eval"))
    assert ta.count() + ea.count() == 400
    assert np.array_equal(ta.to_numpy("feature_array"), tb.to_numpy("feature_array"))


@pytest.mark.parametrize("algo,kind,extra", [
    ("kmeans", "blobs", ["--k", "4", "--maxIter", "5"]),
    ("linear_regression", "regression", ["--regParam", "0.0"]),
    ("random_forest_classifier", "classification", ["--numTrees", "3", "--maxDepth", "4"]),
    ("approximate_nearest_neighbors", "blobs", ["--k", "4", "--algoParams", "{'nlist': 4, 'nprobe': 4}"]),
])
def test_runner(tmp_path, algo, kind, extra):
    out = str(tmp_path / kind)
    gen_data.generate([kind, "--num_rows", "600", "--num_cols", "8", "--feature_type", "array",
                       "--output_num_files", "2", "--output_dir", out, "--device", "cpu"])
    rep = str(tmp_path / "report.csv")
    rows = runner.run([algo, "--train_path", out, "--report_path", rep] + extra)
    assert rows[0]["fit"] > 0 and rows[0]["total"] >= rows[0]["fit"]
    assert os.path.exists(rep)
    if algo == "kmeans":
        assert rows[0]["inertia"] > 0
    if algo == "approximate_nearest_neighbors":
        assert rows[0]["avg_recall"] >= 0.95


def test_comm_sweep_single_rank():
    """tools/comm_sweep.py runs on one rank (the same code path the 8-GPU node runs under torchrun)."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, SRML_FORCE_CPU="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="29577")
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "comm_sweep.py"), "--max-bytes", "16K",
                        "--iters", "2", "--warmup", "1", "--ops", "all_reduce,all_gather"],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert {x["op"] for x in rows} == {"all_reduce", "all_gather"} and all(x["us"] > 0 for x in rows)


def test_chunked_rows_ingest_matches_contiguous():
    """A multi-batch Arrow partition is fitted from per-batch zero-copy views (no host concat)
    and gives the same model as the contiguous array."""
    import numpy as np
    import pyarrow as pa

    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.core.dataframe import ChunkedRows, array_column_chunks, dense_to_list_array
    from spark_rapids_ml_nai_amd.regression import LinearRegression

    rng = np.random.default_rng(1)
    X = rng.standard_normal((1000, 6)).astype(np.float32)
    y = X @ np.arange(1, 7) + 0.5
    rbs = [pa.RecordBatch.from_pydict({"features": dense_to_list_array(X[i:i + 128].copy()),
                                       "label": pa.array(y[i:i + 128])}) for i in range(0, 1000, 128)]
    df = DataFrame([pa.Table.from_batches(rbs)])
    ch = array_column_chunks(df.column("features"), np.float32)
    assert isinstance(ch, ChunkedRows) and ch.shape == (1000, 6) and len(ch.parts) == 8
    assert np.shares_memory(ch.parts[1], rbs[1].column(0).values.to_numpy())
    a = LinearRegression().fit(df)
    b = LinearRegression().fit(DataFrame.from_numpy(X, y))
    np.testing.assert_allclose(a.coefficients.toArray(), b.coefficients.toArray(), rtol=1e-6)
    # transform of the multi-batch partition: per-batch views as well (Arrow's combine_chunks
    # overflows list<float> offsets past 2^31 values), same predictions as the contiguous frame
    pa_ = a.transform(df).to_numpy("prediction")
    pb = a.transform(DataFrame.from_numpy(X, y)).to_numpy("prediction")
    np.testing.assert_allclose(pa_, pb, rtol=1e-6, atol=1e-6)
    from spark_rapids_ml_nai_amd.core.dataframe import array_column_to_dense

    np.testing.assert_array_equal(array_column_to_dense(df.column("features"), np.float32), X)


def test_sparse_regression_density_curves_and_redundant_columns():
    import scipy.sparse as sp

    from spark_rapids_ml_nai_amd.bench import datagen

    for curve in ("Linear", "Exponential"):
        d = datagen.sparse_density_values(0.05, curve, 10, 400, 20000, 4)
        assert d.shape == (10,) and np.isclose(d.mean(), 0.05) and np.all(np.diff(d) > 0)
    X, y, w = datagen.sparse_regression(20000, 400, seed=3, partition_seed=9, density=0.05,
                                        density_curve="Exponential", n_chunk=10, shuffle=False, n_informative=8)
    assert sp.issparse(X) and X.shape == (20000, 400)
    nnz_per_col = np.diff(X.tocsc().indptr)
    first, last = nnz_per_col[:40].mean(), nnz_per_col[-40:].mean()
    assert last > 5 * first  # density ramps across the column chunks
    assert abs(X.nnz / (20000 * 400) - 0.05) < 0.01
    np.testing.assert_allclose(y, X @ w, rtol=1e-10, atol=1e-8)  # noise 0, bias 0
    # redundant columns: exact linear mixes of the informative block
    X2, y2, _ = datagen.sparse_regression(5000, 100, seed=1, partition_seed=2, density=0.3, redundant_cols=10,
                                          n_informative=6, shuffle=False)
    red = X2[:, 90:].toarray()
    inf = X2[:, :6].toarray()
    coef, res, *_ = np.linalg.lstsq(inf, red, rcond=None)
    assert np.allclose(inf @ coef, red, atol=1e-8)
    # binary / multinomial labels
    _, yb, _ = datagen.sparse_regression(3000, 50, density=0.2, logistic_regression=True)
    assert set(np.unique(yb)) <= {0.0, 1.0}
    _, ym, _ = datagen.sparse_regression(3000, 50, density=0.2, logistic_regression=True, n_classes=4)
    assert set(np.unique(ym)) <= {0.0, 1.0, 2.0, 3.0} and len(np.unique(ym)) > 1


def test_gen_data_sparse_regression_cli(tmp_path):
    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.bench.gen_data import generate

    out = str(tmp_path / "sp")
    generate(["sparse_regression", "--num_rows", "3000", "--num_cols", "64", "--density", "0.02,0.2",
              "--output_num_files", "2", "--output_dir", out, "--device", "cpu"])
    df = DataFrame.read_parquet(out)
    assert df.count() == 3000 and df.is_vector("feature_array")


def _class_stats(X, y, c):
    Xc = X[y == c].astype(np.float64)
    ev = np.linalg.eigvalsh(np.cov(Xc, rowvar=False))[::-1]
    return Xc.mean(0), ev


def test_classification_generator_matches_make_classification():
    """The device classification generator follows the reference's distributed make_classification
    (2 clusters per class, per-cluster covariance A_k, unscaled redundant mix B, column shuffle,
    flip_y): at 20k x 60 (20 informative, 20 redundant) its per-class statistics match sklearn's
    make_classification drawn with the same random_state — the same centroids / A_k / B come out of
    that RandomState, the rows differ only by sampling."""
    import torch
    from sklearn.datasets import make_classification

    from spark_rapids_ml_nai_amd.bench import datagen

    m, n, ni, nr = 20000, 60, 20, 20
    X, y = datagen.classification(m, n, torch.device("cpu"), seed=11, n_informative=ni, n_redundant=nr,
                                  random_state=1)
    X, y = X.numpy(), y.numpy()
    Xs, ys = make_classification(n_samples=m, n_features=n, n_informative=ni, n_redundant=nr, n_classes=2,
                                 n_clusters_per_class=2, flip_y=0.01, random_state=1)
    assert abs(y.mean() - 0.5) < 0.02 and abs(ys.mean() - 0.5) < 0.02
    for c in (0, 1):
        mu, ev = _class_stats(X, y, c)
        mus, evs = _class_stats(Xs, ys, c)
        # covariance rank: redundant columns are linear in the informative ones -> n - nr
        tol = 1e-8 * ev[0]
        assert (ev > tol).sum() == (evs > 1e-8 * evs[0]).sum() == n - nr
        # spectrum shape: total variance and the leading eigenvalues within sampling / A_k noise
        np.testing.assert_allclose(ev.sum(), evs.sum(), rtol=0.25)
        np.testing.assert_allclose(ev[:5] / ev.sum(), evs[:5] / evs.sum(), atol=0.05)
        # class means: same scale (the centroid geometry, mapped through B)
        np.testing.assert_allclose(np.linalg.norm(mu), np.linalg.norm(mus), rtol=0.3)
    # the classes are separated only jointly: a linear model is far from perfect and far from chance
    from sklearn.linear_model import LogisticRegression as SkLR

    acc = SkLR(max_iter=300).fit(X[:15000], y[:15000]).score(X[15000:], y[15000:])
    acc_s = SkLR(max_iter=300).fit(Xs[:15000], ys[:15000]).score(Xs[15000:], ys[15000:])
    assert 0.6 < acc < 0.99 and abs(acc - acc_s) < 0.1, (acc, acc_s)


def test_logistic_labels_are_bernoulli_of_the_unscaled_target():
    import torch

    from spark_rapids_ml_nai_amd.bench import datagen

    z = torch.linspace(-4, 4, 200001, dtype=torch.float64)
    yb = datagen.logistic_labels(z, seed=3)
    assert set(np.unique(yb.numpy()).tolist()) == {0.0, 1.0}
    # P(y = 1 | z) = sigmoid(z): E[y] over the symmetric grid is 1/2, and near z = 0 it is mixed
    assert abs(float(yb.mean()) - 0.5) < 0.01
    mid = yb[(z.abs() < 0.2)].mean().item()
    assert 0.4 < mid < 0.6
    Y = torch.stack([z, -z, torch.zeros_like(z)], 1)
    ym = datagen.logistic_labels(Y, seed=4).numpy()
    assert set(np.unique(ym).tolist()) <= {0.0, 1.0, 2.0}
    p = torch.softmax(Y, 1).mean(0).numpy()
    np.testing.assert_allclose(np.bincount(ym.astype(int), minlength=3) / len(ym), p, atol=0.01)


def test_regression_family_matches_sklearn_make_regression():
    """The bench's regression family has sklearn make_regression's semantics at the reference's
    settings (n_informative 10; noise 10 for the linear-regression data, 0 for the forest data;
    bias 0): the same coefficient support size and range, the same residual noise variance."""
    import torch
    from sklearn.datasets import make_regression

    from spark_rapids_ml_nai_amd.bench import datagen
    from spark_rapids_ml_nai_amd.bench.suite import make_shard

    m, n = 20000, 300
    for noise, family in ((10.0, "regression_noise10"), (0.0, "regression")):
        X, y = make_shard(family, m, n, torch.device("cpu"), 0, m)
        Xs, ys, cs = make_regression(n_samples=m, n_features=n, noise=noise, coef=True, random_state=0)
        X64 = X.astype(np.float64)
        w, *_ = np.linalg.lstsq(X64, y.astype(np.float64), rcond=None)
        ws, *_ = np.linalg.lstsq(Xs, ys, rcond=None)
        # support: exactly 10 informative columns, coefficients in (0, 100) like sklearn's 100 U(0, 1)
        assert int((np.abs(w) > 1.0).sum()) == int((np.abs(ws) > 1.0).sum()) == int(np.count_nonzero(cs)) == 10
        big = w[np.abs(w) > 1.0]
        assert big.min() > 0 and big.max() < 100
        # noise: residual standard deviation equals the requested noise (0 -> fp32 rounding only)
        res, res_s = np.std(y - X64 @ w), np.std(ys - Xs @ ws)
        if noise > 0:
            assert abs(res / noise - 1) < 0.03 and abs(res_s / noise - 1) < 0.03
        else:
            assert res < 1e-3 * np.std(y) and res_s < 1e-9
        assert abs(float(np.mean(y))) < 0.1 * np.std(y)  # bias 0
    # the generator's defaults are make_regression's
    _, y0 = datagen.regression(2000, 50, torch.device("cpu"), seed=3)
    Xd, _ = datagen.regression(2000, 50, torch.device("cpu"), seed=3)
    w, *_ = np.linalg.lstsq(Xd.double().numpy(), y0.double().numpy(), rcond=None)
    assert int((np.abs(w) > 1.0).sum()) == 10
