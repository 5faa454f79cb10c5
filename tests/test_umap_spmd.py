"""Distributed UMAP fit under torchrun (2 and 4 gloo ranks) vs one process on the same data:
every phase shards (per-rank rows ~ N / W for the quantiser sample, the bucketing, the kNN query
tiles, the spectral row block and the epoch edges; only the fuzzy union is replicated), all ranks
end with the same embedding, and the quality matches the one-process fit (trustworthiness within
0.01; reference tests/test_umap.py:146,377 gate multi-GPU UMAP on trustworthiness)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "umap_spmd_driver.py")
pytestmark = [pytest.mark.dist]
sys.path.insert(0, os.path.join(ROOT, "tests"))
from umap_spmd_driver import data  # noqa: E402


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env() -> dict:
    env = dict(os.environ, SRML_FORCE_CPU="1", OMP_NUM_THREADS="1", PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "SRML_NUM_WORKERS"):
        env.pop(k, None)
    return env


@pytest.fixture(scope="module")
def fits(tmp_path_factory):
    out = {}
    d = str(tmp_path_factory.mktemp("single"))
    r = subprocess.run([sys.executable, DRIVER, "--single", "--out", d], env=_env(), capture_output=True, text=True,
                       timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out[1] = [dict(np.load(os.path.join(d, "rank0.npz")))]
    for w in (2, 4):
        d = str(tmp_path_factory.mktemp("w%d" % w))
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % w,
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), DRIVER, "--out", d]
        r = subprocess.run(cmd, env=_env(), capture_output=True, text=True, timeout=900, cwd=ROOT)
        assert r.returncode == 0, r.stderr[-3000:]
        out[w] = [dict(np.load(os.path.join(d, "rank%d.npz" % i))) for i in range(w)]
    return out


@pytest.mark.parametrize("w", [2, 4])
def test_every_phase_shards(fits, w):
    N = data().shape[0]
    one = json.loads(str(fits[1][0]["phases"]))
    for r in fits[w]:
        ph = json.loads(str(r["phases"]))
        assert set(ph) >= {"quantizer", "bucketing", "knn_lists", "fuzzy_union", "spectral", "epochs"}, ph
        assert abs(ph["bucketing"]["rows"] - N / w) <= 1
        assert abs(ph["spectral"]["rows"] - N / w) <= 1
        assert abs(ph["quantizer"]["rows"] - one["quantizer"]["rows"] / w) <= 1
        assert 0.5 * N / w <= ph["knn_lists"]["rows"] <= 1.5 * N / w  # work-balanced tile ranges
        assert abs(ph["epochs"]["rows"] - one["epochs"]["rows"] / w) <= 1  # edges e % W == r
        assert ph["fuzzy_union"]["rows"] == N  # the only replicated phase
        # per-query probing (seed / probes / pairs) and the NN-descent round shard by rows too
        for name in ("query_seed", "query_probes", "query_pairs"):
            assert 0.5 * N / w <= ph[name]["rows"] <= 1.5 * N / w, (name, ph[name])
        assert abs(ph["nn_descent"]["rows"] - N / w) <= 1


@pytest.mark.parametrize("w", [2, 4])
def test_ranks_agree_and_quality_matches(fits, w):
    from sklearn.manifold import trustworthiness

    X = data()
    e0 = fits[w][0]["emb"]
    for r in fits[w][1:]:
        np.testing.assert_array_equal(r["emb"], e0)
    assert np.isfinite(e0).all()
    t_w = trustworthiness(X, e0, n_neighbors=12)
    t_1 = trustworthiness(X, fits[1][0]["emb"], n_neighbors=12)
    assert t_w >= t_1 - 0.01, (t_w, t_1)
