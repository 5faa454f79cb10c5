"""RCCL code paths on a one-GPU box: with ``SRML_COMM_FORCE_PG=1`` a size-1
communicator over an initialised ``nccl`` (RCCL) process group runs every collective through the
backend instead of short-circuiting, so ``init_process_group(device_id=)``, event-timed
``CommStats``, ``batch_isend_irecv``, ``allgatherv`` / ``allgather_bytes`` and the one-shot mode
selection execute for real. Reference: common/cuml_context.py:68-124 (NCCL bootstrap)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

_SCRIPT = r"""
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
import numpy as np, torch, torch.distributed as dist
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%s" % os.environ["PORT"], rank=0, world_size=1,
                        device_id=dev)
from spark_rapids_ml_nai_amd import DataFrame
from spark_rapids_ml_nai_amd.parallel.context import WorkerContext, use_context
from spark_rapids_ml_nai_amd.parallel import oneshot
out = {"backend": dist.get_backend()}
ctx = WorkerContext.single(dev)
c = ctx.comm
out["comm_backend"] = c.backend
t = torch.arange(6, dtype=torch.float64, device=dev)
c.allreduce(t)
out["allreduce_ok"] = bool(torch.equal(t, torch.arange(6, dtype=torch.float64, device=dev)))
parts = c.allgatherv(torch.ones(3, 2, device=dev))
out["allgatherv_ok"] = len(parts) == 1 and tuple(parts[0].shape) == (3, 2)
out["bytes_ok"] = c.allgather_bytes(b"xyz") == [b"xyz"]
b = torch.full((4,), 7.0, device=dev)
out["bcast_ok"] = bool(torch.equal(c.broadcast(b, 0), torch.full((4,), 7.0, device=dev)))
r = torch.zeros(5, device=dev)
c.sendrecv(torch.arange(5, dtype=torch.float32, device=dev), 0, r, 0)
out["sendrecv_ok"] = bool(torch.equal(r, torch.arange(5, dtype=torch.float32, device=dev)))
out["single_node"] = bool(oneshot.single_node(c))
c.barrier()
out["stats_calls"] = c.stats.calls
out["stats_s"] = c.stats.seconds()
rng = np.random.default_rng(0)
X = rng.standard_normal((20000, 64)).astype(np.float32)
y = (X[:, 0] > 0).astype(np.float64)
df = DataFrame.from_numpy(X, y)
from spark_rapids_ml_nai_amd.feature import PCA
from spark_rapids_ml_nai_amd.clustering import KMeans
from spark_rapids_ml_nai_amd.classification import LogisticRegression
fits = {}
with use_context(ctx):
    for name, est in (("pca", PCA(k=3, inputCol="features", outputCol="o")), ("kmeans", KMeans(k=8, maxIter=5)),
                      ("logreg", LogisticRegression(maxIter=20))):
        m = est.fit(df)
        fits[name] = m._rank_stats[0]
out["fits"] = fits
from spark_rapids_ml_nai_amd.models import qn as qnm
out["qn_graph"] = dict(qnm.GRAPH_STATS)
# the same LogReg on the one-rank path (no collectives): the captured-RCCL fit must equal it
os.environ["SRML_COMM_FORCE_PG"] = "0"
ctx1 = WorkerContext.single(dev)
with use_context(ctx1):
    m1 = LogisticRegression(maxIter=20).fit(df)
os.environ["SRML_COMM_FORCE_PG"] = "1"
with use_context(ctx):
    m2 = LogisticRegression(maxIter=20).fit(df)
out["lr_same"] = bool(np.allclose(np.asarray(m1.coef_), np.asarray(m2.coef_), rtol=1e-5, atol=1e-8))
print("RESULT " + json.dumps(out))
dist.destroy_process_group()
"""


def _port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_paths_on_one_gpu():
    env = dict(os.environ, SRML_COMM_FORCE_PG="1", REPO=ROOT, PORT=str(_port()))
    r = subprocess.run([sys.executable, "-c", _SCRIPT], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("RESULT ")][-1][7:])
    assert out["backend"] == "nccl" and out["comm_backend"] == "nccl"
    for k in ("allreduce_ok", "allgatherv_ok", "bytes_ok", "bcast_ok", "sendrecv_ok", "single_node"):
        assert out[k], (k, out)
    assert out["stats_calls"] > 0 and out["stats_s"] > 0
    # the LogReg batches (small shard: graph-safe) were captured WITH their RCCL all-reduces
    assert out["qn_graph"]["captures"] >= 1 and out["qn_graph"].get("comm_capture_failed", 0) == 0, out["qn_graph"]
    assert out["lr_same"]
    for name, st in out["fits"].items():
        assert st["comm_calls"] > 0, (name, st)
        if name != "logreg":  # captured collectives are counted, not timed
            assert st["comm_s"] > 0, (name, st)
        parts = st["h2d_exposed_s"] + st["compute_s"] + st["comm_s"]
        assert abs(parts - st["wall_s"]) <= 0.05 * st["wall_s"] + 1e-6, (name, st)


def test_bench_forced_rccl_group():
    env = dict(os.environ, SRML_COMM_FORCE_PG="1", MASTER_PORT=str(_port()))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--rows", "40000", "--cols", "128",
                        "--algos", "pca,kmeans,logistic_regression", "--steps", "1", "--warmup", "1",
                        "--no-transform", "--no-quality"], env=env, capture_output=True, text=True, timeout=600,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["config"]["comm_backend"] == "nccl" and not line["config"]["missing_or_failed"]
    for name, w in line["config"]["workloads"].items():
        assert w["per_rank"][0]["comm_calls"] > 0, (name, w["per_rank"])
