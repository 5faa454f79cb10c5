"""SPMD launch-mode edges (torchrun, gloo ranks): concurrent overwrite-saves of one model path from
every rank, and an empty shard on one rank.

Reference semantics: the Spark driver is the only model writer (``core.py:249-336``), and a worker
without rows fails the fit with "A worker received no data" (``core.py:750-753``). Under SPMD every
rank calls ``save`` and every rank runs the fit, so the ranks must (a) leave ONE complete, loadable
model directory after every save and raise the same error if the write fails, and (b) agree on the
empty-shard error instead of the peers blocking in their first collective.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "tests", "spmd_edge_driver.py")
pytestmark = [pytest.mark.dist]


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(tmp_path, world, *extra):
    env = dict(os.environ, SRML_FORCE_CPU="1", OMP_NUM_THREADS="1", PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT", "SRML_NUM_WORKERS"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % world,
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), DRIVER, "--out", str(tmp_path)] + list(extra)
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    out = []
    for i in range(world):
        with open(os.path.join(str(tmp_path), "rank%d.json" % i)) as f:
            out.append(json.load(f))
    return out


@pytest.mark.parametrize("world", [2, 4])
def test_concurrent_overwrite_saves_stay_loadable(tmp_path, world):
    ranks = _run(tmp_path, world, "--mode", "saves", "--reps", "10")
    for r in ranks:
        assert r["save_errors"] == [], r["save_errors"]
        assert r["load_ok"] == r["reps"] == 10
        assert r["leftovers"] == []  # no temporary directories left behind
        assert r["exists_error"] is not None and "already exists" in r["exists_error"]
    assert len({r["exists_error"] for r in ranks}) == 1  # every rank raises the same error


@pytest.mark.parametrize("world,empty", [(2, 1), (4, 0)])
def test_empty_shard_error_is_agreed(tmp_path, world, empty):
    ranks = _run(tmp_path, world, "--mode", "empty", "--empty-rank", str(empty))
    names = ranks[0]["fits"].keys()
    assert set(names) >= {"PCA", "KMeans", "LinearRegression", "LogisticRegression", "RandomForestClassifier"}
    for name in names:
        msgs = {r["fits"][name]["error"] for r in ranks}
        assert len(msgs) == 1, (name, msgs)
        msg = msgs.pop()
        assert msg is not None and msg.startswith("A worker received no data"), msg
        assert "[%d]" % empty in msg
        assert max(r["fits"][name]["seconds"] for r in ranks) < 5.0


def test_multi_rank_bench_fails_fast_on_stuck_collective():
    """bench.py with 2 ranks, rank 1 stuck before its fit's collectives: rank 0's fit watchdog
    (SRML_COMM_TIMEOUT, defaulted for multi-rank runs) aborts the communicator and the whole job
    exits non-zero, long before the process-group timeout."""
    import time

    env = dict(os.environ, SRML_FORCE_CPU="1", OMP_NUM_THREADS="1", PYTHONPATH=ROOT, SRML_FAULT_RANK="1",
               SRML_FAULT_MODE="hang", SRML_FAULT_HANG_S="120", SRML_COMM_TIMEOUT="5")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "SRML_NUM_WORKERS"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rows", "2000", "--cols", "16",
           "--steps", "1", "--warmup", "0", "--algos", "linear_regression", "--no-transform", "--no-quality"]
    t0 = time.time()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode != 0
    assert time.time() - t0 < 100
    assert "communicator aborted" in r.stderr or "communicator failed" in r.stderr, r.stderr[-3000:]
