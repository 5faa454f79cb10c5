"""Communicator semantics on CPU ranks (gloo): the ragged all-gather that every backend runs the
same way, per-rank collective accounting, comm-mode validation, bench.py's rank-count contract.
The one-shot missing-peer failure path runs on the GPU box (two processes on one MI355X)."""
import json
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.dist


def _ragged(ctx, payload):
    import torch

    rows, tail = payload
    t = torch.arange(rows * tail, dtype=torch.float64).view(rows, tail) + 1000 * ctx.rank
    parts = ctx.comm.allgatherv(t)
    blobs = ctx.comm.allgather_bytes(bytes([ctx.rank]) * (ctx.rank * 3))
    return [p.numpy().copy() for p in parts], blobs, ctx.comm.stats.calls, ctx.comm.stats.bytes


@pytest.mark.parametrize("sizes", [[5, 0, 3], [1, 7, 2, 7]])
def test_allgatherv_ragged(monkeypatch, sizes):
    monkeypatch.setenv("SRML_FORCE_CPU", "1")
    from spark_rapids_ml_nai_amd.parallel.launcher import run_barrier_job

    W = len(sizes)
    res = run_barrier_job(_ragged, [(s, 3) for s in sizes], use_gpu=False, timeout_s=300)
    for r, (parts, blobs, calls, nbytes) in enumerate(res):
        assert [p.shape[0] for p in parts] == sizes
        for q, p in enumerate(parts):
            np.testing.assert_array_equal(p, np.arange(sizes[q] * 3, dtype=np.float64).reshape(-1, 3) + 1000 * q)
        assert blobs == [bytes([q]) * (q * 3) for q in range(W)]
        assert calls >= 4 and nbytes > 0  # sizes + payload, twice


def _mode_worker(ctx, payload):
    import torch

    x = torch.full((4,), float(ctx.rank + 1), dtype=torch.float64)
    ctx.comm.allreduce(x)
    ctx.comm.poll()
    ctx.comm.check()
    return x.tolist(), ctx.comm.stats.snapshot()


def test_auto_mode_on_gloo_falls_back(monkeypatch):
    """``auto`` / ``oneshot`` only apply to device tensors on RCCL; gloo keeps working unchanged."""
    monkeypatch.setenv("SRML_FORCE_CPU", "1")
    monkeypatch.setenv("SRML_COMM", "auto")
    from spark_rapids_ml_nai_amd.parallel.launcher import run_barrier_job

    res = run_barrier_job(_mode_worker, [None, None], use_gpu=False, timeout_s=300)
    for vals, snap in res:
        assert vals == [3.0] * 4
        assert snap["comm_calls"] == 1 and snap["comm_bytes"] == 32 and snap["comm_s"] >= 0.0


def test_comm_mode_validation(monkeypatch):
    from spark_rapids_ml_nai_amd.parallel import oneshot

    monkeypatch.setenv("SRML_COMM", "AUTO")
    assert oneshot.comm_mode() == "auto"
    monkeypatch.setenv("SRML_COMM", "fastest")
    with pytest.raises(ValueError):
        oneshot.comm_mode()


def test_spark_comm_conf_read(monkeypatch):
    from spark_rapids_ml_nai_amd.parallel.spark import spark_comm_mode

    class _Conf(dict):
        pass

    class _Session:
        def __init__(self, **conf):
            self.conf = _Conf(conf)

    monkeypatch.delenv("SRML_COMM", raising=False)
    assert spark_comm_mode(_Session()) == "rccl"
    assert spark_comm_mode(_Session(**{"spark.rocm.ml.comm": "auto"})) == "auto"
    with pytest.raises(ValueError):
        spark_comm_mode(_Session(**{"spark.rocm.ml.comm": "bogus"}))


def _bench_env():
    env = dict(os.environ, SRML_FORCE_CPU="1", OMP_NUM_THREADS="1", PYTHONPATH=ROOT)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_bench_refuses_world_mismatch():
    env = dict(_bench_env(), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--rows", "64", "--cols", "8",
                        "--algos", "pca"], env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 2 and "WORLD_SIZE" in r.stderr


@pytest.mark.slow
def test_bench_self_spawns_ranks():
    """``bench.py --gpus 2`` without a launcher runs 2 ranks and reports them with a per-rank split."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rows", "4000", "--cols",
                        "16", "--algos", "pca,logistic_regression", "--steps", "1", "--warmup", "0", "--no-transform"],
                       env=dict(_bench_env(), SRML_LOG_LEVEL="INFO"), capture_output=True, text=True, timeout=900,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["config"]["parallelism"] == "dp2"
    for name, w in line["config"]["workloads"].items():
        pr = w["per_rank"]
        assert [p["rank"] for p in pr] == [0, 1], name
        for p in pr:
            assert p["comm_calls"] > 0 and p["wall_s"] > 0 and p["compute_s"] <= p["wall_s"] + 1e-9
            # the split adds up: wall = exposed H2D + compute + collectives (within 5 %)
            parts = p["h2d_exposed_s"] + p["compute_s"] + p["comm_s"]
            assert abs(parts - p["wall_s"]) <= 0.05 * p["wall_s"] + 1e-6, (name, p)
    # the estimator logger prints one line per rank of every timed fit (from rank 0 only), plus the
    # worker stages of each rank
    for est in ("PCA", "LogisticRegression"):
        for rk in (0, 1):
            lines = [ln for ln in r.stderr.splitlines() if "srml.%s - INFO - %s fit rank %d:" % (est, est, rk) in ln]
            assert len(lines) == 1, (est, rk, r.stderr[-3000:])
    for stage in ("Loading data", "Initializing context", "Invoking fit", "Fit complete"):
        for rk in (0, 1):
            assert "rank %d/2: %s" % (rk, stage) in r.stderr, (stage, rk)


_MISSING_PEER = textwrap.dedent("""
    import os, sys, datetime, time
    sys.path.insert(0, os.environ["REPO"])
    os.environ["SRML_ONESHOT_TIMEOUT_S"] = "2"
    import torch, torch.distributed as dist
    from spark_rapids_ml_nai_amd.parallel.comm import Communicator, CommError
    from spark_rapids_ml_nai_amd.parallel.oneshot import OneShotAllreduce
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=60))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    comm = Communicator(rank, world, torch.device("cpu"))
    os_ = OneShotAllreduce(comm, dev, max_bytes=4096)
    assert os_.ok, os_.reason
    comm._oneshot = os_          # what Communicator.allreduce selects on RCCL
    x = torch.ones(64, dtype=torch.float64, device=dev)
    mode = os.environ["MODE"]
    t0 = time.monotonic()
    try:
        for it in range(6):
            if rank == 1 and it == 2:
                if mode == "skip":
                    continue     # rank 1 skips one call: its peer must not hang or return a partial
                time.sleep(5)    # straggler: arrives after the peer's 2 s deadline
            y = os_.allreduce(x.clone())
            comm.poll()
        torch.cuda.synchronize()
        bad = bool(torch.isnan(y).any().item())
        comm.check()
        print("NO_ERROR", rank, bad, flush=True)
        sys.exit(0)
    except Exception as e:
        print("COMM_ERROR", rank, type(e).__name__, "%.1f" % (time.monotonic() - t0), e, flush=True)
        sys.exit(3)
""")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["skip", "straggle"])
def test_oneshot_missing_peer_fails_both_ranks(tmp_path, mode):
    script = tmp_path / "w.py"
    script.write_text(_MISSING_PEER)
    env = dict(os.environ, REPO=ROOT, MASTER_ADDR="127.0.0.1", MODE=mode, WORLD_SIZE="2",
               MASTER_PORT=str(29500 + os.getpid() % 200 + (7 if mode == "skip" else 0)))
    procs = [subprocess.Popen([sys.executable, "-u", str(script)], env=dict(env, RANK=str(r)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for r in range(2)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=90)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for rc, out in outs:
        assert rc == 3 and "COMM_ERROR" in out, out[-2000:]
    assert "CommError" in outs[0][1]  # the rank that waited names the lost peer
