"""bench.py driver contract: one JSON line with the required keys, single process and SPMD
(torch.distributed.run, 2 gloo ranks on CPU — the same code path as one rank per MI355X)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _json_line(out: str) -> dict:
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _env():
    env = dict(os.environ, SRML_FORCE_CPU="1", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")
    env["PYTHONPATH"] = ROOT
    return env


def test_bench_single_process():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0", "--rows",
                        "3000", "--cols", "12", "--algos", "pca,linear_regression,kmeans"],
                       capture_output=True, text=True, timeout=600, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-2000:]
    d = _json_line(r.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 1 and d["value"] > 0
    assert {"model", "global_batch", "seq_len", "parallelism"} <= set(d["config"])
    assert not d["config"]["missing_or_failed"]


@pytest.mark.dist
def test_bench_spmd_two_ranks():
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29561", os.path.join(ROOT, "bench.py"),
                        "--gpus", "2", "--steps", "1", "--warmup", "0", "--rows", "3000", "--cols", "12"],
                       capture_output=True, text=True, timeout=900, env=_env(), cwd="/tmp")
    assert r.returncode == 0, r.stderr[-3000:]
    d = _json_line(r.stdout)
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "dp2"
    assert not d["config"]["missing_or_failed"], d["config"]["missing_or_failed"]
    assert len(d["config"]["workloads"]) == 8
