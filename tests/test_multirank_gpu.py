"""Two ranks sharing the GPU (gloo process group over cuda:0 tensors, launched by torchrun as the
north-star script is): the paths a one-rank-per-process job takes that the in-process tests do not —
each rank's own page-locked shard streamed in (PendingBins streamed root level) under the
node-partitioned histogram reduce-scatter (the padded node count of round 4's first 2-rank
north-star failure)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
@pytest.mark.parametrize("scatter", ["1", "0"])
def test_rf_data_parallel_two_ranks_streamed_root(tmp_path, scatter):
    out = tmp_path / "ns.jsonl"
    env = dict(os.environ, SRML_NS_BACKEND="gloo", SRML_RF_DP_SCATTER=scatter, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(29600 + int(scatter)),
           os.path.join(ROOT, "tools", "northstar.py"), "--configs", "rf", "--scale", "0.002", "--out", str(out)]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    rec = json.loads(out.read_text().strip().splitlines()[-1])
    assert "error" not in rec, rec
    assert rec["n_gpus"] == 2 and rec["split_mode"] == "data_parallel"
    assert rec["holdout_accuracy"] > 0.85, rec
    assert all(rk["comm_calls"] > 0 for rk in rec["ranks"]), rec["ranks"]


@pytest.mark.gpu
def test_rf_ensemble_fit_multiple_fewer_trees_than_ranks_streamed():
    """ADVICE r3 (forest.py pending bins): a param map with numTrees < ranks leaves one rank with no
    tree; its streamed chunks must still be binned before the next map reuses them."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29611", os.path.join(ROOT, "tools", "rf_pending_check.py")]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    rec = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert rec["equal"] and rec["trees"] == [1, 4], rec


@pytest.mark.gpu
def test_umap_two_ranks_ivf_pull_neg_lines():
    """UMAP on 2 ranks sharing the GPU: IVF graph built tile-range parallel in list order, pull-mode
    epochs over strided edge shards with line-shared negatives from each rank's snapshot, one
    all-reduce of the layout deltas per epoch; the scattered-back embedding must keep its quality."""
    env = dict(os.environ, SRML_NS_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    out = os.path.join(ROOT, "gpurun_out", "ns_umap_2rank_test.jsonl")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29621",
           os.path.join(ROOT, "tools", "northstar.py"), "--configs", "umap", "--scale", "0.006", "--out", out]
    r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=115)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    with open(out) as f:
        rec = json.loads(f.read().strip().splitlines()[-1])
    assert "error" not in rec, rec
    assert rec["n_gpus"] == 2 and rec["finite"], rec
    assert rec["trustworthiness"] > 0.9, rec


@pytest.mark.gpu
def test_kmeans_small_k_two_ranks_delta_steps_match_full_steps():
    """The small-k Lloyd loop on 2 ranks sharing the GPU (gloo all-reduce of the step buffer), on
    blobs from random start rows: with delta steps (label book; the mode follows the REDUCED moved count,
    so both ranks switch together) the fit reaches the same centres in the same iterations as with
    every step summing all rows."""
    import numpy as np

    recs = {}
    for delta in ("1", "0"):
        env = dict(os.environ, SRML_LLOYD_SMALL_DELTA=delta, MASTER_ADDR="127.0.0.1")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(29631 + int(delta)),
               os.path.join(ROOT, "tools", "kmeans_spmd_check.py")]
        r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=55)
        assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
        recs[delta] = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    a, b = np.asarray(recs["1"]["centres"]), np.asarray(recs["0"]["centres"])
    assert a.shape == (20, 64) and recs["1"]["world"] == 2
    assert min(recs["1"]["iters"], recs["0"]["iters"]) >= 3, (recs["1"]["iters"], recs["0"]["iters"])
    # the two runs' sums round differently (measured: 20 / 20 iterations, centres 3e-8 apart); a
    # near-tie row taking the other side would move its centres by ~4e-4, wrong delta sums by O(1)
    assert abs(recs["1"]["iters"] - recs["0"]["iters"]) <= 2, (recs["1"]["iters"], recs["0"]["iters"])
    assert float(np.abs(a - b).max()) < 1e-3, float(np.abs(a - b).max())
