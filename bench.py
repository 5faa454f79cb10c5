#!/usr/bin/env python
"""Headline benchmark: fit time & speedup vs Spark-ML CPU on the reference's workload suite.

Contract (driver): ``python bench.py --gpus N --steps K --warmup W``; for N > 1 launched with
``torch.distributed.run --nproc-per-node N`` (one rank per MI355X, RCCL over xGMI).

What is measured (BASELINE.json metric "fit time (s) & speedup vs Spark-ML CPU at fixed
rows x features"): the reference's 8 headline workloads — KMeans (k=1000, 30 iters, random
init), PCA (k=3), LinearRegression OLS / ElasticNet / Ridge, LogisticRegression (L2, 200
iters), RandomForestClassifier (50 trees, depth 13, 128 bins), RandomForestRegressor (30 trees,
depth 6) — on 1,000,000 x 3000 float32 synthetic data of the same families, split row-wise
over N ranks (strong scaling: total rows fixed). A "step" = one full fit of every workload
through the public estimator API, starting from host-resident (pinned) Arrow-backed
DataFrames, so the timed region includes host->device ingest, every kernel, every RCCL
collective and model construction. ``value`` = geometric-mean speedup of our fit time over
the Spark-ML CPU fit time; ``vs_baseline`` = value / the reference GPU's own
geometric-mean speedup on the same table (20.1x).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import traceback


def _batched_frame(X, y, batch_rows):
    """A rank's shard as pageable Arrow record batches of ``batch_rows`` rows (each its own buffer,
    like Spark's ``spark.sql.execution.arrow.maxRecordsPerBatch`` batches)."""
    import numpy as np
    import pyarrow as pa

    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.core.dataframe import dense_to_list_array

    rbs = []
    for r0 in range(0, X.shape[0], batch_rows):
        xb = np.array(X[r0: r0 + batch_rows], copy=True)  # fresh pageable buffer per batch
        cols = {"features": dense_to_list_array(xb)}
        if y is not None:
            cols["label"] = pa.array(np.array(y[r0: r0 + batch_rows], copy=True))
        rbs.append(pa.RecordBatch.from_pydict(cols))
    return DataFrame([pa.Table.from_batches(rbs)])


def _spawn_ranks(n: int) -> int:
    """Re-run this command as an n-rank torch.distributed job on this node (127.0.0.1 rendezvous)."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--cols", type=int, default=3000)
    ap.add_argument("--algos", type=str, default="all")
    ap.add_argument("--global-data", action="store_true",
                    help="every rank generates the whole dataset from one seed and keeps its row slice "
                         "(N-invariant data: multi-rank rehearsals compare models against the 1-rank fit)")
    ap.add_argument("--ingest", choices=("pinned", "batches"), default="pinned",
                    help="pinned: each rank's shard is one page-locked buffer (headline); batches: pageable "
                         "Arrow record batches of --batch-rows rows, as Spark's mapInArrow delivers them")
    ap.add_argument("--batch-rows", type=int, default=20000)
    ap.add_argument("--no-transform", action="store_true",
                    help="skip the per-workload transform timing (outside the timed fit steps)")
    ap.add_argument("--no-quality", action="store_true",
                    help="skip the held-out quality metrics (scored after the timed fits)")
    ap.add_argument("--dump-models", type=str, default=None,
                    help="saves each workload's last fitted model under this directory (rank 0 writes)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # not under a launcher: start the N ranks ourselves (one process per GPU) from this parent,
        # which has not touched the GPU, and exit with the launcher's status
        sys.exit(_spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d; launch one rank per GPU (torch.distributed.run "
              "--nproc-per-node %d) or drop --gpus" % (args.gpus, world, args.gpus), file=sys.stderr)
        sys.exit(2)

    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and os.environ.get("SRML_FORCE_CPU", "0") != "1"
    device = torch.device("cuda", local_rank % torch.cuda.device_count()) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
        from spark_rapids_ml_nai_amd.parallel.context import bind_numa_local

        bind_numa_local(device)  # pinned staging buffers on the GPU's own socket
    force_pg = os.environ.get("SRML_COMM_FORCE_PG", "0") == "1"
    if world > 1:
        # bound every multi-rank fit: a stuck collective aborts the communicator after this many
        # seconds and the fit raises CommTimeout (the bench then exits non-zero) instead of holding
        # the node until the launcher's lease runs out
        os.environ.setdefault("SRML_COMM_TIMEOUT", "300")
    if world > 1 or force_pg:
        from datetime import timedelta

        if world == 1:  # SRML_COMM_FORCE_PG (test-only): a 1-rank group, so the RCCL paths run
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        # SRML_DIST_BACKEND=gloo: multi-rank rehearsal with several ranks sharing one GPU
        # (RCCL refuses two ranks on one device); the default on GPUs is RCCL ("nccl")
        backend = os.environ.get("SRML_DIST_BACKEND", "nccl" if use_gpu else "gloo")
        from spark_rapids_ml_nai_amd.parallel.comm import comm_timeout

        # per-operation timeout = the fit watchdog's bound: RCCL's own watchdog then tears a stuck
        # collective down, and gloo (whose abort cannot interrupt a blocked collective) times out
        dist.init_process_group(backend, timeout=timedelta(seconds=comm_timeout(600) if world > 1 else 600),
                                **({"device_id": device} if use_gpu and backend == "nccl" else {}))

    from spark_rapids_ml_nai_amd import DataFrame
    from spark_rapids_ml_nai_amd.bench.suite import (HOLDOUT_ROWS, HOLDOUT_SEED, REF_GEOMEAN_SPEEDUP, REF_GPU_S,
                                                      SPARK_CPU_S, geomean, make_shard, model_evidence,
                                                      model_quality, registry)
    from spark_rapids_ml_nai_amd.ops import native

    if use_gpu:
        native.lib()  # fail loudly if the HIP kernels are not available

    def barrier_sync() -> None:
        if use_gpu:
            torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()
        if use_gpu:
            torch.cuda.synchronize(device)

    reg = registry()
    names = list(SPARK_CPU_S.keys()) if args.algos == "all" else args.algos.split(",")
    m_total = args.rows
    bounds = np.linspace(0, m_total, world + 1).astype(np.int64)
    m_local = int(bounds[rank + 1] - bounds[rank])

    results = {}
    errors = {}
    for name in names:
        wl = reg.get(name)
        if wl is None:
            errors[name] = "not implemented"
            continue
        try:
            if args.global_data:
                Xg, yg = make_shard(wl.data, m_total, args.cols, device, 0, m_total)
                lo, hi = int(bounds[rank]), int(bounds[rank + 1])
                Xh = Xg[lo:hi]
                yh = yg[lo:hi] if yg is not None else None
                del Xg, yg
            else:
                Xh, yh = make_shard(wl.data, m_local, args.cols, device, rank, m_total)
            if args.ingest == "batches":
                df = _batched_frame(Xh, yh if wl.label else None, args.batch_rows)
                del Xh
                Xh = None
            else:
                df = DataFrame.from_numpy(Xh, yh if wl.label else None)
            est = wl.make_estimator()
            est.num_workers = world
            for _ in range(args.warmup):
                est.fit(df)
            barrier_sync()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                ts = time.perf_counter()
                model = est.fit(df)
                if os.environ.get("SRML_BENCH_VERBOSE") == "1":
                    print(f"[bench] {name} step {time.perf_counter() - ts:.4f} s", file=sys.stderr)
            barrier_sync()
            dt = time.perf_counter() - t0
            if world > 1:
                t = torch.tensor([dt], dtype=torch.float64, device=device)
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                dt = float(t.item())
            per_fit = dt / args.steps
            # per-rank split of the last timed fit (wall = h2d_exposed + compute + comm; all-gathered
            # by the fit itself at its end)
            per_rank = list(getattr(model, "_rank_stats", None) or [])
            results[name] = {
                "fit_s": round(per_fit, 4),
                "speedup_vs_spark_cpu": round(SPARK_CPU_S[name] / per_fit, 1) if name in SPARK_CPU_S else None,
                "ref_gpu_fit_s": REF_GPU_S.get(name),
                "vs_ref_gpu": round(REF_GPU_S[name] / per_fit, 1) if name in REF_GPU_S else None,
                "phases": {k: round(v, 4) for k, v in getattr(model, "_fit_timings", {}).items()},
                "evidence": model_evidence(name, model),
                "per_rank": per_rank,
            }
            if not args.no_transform:
                # reference BenchmarkBase times transform separately (benchmark/base.py:221-271):
                # one pass of model.transform over this rank's rows (H2D + kernels + D2H of the
                # output columns), outside the fit steps; failures are recorded, never fatal
                try:
                    barrier_sync()
                    t1 = time.perf_counter()
                    out = model.transform(df)
                    nout = out.count()
                    barrier_sync()
                    tr = time.perf_counter() - t1
                    if world > 1:
                        t = torch.tensor([tr], dtype=torch.float64, device=device)
                        dist.all_reduce(t, op=dist.ReduceOp.MAX)
                        tr = float(t.item())
                    results[name]["transform_s"] = round(tr, 4)
                    results[name]["transform_rows"] = int(nout)
                    del out
                except Exception as e:  # noqa: BLE001
                    results[name]["transform_error"] = repr(e)[:200]
            if rank == 0 and not args.no_quality:
                # held-out quality next to the speed (outside every timed region): fresh rows of the
                # same family and ground truth, scored through the public transform API
                H = min(HOLDOUT_ROWS, max(1, m_local))
                Xq, yq = make_shard(wl.data, H, args.cols, device, rank, m_total, seed=HOLDOUT_SEED)
                results[name]["quality"] = model_quality(name, model, Xq, yq if wl.label else None)
                del Xq, yq
            if args.dump_models:  # every rank calls save; under SPMD rank 0 alone writes
                model.write().overwrite().save(os.path.join(args.dump_models, name))
            del df, Xh, yh, model
        except Exception as e:  # noqa: BLE001
            errors[name] = repr(e)[:400]
            if rank == 0:
                traceback.print_exc(file=sys.stderr)
            from spark_rapids_ml_nai_amd.parallel.comm import CommError

            if isinstance(e, CommError) or (world > 1 and not dist.is_initialized()):
                # the communicator was aborted (watchdog / dead peer): no later workload can run
                print("bench.py: rank %d: communicator failed during %s: %r" % (rank, name, e), file=sys.stderr,
                      flush=True)
                sys.exit(3)
        if use_gpu:
            torch.cuda.empty_cache()

    speedups = [SPARK_CPU_S[k] / r["fit_s"] for k, r in results.items() if k in SPARK_CPU_S]
    value = geomean(speedups) if speedups else 0.0
    step_s = sum(r["fit_s"] for k, r in results.items() if k in SPARK_CPU_S)
    line = {
        "metric": "fit-time speedup vs Spark-ML CPU (geomean over reference headline workloads, 1Mx3000 fp32)",
        "value": round(value, 2),
        "unit": "x",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(step_s * 1000.0, 2),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": round(value / REF_GEOMEAN_SPEEDUP, 3) if speedups else None,
        "dtype": "fp32",
        "data": ("synthetic (device-generated, pinned host Arrow-backed DataFrames; H2D ingest inside timed fit)"
                 if args.ingest == "pinned" else
                 "synthetic (device-generated; pageable %d-row Arrow record batches per rank, as Spark delivers "
                 "them; H2D ingest inside timed fit)" % args.batch_rows),
        "config": {
            "model": "spark-rapids-ml headline suite: " + ",".join(results.keys()),
            "global_batch": m_total,
            "seq_len": args.cols,
            "rows": m_total,
            "features": args.cols,
            "parallelism": "dp%d" % world,
            "workloads": results,
            "missing_or_failed": errors,
            "ref_geomean_speedup": round(REF_GEOMEAN_SPEEDUP, 2),
            "ingest": args.ingest,
            "comm_backend": dist.get_backend() if dist.is_initialized() else "none",
        },
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1 or force_pg:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
