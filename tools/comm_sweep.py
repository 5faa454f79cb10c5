"""Collective latency / bandwidth sweep over RCCL (GPU) or gloo (CPU), for the 8-GPU node.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/comm_sweep.py [--min-bytes 1K --max-bytes 64M]
    python tools/comm_sweep.py            # 1 rank: exercises the same code path (no peers)

Per op and message size: median time of --iters calls (after --warmup), algorithm bandwidth
(bytes / t) and bus bandwidth with the nccl-tests conventions (all_reduce x 2(n-1)/n,
all_gather / reduce_scatter / all_to_all x (n-1)/n, broadcast x 1), so the numbers compare with
the xGMI model in SURVEY §2.7 (7 links x ~153 GB/s per MI355X: a single ring is per-link bound,
the one-shot / multi-channel mesh is not). One JSON line per (op, size) on rank 0; the KB-sized
rows are the payloads of the latency-bound solver loops (LogReg gradient 24 KB, KMeans k=20
centroid sums), the MB rows the Gram / centroid all-reduces (36-72 MB).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def _size(s: str) -> int:
    s = s.strip().upper()
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    return int(float(s[:-1]) * mult[s[-1]]) if s[-1] in mult else int(s)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-bytes", default="1K")
    ap.add_argument("--max-bytes", default="64M")
    ap.add_argument("--factor", type=int, default=4)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--ops", default="all_reduce,all_gather,reduce_scatter,broadcast,all_to_all")
    ap.add_argument("--dtype", default="float32")
    ap.add_argument("--out", default=None, help="also append the JSON lines to this file (rank 0)")
    ap.add_argument("--backend", choices=("auto", "nccl", "gloo"), default="auto",
                    help="gloo with GPUs: ranks may share one device (one-shot rehearsal on a 1-GPU box)")
    ap.add_argument("--oneshot", action="store_true",
                    help="add the peer-mapped one-shot all-reduce (<= 256 KB) next to the collectives")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    gpu = torch.cuda.is_available() and os.environ.get("SRML_FORCE_CPU", "0") != "1"
    dev = torch.device("cuda", local % max(1, torch.cuda.device_count())) if gpu else torch.device("cpu")
    if gpu:
        torch.cuda.set_device(dev)
    if "MASTER_ADDR" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ.get("MASTER_PORT", "29531"))
    backend = a.backend if a.backend != "auto" else ("nccl" if gpu else "gloo")
    dist.init_process_group(backend, rank=rank, world_size=world, timeout=timedelta(minutes=10),
                            **({"device_id": dev} if backend == "nccl" else {}))
    oneshot = None
    if a.oneshot and gpu:
        from spark_rapids_ml_nai_amd.parallel.comm import Communicator
        from spark_rapids_ml_nai_amd.parallel.oneshot import MAX_BYTES, OneShotAllreduce

        oneshot = OneShotAllreduce(Communicator(rank, world, dev if backend == "nccl" else torch.device("cpu")), dev)
    dt = getattr(torch, a.dtype)
    esz = torch.tensor([], dtype=dt).element_size()
    sizes = []
    s = _size(a.min_bytes)
    while s <= _size(a.max_bytes):
        sizes.append(s)
        s *= a.factor

    def sync() -> None:
        if gpu:
            torch.cuda.synchronize(dev)

    n = world
    bus = {"all_reduce": 2 * (n - 1) / n, "all_gather": (n - 1) / n, "reduce_scatter": (n - 1) / n,
           "broadcast": 1.0, "all_to_all": (n - 1) / n, "oneshot_all_reduce": 2 * (n - 1) / n}
    ops = a.ops.split(",") + (["oneshot_all_reduce"] if oneshot is not None else [])
    rows = []
    for op in ops:
        for nbytes in sizes:
            if op == "oneshot_all_reduce" and nbytes > MAX_BYTES:
                continue
            cnt = max(n, nbytes // esz // n * n)
            x = torch.ones(cnt, dtype=dt, device=dev)
            if op == "all_reduce":
                f = lambda: dist.all_reduce(x)  # noqa: E731
            elif op == "oneshot_all_reduce":
                x = torch.ones(min(cnt, MAX_BYTES // 8), dtype=torch.float64, device=dev)
                f = lambda: oneshot.allreduce(x)  # noqa: E731
            elif op == "all_gather":
                out = torch.empty(cnt * n, dtype=dt, device=dev)
                f = lambda: dist.all_gather_into_tensor(out, x)  # noqa: E731
            elif op == "reduce_scatter":
                out = torch.empty(cnt // n, dtype=dt, device=dev)
                f = lambda: dist.reduce_scatter_tensor(out, x)  # noqa: E731
            elif op == "broadcast":
                f = lambda: dist.broadcast(x, 0)  # noqa: E731
            elif op == "all_to_all":
                out = torch.empty_like(x)
                f = lambda: dist.all_to_all_single(out, x)  # noqa: E731
            else:
                raise ValueError(op)
            for _ in range(a.warmup):
                f()
            sync()
            ts = []
            for _ in range(a.iters):
                dist.barrier()
                sync()
                t0 = time.perf_counter()
                f()
                sync()
                ts.append(time.perf_counter() - t0)
            t = torch.tensor([sorted(ts)[len(ts) // 2]], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            t = float(t.item())
            algbw = cnt * esz / t / 1e9
            row = {"op": op, "bytes": int(cnt * esz), "ranks": n, "backend": backend, "us": round(t * 1e6, 2),
                   "algbw_GBps": round(algbw, 3), "busbw_GBps": round(algbw * bus[op], 3)}
            rows.append(row)
            if rank == 0:
                print(json.dumps(row), flush=True)
    if oneshot is not None:
        oneshot.check()
        oneshot.close()
    if rank == 0 and a.out:
        with open(a.out, "a") as fh:
            for r in rows:
                fh.write(json.dumps(r) + "\n")
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
