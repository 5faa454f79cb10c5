"""LocalBarrierRunner: an N-process barrier job without Spark.

The reference runs its per-GPU fit closure inside Spark barrier-mode ``mapInPandas`` tasks
(``core.py:694-785``) and bootstraps NCCL through ``BarrierTaskContext.allGather``. Spark is an
optional dependency of this framework, so the same "one task per GPU, all-or-nothing" stage is
provided natively: N worker processes (one per MI355X, or CPU ranks on gloo), a loopback
TCP rendezvous, ``torch.distributed`` over RCCL/gloo, the closure shipped with cloudpickle
(as Spark ships UDFs) and rank results returned to the caller. Barrier semantics are kept: if
any rank raises, the others are torn down and the whole job fails with that traceback.
"""
from __future__ import annotations

import os
import socket
import traceback
from datetime import timedelta
from typing import Any, Callable, List, Optional, Sequence

import cloudpickle


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _child(rank: int, world: int, port: int, use_gpu: bool, payload: bytes, q: Any, timeout_s: float) -> None:
    os.environ.update(
        MASTER_ADDR="127.0.0.1",
        MASTER_PORT=str(port),
        RANK=str(rank),
        WORLD_SIZE=str(world),
        LOCAL_RANK=str(rank),
    )
    if not use_gpu:
        os.environ["SRML_FORCE_CPU"] = "1"
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    import torch
    import torch.distributed as dist

    from .comm import comm_timeout
    from .context import WorkerContext, local_device, use_context

    ctx = None
    try:
        device = local_device(rank) if use_gpu else torch.device("cpu")
        if device.type == "cuda":
            torch.cuda.set_device(device)
            from .context import bind_numa_local

            bind_numa_local(device)
        # RCCL needs one device per rank: more workers than visible GPUs (ranks sharing a device,
        # e.g. num_workers=2 on a one-GPU box) run their collectives over gloo instead
        rccl = device.type == "cuda" and world <= torch.cuda.device_count()
        dist.init_process_group(
            "nccl" if rccl else "gloo",
            rank=rank,
            world_size=world,
            timeout=timedelta(seconds=comm_timeout(timeout_s)),
            **({"device_id": device} if rccl else {}),
        )
        ctx = WorkerContext.from_process_group(device)
        fn, inp = cloudpickle.loads(payload)
        with use_context(ctx):
            res = fn(ctx, inp)
        ctx.comm.barrier()
        q.put((rank, "ok", cloudpickle.dumps(res)))
    except BaseException:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))
        if ctx is not None:
            ctx.comm.abort()
        return
    try:
        dist.destroy_process_group()
    except Exception:  # noqa: BLE001
        pass


def run_barrier_job(
    fn: Callable[[Any, Any], Any],
    per_rank_inputs: Sequence[Any],
    use_gpu: Optional[bool] = None,
    timeout_s: float = 1800.0,
) -> List[Any]:
    """Run ``fn(ctx, per_rank_inputs[rank])`` on ``len(per_rank_inputs)`` ranks; return all results."""
    import multiprocessing as mp

    from .context import gpu_available

    world = len(per_rank_inputs)
    timeout_s = float(os.environ.get("SRML_BARRIER_TIMEOUT", timeout_s))
    if use_gpu is None:
        use_gpu = gpu_available()
    # always spawn: forking a process whose torch CPU thread pool (OpenMP) or HIP runtime is
    # already initialised deadlocks the child inside its first parallel op
    method = os.environ.get("SRML_MP_START", "spawn")
    mpctx = mp.get_context(method)
    q = mpctx.Queue()
    port = free_port()
    procs = []
    for r in range(world):
        payload = cloudpickle.dumps((fn, per_rank_inputs[r]))
        p = mpctx.Process(target=_child, args=(r, world, port, use_gpu, payload, q, timeout_s), daemon=False)
        p.start()
        procs.append(p)
    results: List[Any] = [None] * world
    errors: List[str] = []
    got = 0
    import queue as _queue

    import time as _time

    deadline = _time.monotonic() + timeout_s
    while got < world:
        try:
            rank, status, body = q.get(timeout=1.0)
        except _queue.Empty:
            # watchdog: a rank that died without reporting fails the whole barrier stage
            dead = [i for i, p in enumerate(procs) if not p.is_alive() and p.exitcode not in (0, None)]
            if dead:
                errors.append("rank(s) %s exited with code(s) %s before reporting"
                              % (dead, [procs[i].exitcode for i in dead]))
                break
            if _time.monotonic() > deadline:
                errors.append("barrier job timed out after %.0fs" % timeout_s)
                break
            continue
        got += 1
        if status == "ok":
            results[rank] = cloudpickle.loads(body)
        else:
            errors.append("rank %d failed:\n%s" % (rank, body))
            break
    if errors:
        # a peer's error is often just the symptom (its collective saw the connection drop):
        # name any rank that died first so the root cause is in the message
        if not any("exited with code" in e for e in errors):
            _time.sleep(0.5)
            dead = [i for i, p in enumerate(procs) if not p.is_alive() and p.exitcode not in (0, None)]
            if dead:
                errors.insert(0, "rank(s) %s exited with code(s) %s" % (dead, [procs[i].exitcode for i in dead]))
        for p in procs:
            if p.is_alive():
                p.terminate()
        for p in procs:
            p.join(timeout=10)
        raise RuntimeError("barrier job failed: " + "\n".join(errors))
    for p in procs:
        p.join(timeout=60)
        if p.is_alive():
            p.terminate()
    return results
