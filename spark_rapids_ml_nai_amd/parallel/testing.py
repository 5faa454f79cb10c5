"""Multi-process stand-in for Spark's ``BarrierTaskContext`` (``partitionId / allGather /
barrier / resources``) so the Spark barrier worker path (``parallel/spark.py``) can be exercised
without a JVM: each partition runs in its own spawned process, exactly one task per rank."""
from __future__ import annotations

import multiprocessing as mp
import traceback
from typing import Any, Dict, List

import cloudpickle


class FakeBarrierTaskContext:
    def __init__(self, rank: int, world: int, board: Any, barrier: Any) -> None:
        self._rank, self._world, self._board, self._barrier = rank, world, board, barrier
        self._round = 0

    def partitionId(self) -> int:
        return self._rank

    def resources(self) -> Dict[str, Any]:
        return {}

    def barrier(self) -> None:
        self._barrier.wait()

    def allGather(self, message: str = "") -> List[str]:
        key = self._round
        self._round += 1
        self._board[(key, self._rank)] = message
        self._barrier.wait()
        out = [self._board[(key, r)] for r in range(self._world)]
        self._barrier.wait()
        return out


def _task(rank: int, world: int, board: Any, barrier: Any, blob: bytes, q: Any) -> None:
    import os

    os.environ["SRML_FORCE_CPU"] = "1"
    os.environ["SRML_RENDEZVOUS_HOST"] = "127.0.0.1"
    try:
        fn, parts = cloudpickle.loads(blob)
        ctx = FakeBarrierTaskContext(rank, world, board, barrier)
        out = list(fn(ctx, iter(parts[rank])))
        q.put((rank, "ok", cloudpickle.dumps(out)))
    except BaseException:  # noqa: BLE001
        q.put((rank, "err", traceback.format_exc()))


def run_fake_barrier_stage(fn: Any, partitions: List[List[Any]], timeout_s: float = 600.0) -> List[Any]:
    """Run ``fn(task_ctx, batch_iterator)`` for every partition; returns the yielded rows in rank order."""
    world = len(partitions)
    mpc = mp.get_context("spawn")
    with mpc.Manager() as mgr:
        board = mgr.dict()
        barrier = mgr.Barrier(world)
        q = mpc.Queue()
        blob = cloudpickle.dumps((fn, partitions))
        procs = [mpc.Process(target=_task, args=(r, world, board, barrier, blob, q)) for r in range(world)]
        for p in procs:
            p.start()
        results: Dict[int, Any] = {}
        errors = []
        for _ in range(world):
            rank, status, body = q.get(timeout=timeout_s)
            if status == "ok":
                results[rank] = cloudpickle.loads(body)
            else:
                errors.append("rank %d:\n%s" % (rank, body))
                break
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
        if errors:
            raise RuntimeError("barrier stage failed: " + "\n".join(errors))
    return [row for r in range(world) for row in results[r]]
