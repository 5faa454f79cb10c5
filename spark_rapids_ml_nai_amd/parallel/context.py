"""Per-rank worker context: rank, world size, pinned device and communicator.

Equivalent of the reference's ``_CumlCommon._set_gpu_device`` + ``CumlContext``
(``core.py:343-388``, ``common/cuml_context.py:35-193``) and ``PartitionDescriptor``
(``utils.py:173-210``), re-designed for one process per MI355X:

* device pinning: ``cuda:<local_rank>`` (HIP device) from ``LOCAL_RANK`` / the Spark task's
  ``gpu`` resource / ``HIP_VISIBLE_DEVICES``; CPU when no GPU is visible (tests).
* communicator: ``torch.distributed`` group on RCCL (GPU) or gloo (CPU); bootstrap via
  env rendezvous (torchrun / LocalBarrierRunner) or Spark barrier ``allGather`` of the rank-0
  TCPStore address (see ``parallel/spark.py``).
* ``PartitionDescriptor``: global ``m``, ``n`` and per-rank row counts obtained with ONE
  device all-gather, not a JSON list through the Spark driver.
"""
from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field
from typing import Any, List, Optional

import torch
import torch.distributed as dist

from .comm import Communicator

_tls = threading.local()


def gpu_available() -> bool:
    if os.environ.get("SRML_FORCE_CPU", "0") == "1":
        return False
    try:
        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:  # noqa: BLE001
        return False


def local_device(local_rank: Optional[int] = None) -> torch.device:
    """Device this rank computes on."""
    if not gpu_available():
        return torch.device("cpu")
    n = torch.cuda.device_count()
    if local_rank is None:
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    return torch.device("cuda", local_rank % n)


def _parse_cpulist(text: str) -> List[int]:
    cpus: List[int] = []
    for part in text.strip().split(","):
        if not part:
            continue
        if "-" in part:
            a, b = part.split("-")
            cpus.extend(range(int(a), int(b) + 1))
        else:
            cpus.append(int(part))
    return cpus


_numa_bound: dict = {}


def bind_numa_local(device: torch.device) -> Optional[List[int]]:
    """Restrict this process's CPU affinity to the cores on the GPU's own NUMA node.

    Pinned host staging buffers are first-touch allocated on the node of the allocating thread,
    so a process left on the far socket pushes every host->device byte of the ingest across the
    inter-socket link as well as PCIe. Called before any staging buffer is allocated (worker
    device pinning, bench start). ``SRML_NUMA_BIND=0`` disables it; a failure leaves affinity
    unchanged. Returns the CPU list applied (None if nothing changed).
    """
    if device.type != "cuda" or os.environ.get("SRML_NUMA_BIND", "1") == "0" or not hasattr(os, "sched_setaffinity"):
        return None
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx in _numa_bound:
        return _numa_bound[idx]
    applied = None
    try:
        p = torch.cuda.get_device_properties(idx)
        bdf = "%04x:%02x:%02x.0" % (int(getattr(p, "pci_domain_id", 0)), int(p.pci_bus_id), int(p.pci_device_id))
        with open(f"/sys/bus/pci/devices/{bdf}/local_cpulist") as f:
            local = set(_parse_cpulist(f.read()))
        cur = os.sched_getaffinity(0)
        want = sorted(local & cur)
        if want and set(want) != cur:
            os.sched_setaffinity(0, want)
            applied = want
    except Exception:  # noqa: BLE001 - topology info is best-effort
        applied = None
    _numa_bound[idx] = applied
    return applied


def spmd_active() -> bool:
    """True when the caller already runs one process per GPU inside a torch.distributed world."""
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def spmd_row_offset(n_local: int) -> int:
    """This rank's first global row index in an SPMD job: the exclusive prefix sum of every rank's
    local row count (ONE small all-gather; 0 outside SPMD). Collective: every rank must call it.
    Gives a rank-local frame globally unique, rank-major row ids (the torchrun counterpart of
    Spark's partition-major ``monotonically_increasing_id``)."""
    if not spmd_active():
        return 0
    ctx = current_context() or spmd_context()
    t = torch.tensor([int(n_local)], dtype=torch.int64, device=ctx.device)
    sizes = ctx.comm.allgather(t).tolist()
    return int(sum(sizes[: ctx.rank]))


def infer_num_workers() -> int:
    if spmd_active():
        return dist.get_world_size()
    env = os.environ.get("SRML_NUM_WORKERS")
    if env:
        return int(env)
    if gpu_available():
        return torch.cuda.device_count()
    return 1


@dataclass
class WorkerContext:
    rank: int = 0
    world_size: int = 1
    device: torch.device = field(default_factory=lambda: torch.device("cpu"))
    comm: Communicator = field(default_factory=Communicator)
    partition_id: int = 0
    timers: dict = field(default_factory=dict)
    # transform-evaluate passes set this: predict functions then hand back device tensors (the
    # metric partials are computed where the predictions are) instead of host arrays
    device_outputs: bool = False

    @property
    def distributed(self) -> bool:
        """The fit takes the multi-rank code path: world_size > 1, or a one-rank communicator over
        a live process group (``SRML_COMM_FORCE_PG=1``: the per-rank proxy runs the collectives and
        the multi-rank kernels of an N-GPU fit on one GPU)."""
        return self.world_size > 1 or not getattr(self.comm, "_solo", True)

    @property
    def is_gpu(self) -> bool:
        return self.device.type == "cuda"

    def output(self, t: torch.Tensor) -> Any:
        """A predict function's output column: the device tensor itself in a transform-evaluate
        pass (``device_outputs``), otherwise a host numpy array."""
        return t if self.device_outputs else t.cpu().numpy()

    def sync(self) -> None:
        if self.is_gpu:
            torch.cuda.synchronize(self.device)

    @staticmethod
    def single(device: Optional[torch.device] = None) -> "WorkerContext":
        dev = device if device is not None else local_device()
        if dev.type == "cuda":
            bind_numa_local(dev)
        return WorkerContext(0, 1, dev, Communicator(0, 1, dev))

    @staticmethod
    def from_process_group(device: Optional[torch.device] = None) -> "WorkerContext":
        rank, size = dist.get_rank(), dist.get_world_size()
        dev = device if device is not None else local_device()
        if dev.type == "cuda":
            torch.cuda.set_device(dev)
            bind_numa_local(dev)
        return WorkerContext(rank, size, dev, Communicator(rank, size, dev), partition_id=rank)


_SPMD: List[Any] = []  # [(world group, WorkerContext)] of the live process group


def spmd_context() -> WorkerContext:
    """The rank's context in an SPMD job (torchrun / Spark barrier group), built once per process
    group: every fit of the job reuses one Communicator, so its lazily mapped one-shot buffers and
    its accounting persist instead of being re-created per fit."""
    grp = dist.group.WORLD
    if _SPMD and _SPMD[0][0] is grp and not _SPMD[0][1].comm.aborted:
        return _SPMD[0][1]
    ctx = WorkerContext.from_process_group()
    _SPMD[:] = [(grp, ctx)]
    return ctx


def current_context() -> Optional[WorkerContext]:
    return getattr(_tls, "ctx", None)


class use_context:
    def __init__(self, ctx: WorkerContext) -> None:
        self.ctx = ctx
        self.prev: Optional[WorkerContext] = None

    def __enter__(self) -> WorkerContext:
        self.prev = current_context()
        _tls.ctx = self.ctx
        return self.ctx

    def __exit__(self, *exc: Any) -> None:
        _tls.ctx = self.prev


@dataclass
class PartitionDescriptor:
    """Global layout of the row-partitioned input (reference ``utils.py:173-210``)."""

    m: int
    n: int
    rank: int
    parts_rank_size: List[tuple]

    @classmethod
    def build(cls, ctx: WorkerContext, local_rows: int, n_cols: int) -> "PartitionDescriptor":
        t = torch.tensor([local_rows, n_cols], dtype=torch.int64, device=ctx.device)
        g = ctx.comm.allgather(t.view(1, 2)).view(-1, 2).cpu().tolist()
        ns = {int(r[1]) for r in g if r[0] > 0}
        if len(ns) > 1:
            raise ValueError("ranks disagree on the number of columns: %s" % ns)
        n = ns.pop() if ns else n_cols
        parts = [(r, int(g[r][0])) for r in range(ctx.world_size)]
        return cls(sum(p[1] for p in parts), n, ctx.rank, parts)
