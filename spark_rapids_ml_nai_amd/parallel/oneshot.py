"""One-shot small-message all-reduce over peer-mapped device buffers (``ops/csrc/oneshot.hip``).

Selected by ``spark.rocm.ml.comm`` / ``SRML_COMM`` = ``oneshot | rccl | auto`` (default ``rccl``):
``oneshot`` routes every all-reduce of <= ``SRML_ONESHOT_MAX_BYTES`` (256 KB) through it;
``auto`` does so only when all ranks share one node (``single_node``). Larger payloads and any
failure to set it up (agreed across ranks) fall back to RCCL.

Setup (once per communicator): each rank allocates its uncached exchange buffer, exports the IPC
handle, the 64-byte handles are all-gathered over the process group, every rank opens its
peers' buffers and keeps a device array of the W pointers. A call is ONE kernel: publish,
flag, bounded wait for all peers, read all W payloads over xGMI, sum in rank order.

The epoch / double-slot protocol is mirrored on the host by ``HostOneShot`` (threads over shared
numpy buffers) for the CPU tests.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Any, List

import numpy as np
import torch

from ..ops import native

MAX_BYTES = int(os.environ.get("SRML_ONESHOT_MAX_BYTES", str(256 * 1024)))
TIMEOUT_S = float(os.environ.get("SRML_ONESHOT_TIMEOUT_S", "10"))
_WALLCLOCK_HZ = 100e6  # s_memrealtime / wall_clock64 on CDNA3/4
MODES = ("rccl", "oneshot", "auto")


def comm_mode() -> str:
    """``SRML_COMM`` (set from the Spark conf ``spark.rocm.ml.comm`` on the workers)."""
    m = os.environ.get("SRML_COMM", "rccl").lower()
    if m not in MODES:
        raise ValueError("SRML_COMM / spark.rocm.ml.comm must be one of %s, got %r" % (MODES, m))
    return m


def single_node(comm: Any) -> bool:
    """Whether every rank of ``comm`` runs on this host (peer-mappable device memory)."""
    import socket

    if int(os.environ.get("LOCAL_WORLD_SIZE", "0") or 0) == comm.size:
        return True
    hosts = comm.allgather_object(socket.gethostname())
    return len(set(hosts)) == 1


class OneShotAllreduce:
    """Peer-mapped one-shot all-reduce for one process group (one rank per GPU).

    Construction never raises and never leaves ranks out of step: every rank takes part in the
    handle exchange even if its own allocation failed, and the ranks then agree (a MIN all-reduce
    on the group's own backend) whether the set-up worked everywhere; ``ok`` is that verdict.

    Errors: a call whose peers do not arrive within ``SRML_ONESHOT_TIMEOUT_S`` sets the sticky
    device error word; that call and every later one on the rank write NaN (never a silent local
    partial) and stop publishing, so the peers time out as well. ``poll()`` (non-blocking) and
    ``failed()`` (blocking) read the word; ``Communicator.poll/check`` turn it into ``CommError``."""

    def __init__(self, comm: Any, device: torch.device, max_bytes: int = MAX_BYTES) -> None:
        self.comm = comm
        self.device = device
        self.world = comm.size
        self.rank = comm.rank
        self.max_elems = max(1, max_bytes // 8)
        self.epoch = 0
        self._peers: List[int] = []
        self._own = None
        self.reason = ""
        ok = True
        handle = (ctypes.c_char * 64)()
        try:
            lib = native.lib()
            ptr = ctypes.c_void_p()
            with torch.cuda.device(device):
                rc = lib.srml_oneshot_alloc(self.max_elems, ctypes.byref(ptr), handle)
            if rc != 0:
                ok, self.reason = False, "srml_oneshot_alloc failed with HIP status %d" % rc
            else:
                self._own = ptr.value
        except Exception as e:  # noqa: BLE001
            ok, self.reason = False, repr(e)
        handles = comm.allgather_bytes(bytes(handle) if ok else b"\0" * 64)
        ptrs = []
        if ok:
            for r, h in enumerate(handles):
                if r == self.rank:
                    ptrs.append(self._own)
                    continue
                pp = ctypes.c_void_p()
                hb = (ctypes.c_char * 64).from_buffer_copy(h)
                with torch.cuda.device(device):
                    rc = lib.srml_oneshot_open(hb, ctypes.byref(pp))
                if rc != 0:
                    ok, self.reason = False, "srml_oneshot_open(rank %d) failed with HIP status %d" % (r, rc)
                    break
                self._peers.append(pp.value)
                ptrs.append(pp.value)
        flag = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=comm.device)
        comm.allreduce(flag, op="min")  # the one-shot path is not set yet: this goes over RCCL/gloo
        self.ok = bool(flag.item() > 0)
        if not self.ok:
            self.reason = self.reason or "a peer could not map the exchange buffers"
            self.close()
            return
        self._bufs = torch.tensor(ptrs, dtype=torch.int64, device=device)
        self._err = torch.zeros(1, dtype=torch.int32, device=device)
        self._host_err = torch.zeros(2, dtype=torch.int32, pin_memory=True)
        self._pending: List[Any] = []
        self._npoll = 0
        self._timeout = int(TIMEOUT_S * _WALLCLOCK_HZ)
        comm.barrier()  # every buffer is open before the first flag is raised

    def allreduce(self, t: torch.Tensor) -> torch.Tensor:
        """In-place sum over ranks of a contiguous fp32/fp64 device tensor (<= max_elems)."""
        n = t.numel()
        if n > self.max_elems or t.dtype not in (torch.float32, torch.float64) or not t.is_contiguous():
            raise ValueError("one-shot all-reduce: unsupported payload")
        self.epoch += 1
        native.call("srml_oneshot_allreduce", t.data_ptr(), t.data_ptr(), n, 1 if t.dtype == torch.float64 else 0,
                    self._bufs.data_ptr(), self.world, self.rank, self.epoch, self.max_elems, self._timeout,
                    self._err.data_ptr(), native.stream(t.device))
        return t

    def poll(self) -> bool:
        """Non-blocking: queue a copy of the error word and report the copies that have landed
        (True = a call issued before one of the earlier polls failed)."""
        failed = False
        while self._pending and self._pending[0][0].query():
            _, s0 = self._pending.pop(0)
            failed |= int(s0.item()) != 0
        if len(self._pending) < 2:  # two pinned slots, used alternately
            k = self._npoll % 2
            self._npoll += 1
            slot = self._host_err[k: k + 1]
            slot.copy_(self._err, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream(self.device))
            self._pending.append((ev, slot))
        return failed

    def failed(self) -> bool:
        """Blocking: whether any call so far timed out waiting for a peer."""
        return int(self._err.item()) != 0

    def check(self) -> None:
        """Raise if any call so far timed out waiting for a peer (synchronises)."""
        if self.failed():
            raise RuntimeError("one-shot all-reduce: a peer did not arrive within %.1f s" % TIMEOUT_S)

    def close(self) -> None:
        lib = native.lib()
        for p in self._peers:
            lib.srml_oneshot_close(ctypes.c_void_p(p))
        self._peers = []
        if getattr(self, "_own", None):
            lib.srml_oneshot_free(ctypes.c_void_p(self._own))
            self._own = None


class HostOneShot:
    """Host mirror of the kernel's protocol for W in-process ranks (threads): per rank a flag and two
    payload slots; epoch e publishes into slot e & 1, raises the flag, waits for every peer's flag
    >= e and sums the W slots in rank order."""

    def __init__(self, world: int, max_elems: int) -> None:
        self.world = world
        self.max_elems = max_elems
        self.flags = [0] * world
        self.slots = [np.zeros((2, max_elems)) for _ in range(world)]
        self.cv = threading.Condition()

    def allreduce(self, rank: int, epoch: int, x: np.ndarray, timeout: float = 10.0) -> np.ndarray:
        n = x.shape[0]
        s = epoch & 1
        self.slots[rank][s, :n] = x
        with self.cv:
            self.flags[rank] = epoch
            self.cv.notify_all()
            if not self.cv.wait_for(lambda: min(self.flags) >= epoch, timeout=timeout):
                raise TimeoutError("peer did not arrive")
        out = np.zeros(n)
        for p in range(self.world):
            out += self.slots[p][s, :n]
        return out
