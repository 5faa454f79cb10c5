"""One-shot small-message all-reduce over peer-mapped device buffers (``ops/csrc/oneshot.hip``).

Selected by ``spark.rocm.ml.comm`` / ``SRML_COMM`` = ``oneshot | rccl | auto`` (default ``rccl``):
``oneshot`` routes every all-reduce of <= ``SRML_ONESHOT_MAX_BYTES`` (256 KB) through it;
``auto`` does so only when all ranks share one node and peer access works. Larger payloads and
any failure to set it up fall back to RCCL.

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


def comm_mode() -> str:
    return os.environ.get("SRML_COMM", "rccl").lower()


class OneShotAllreduce:
    """Peer-mapped one-shot all-reduce for one process group (one rank per GPU)."""

    def __init__(self, comm: Any, device: torch.device, max_bytes: int = MAX_BYTES) -> None:
        self.comm = comm
        self.device = device
        self.world = comm.size
        self.rank = comm.rank
        self.max_elems = max(1, max_bytes // 8)
        self.epoch = 0
        self._peers: List[int] = []
        lib = native.lib()
        ptr = ctypes.c_void_p()
        handle = (ctypes.c_char * 64)()
        with torch.cuda.device(device):
            rc = lib.srml_oneshot_alloc(self.max_elems, ctypes.byref(ptr), handle)
        if rc != 0:
            raise RuntimeError("srml_oneshot_alloc failed with HIP status %d" % rc)
        self._own = ptr.value
        handles = comm.allgather_bytes(bytes(handle))
        ptrs = []
        for r, h in enumerate(handles):
            if r == self.rank:
                ptrs.append(self._own)
                continue
            pp = ctypes.c_void_p()
            hb = (ctypes.c_char * 64).from_buffer_copy(h)
            with torch.cuda.device(device):
                rc = lib.srml_oneshot_open(hb, ctypes.byref(pp))
            if rc != 0:
                self.close()
                raise RuntimeError("srml_oneshot_open(rank %d) failed with HIP status %d" % (r, rc))
            self._peers.append(pp.value)
            ptrs.append(pp.value)
        self._bufs = torch.tensor(ptrs, dtype=torch.int64, device=device)
        self._err = torch.zeros(1, dtype=torch.int32, device=device)
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

    def check(self) -> None:
        """Raise if any call so far timed out waiting for a peer (synchronises)."""
        if int(self._err.item()) != 0:
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
