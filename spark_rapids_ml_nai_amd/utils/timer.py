"""Phase timers + roctx ranges.

Each fit records wall time per phase (ingest, fit, per-algorithm stages); with
``SRML_PROFILE=1`` every phase is also pushed as a roctx range so rocprofv3
``--marker-trace`` timelines show ingest / H2D / kernels / RCCL per rank (the reference only
has NVTX ranges in its Scala PCA, ``RapidsRowMatrix.scala:62-89``).
"""
from __future__ import annotations

import ctypes
import os
import time
from contextlib import contextmanager
from typing import Dict, Iterator, Optional

_roctx = None


def _roctx_lib() -> Optional[ctypes.CDLL]:
    global _roctx
    if _roctx is None:
        _roctx = False
        if os.environ.get("SRML_PROFILE", "0") == "1":
            for name in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
                try:
                    lib = ctypes.CDLL(name)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    _roctx = lib
                    break
                except OSError:
                    continue
    return _roctx or None


@contextmanager
def range_push(name: str) -> Iterator[None]:
    lib = _roctx_lib()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


class PhaseTimer:
    def __init__(self, sync_device: Optional[object] = None) -> None:
        self.times: Dict[str, float] = {}
        self.sync_device = sync_device
        self.rank_stats: Optional[dict] = None  # this rank's wall / H2D / compute / comm split of the fit

    @contextmanager
    def phase(self, name: str) -> Iterator[None]:
        t0 = time.perf_counter()
        with range_push(name):
            try:
                yield
            finally:
                if self.sync_device is not None:
                    import torch

                    torch.cuda.synchronize(self.sync_device)
                self.times[name] = self.times.get(name, 0.0) + time.perf_counter() - t0
