"""Host -> device ingest with pinned staging and overlapped H2D.

The reference converts each Arrow batch through a per-row Python list and (optionally) copies
to the GPU (``core.py:724-748``) — the dominant host cost at 1M x 3000. Here the numpy view of
the Arrow values buffer is copied into a small ring of pinned staging buffers and DMA'd to a
pre-allocated device tensor with ``non_blocking`` copies: while chunk i is in flight over PCIe
the host fills chunk i+1 (two buffers, event-guarded reuse). Small arrays take the direct path.
"""
from __future__ import annotations

import os

import warnings
from typing import Any, Iterator, Optional

import numpy as np
import torch

_CHUNK_BYTES = 64 << 20
_DIRECT_BYTES = 8 << 20
_staging: dict = {}


def _pinned(device: torch.device, slot: int, nbytes: int) -> torch.Tensor:
    key = (device.index, slot)
    buf = _staging.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(max(nbytes, _CHUNK_BYTES), dtype=torch.uint8, pin_memory=True)
        _staging[key] = buf
    return buf


def _dense_to_device(a: np.ndarray, device: torch.device, dtype: Optional[torch.dtype]) -> torch.Tensor:
    with warnings.catch_warnings():
        # Arrow buffers are read-only; we only ever read them
        warnings.simplefilter("ignore", UserWarning)
        t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None and t.dtype != dtype and not t.dtype.is_floating_point:
        t = t.to(dtype)
    elif dtype is not None and t.dtype != dtype:
        t = t.to(dtype)
    if device.type != "cuda":
        return t.to(device)
    if uvm_enabled() and t.dim() >= 1 and t.numel() * t.element_size() > _DIRECT_BYTES:
        # UVM mode: the device copy lives in managed memory (pages migrate on demand)
        out = managed_empty(t.shape, t.dtype, device)
        out.copy_(t, non_blocking=t.is_pinned())
        return out
    if t.is_pinned():
        # Arrow batch already in page-locked memory: one DMA straight into HBM
        return t.to(device, non_blocking=True)
    nbytes = t.numel() * t.element_size()
    if nbytes <= _DIRECT_BYTES or t.dim() == 0:
        return t.to(device, non_blocking=False)
    out = torch.empty(t.shape, dtype=t.dtype, device=device)
    flat_src = t.reshape(-1).view(torch.uint8)
    flat_dst = out.reshape(-1).view(torch.uint8)
    stream = torch.cuda.current_stream(device)
    events = [None, None]
    off = 0
    slot = 0
    while off < nbytes:
        n = min(_CHUNK_BYTES, nbytes - off)
        if events[slot] is not None:
            events[slot].synchronize()
        buf = _pinned(device, slot, _CHUNK_BYTES)
        buf[:n].copy_(flat_src[off: off + n])
        flat_dst[off: off + n].copy_(buf[:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(stream)
        events[slot] = ev
        off += n
        slot ^= 1
    for ev in events:
        if ev is not None:
            ev.synchronize()
    return out


# ------------------------------------------------------------------------------------------
# Batch-stream ingest: many pageable row blocks (Spark Arrow batches) -> one device matrix
# ------------------------------------------------------------------------------------------
_RING_SLOTS = 3
_ring: dict = {}  # device index -> [(pinned uint8 buffer, event or None)] * slots
_pool = None


def _ingest_threads() -> int:
    return max(1, int(os.environ.get("SRML_INGEST_THREADS", str(min(8, os.cpu_count() or 1)))))


def _thread_pool() -> Any:
    global _pool
    from concurrent.futures import ThreadPoolExecutor

    n = _ingest_threads()
    if _pool is None or _pool._max_workers != n:
        _pool = ThreadPoolExecutor(max_workers=n, thread_name_prefix="srml-ingest")
    return _pool


def parts_to_device(parts: Any, device: torch.device, dtype: Optional[torch.dtype] = None,
                    mode: Optional[str] = None) -> torch.Tensor:
    """Row blocks (list of (rows_i, n) arrays, or ``ChunkedRows``) -> one (sum rows_i, n) device
    tensor, never concatenating them on the host.

    ``staged`` (default): a ring of pinned buffers; each is filled by ``SRML_INGEST_THREADS``
    threads (numpy copies release the GIL; the element-type cast, if any, happens in the same
    copy) and DMA'd on the high-priority copy stream while the next one fills. ``register``: each
    block is page-locked in place (hipHostRegister), DMA'd directly and unregistered. The compute
    stream waits for the last copy on the device; the host never blocks on the transfer except to
    recycle a ring slot."""
    blocks = list(getattr(parts, "parts", parts))
    blocks = [np.ascontiguousarray(b) for b in blocks if b.shape[0] > 0]
    if not blocks:
        raise ValueError("no rows")
    n = int(blocks[0].shape[1])
    rows = int(sum(b.shape[0] for b in blocks))
    np_dt = blocks[0].dtype if dtype is None else {torch.float32: np.dtype(np.float32),
                                                    torch.float64: np.dtype(np.float64)}[dtype]
    tdt = torch.from_numpy(np.zeros(0, dtype=np_dt)).dtype
    if device.type != "cuda":
        return torch.from_numpy(np.concatenate(blocks, 0).astype(np_dt, copy=False)).to(device)
    mode = mode or os.environ.get("SRML_INGEST_MODE", "staged")
    out = torch.empty((rows, n), dtype=tdt, device=device)
    cur = torch.cuda.current_stream(device)
    cs = copy_stream(device)
    cs.wait_stream(cur)
    out.record_stream(cs)
    if mode == "register" and all(b.dtype == np_dt for b in blocks):
        cudart = torch.cuda.cudart()
        regs = []
        r0 = 0
        with torch.cuda.stream(cs):
            for b in blocks:
                cudart.cudaHostRegister(b.ctypes.data, b.nbytes, 0)
                regs.append(b)
                with warnings.catch_warnings():
                    warnings.simplefilter("ignore", UserWarning)
                    out[r0: r0 + b.shape[0]].copy_(torch.from_numpy(b), non_blocking=True)
                r0 += b.shape[0]
        cs.synchronize()  # blocks must stay registered until their DMA has landed
        for b in regs:
            cudart.cudaHostUnregister(b.ctypes.data)
        cur.wait_stream(cs)
        return out
    for _ in _staged_fill(blocks, out, device, cs):
        pass
    cur.wait_stream(cs)
    return out


def _staged_fill(blocks: list, out: torch.Tensor, device: torch.device, cs: "torch.cuda.Stream") -> Iterator[Any]:
    """Generator: fill the pinned ring slot by slot from the row blocks (threaded copies, cast on
    the fly), DMA each slot into ``out`` on ``cs``; yields (row0, row1, event) per slot."""
    rows, n = out.shape
    tdt = out.dtype
    esz = out.element_size()
    idx = device.index if device.index is not None else torch.cuda.current_device()
    slot_bytes = int(os.environ.get("SRML_INGEST_SLOT_MB", "64")) << 20
    ring = _ring.get(idx)
    if ring is None or ring[0][0].numel() < slot_bytes:
        ring = [[torch.empty(slot_bytes, dtype=torch.uint8, pin_memory=True), None] for _ in range(_RING_SLOTS)]
        _ring[idx] = ring
    slot_rows = max(1, slot_bytes // (n * esz))
    flat_out = out.view(-1)
    pool = _thread_pool()
    nth = _ingest_threads()
    s_i = 0
    row_out = 0
    bi, br = 0, 0  # block index, row within block
    while row_out < rows:
        buf, ev = ring[s_i]
        if ev is not None:
            ev.synchronize()
        stage = buf[: slot_rows * n * esz].view(tdt).view(slot_rows, n).numpy()
        jobs = []
        filled = 0
        while filled < slot_rows and bi < len(blocks):
            b = blocks[bi]
            take = min(slot_rows - filled, b.shape[0] - br)
            jobs.append((stage[filled: filled + take], b[br: br + take]))
            filled += take
            br += take
            if br == b.shape[0]:
                bi, br = bi + 1, 0
        pieces = []
        for dst, src in jobs:  # split every copy over the threads by rows
            step = max(1, -(-dst.shape[0] // nth))
            for r in range(0, dst.shape[0], step):
                pieces.append((dst[r: r + step], src[r: r + step]))
        list(pool.map(lambda ds: np.copyto(ds[0], ds[1], casting="unsafe"), pieces))
        with torch.cuda.stream(cs):
            flat_out[row_out * n: (row_out + filled) * n].copy_(buf[: filled * n * esz].view(tdt), non_blocking=True)
            e = torch.cuda.Event(enable_timing=True)  # timed: the exposed-H2D accounting reads it
            e.record(cs)
        ring[s_i][1] = e
        yield row_out, row_out + filled, e
        row_out += filled
        s_i = (s_i + 1) % _RING_SLOTS


class StreamedParts:
    """``StreamedRows`` for a multi-batch pageable partition (``ChunkedRows``): ``chunks()`` fills
    and DMAs the pinned ring slot by slot and yields each slot's rows as soon as its copy is queued,
    so the first pass (moments / Gram / X^T y) runs on slot i while slot i+1 is being filled and
    copied; ``wait_all()`` finishes the transfer (host fill + device ordering)."""

    def __init__(self, parts: Any, device: torch.device, dtype: Optional[torch.dtype] = None) -> None:
        blocks = [np.ascontiguousarray(b) for b in getattr(parts, "parts", parts) if b.shape[0] > 0]
        n = int(blocks[0].shape[1])
        rows = int(sum(b.shape[0] for b in blocks))
        np_dt = blocks[0].dtype if dtype is None else {torch.float32: np.dtype(np.float32),
                                                        torch.float64: np.dtype(np.float64)}[dtype]
        tdt = torch.from_numpy(np.zeros(0, dtype=np_dt)).dtype
        self.device = device
        cur = torch.cuda.current_stream(device)
        self.X = torch.empty((rows, n), dtype=tdt, device=device)
        self._copy = copy_stream(device)
        self._copy.wait_stream(cur)
        self.X.record_stream(self._copy)
        self._t0 = torch.cuda.Event(enable_timing=True)
        self._t1: Optional[Any] = None
        self._t0.record(self._copy)
        self._gen = _staged_fill(blocks, self.X, device, self._copy)
        self._last = None
        self._stalls: list = []  # (compute-stream event before a wait, the copy event it waits on)

    def _finished(self) -> None:
        if self._t1 is None:
            self._t1 = torch.cuda.Event(enable_timing=True)
            self._t1.record(self._copy)

    def h2d_seconds(self) -> float:
        """Copy-stream span of the transfer (host fill of the staging ring included)."""
        self.wait_all()
        assert self._t1 is not None
        self._t1.synchronize()
        return self._t0.elapsed_time(self._t1) / 1e3

    def chunks(self) -> Iterator[Any]:
        cur = torch.cuda.current_stream(self.device)
        for r0, r1, ev in self._gen:
            self._last = ev
            _timed_wait(cur, ev, self._stalls)
            yield r0, r1, self.X[r0:r1]
        self._finished()

    def wait_all(self) -> torch.Tensor:
        for _, _, ev in self._gen:
            self._last = ev
        self._finished()
        if self._last is not None:
            _timed_wait(torch.cuda.current_stream(self.device), self._last, self._stalls)
        return self.X

    def exposed_seconds(self) -> float:
        """Time the compute stream stood waiting for this transfer (the H2D NOT hidden under
        compute); call after the fit has synchronised."""
        return _stall_seconds(self._stalls)


def _timed_wait(cur: "torch.cuda.Stream", ev: Any, stalls: list) -> None:
    """``cur.wait_event(ev)`` with a timing event recorded on ``cur`` just before it: the gap
    t(ev) - t(before), when positive, is how long the compute stream stood at this wait."""
    before = torch.cuda.Event(enable_timing=True)
    before.record(cur)
    cur.wait_event(ev)
    stalls.append((before, ev))


def _stall_seconds(stalls: list) -> float:
    tot = 0.0
    for before, ev in stalls:
        ev.synchronize()
        before.synchronize()
        tot += max(0.0, before.elapsed_time(ev)) / 1e3
    return tot


def host_to_device(X: Any, device: torch.device, dtype: Optional[torch.dtype] = None) -> Any:
    """numpy dense / ``ChunkedRows`` / scipy CSR / torch tensor -> device tensor (or ``core.base.CSR``)."""
    import scipy.sparse as sp

    if hasattr(X, "parts") and getattr(X, "ndim", 0) == 2:  # ChunkedRows (multi-batch partition)
        return parts_to_device(X, device, dtype)
    if isinstance(X, torch.Tensor):
        X = X.to(device)
        return X.to(dtype) if dtype is not None and X.is_floating_point() else X
    if sp.issparse(X):
        from ..core.base import CSR

        csr = sp.csr_matrix(X)
        vals = csr.data
        return CSR(
            indptr=_dense_to_device(csr.indptr.astype(np.int64), device, None),
            indices=_dense_to_device(csr.indices.astype(np.int32), device, None),
            data=_dense_to_device(vals, device, dtype),
            shape=(int(csr.shape[0]), int(csr.shape[1])),
        )
    a = np.asarray(X)
    if a.dtype.kind in "iub" and dtype is not None and dtype.is_floating_point:
        a = a.astype(np.float32 if dtype == torch.float32 else np.float64)
    return _dense_to_device(a, device, dtype if a.dtype.kind == "f" else None)


_copy_streams: dict = {}


def copy_stream(device: torch.device) -> "torch.cuda.Stream":
    """One persistent, HIGH-priority H2D stream per device.

    HIP maps streams onto a few hardware queues (GPU_MAX_HW_QUEUES, 4 by default) round-robin
    per priority level. A fresh normal-priority pool stream per ingest landed on the compute
    stream's queue about one fit in four: the chunk copies then serialised behind the statistics
    kernels instead of overlapping them (+0.11 s on a 12 GB LinearRegression fit). A
    high-priority stream never shares a queue with normal-priority compute.
    ``SRML_COPY_STREAM=new`` restores a fresh normal-priority pool stream per ingest."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if os.environ.get("SRML_COPY_STREAM", "persistent") == "new":
        return torch.cuda.Stream(device)
    st = _copy_streams.get(idx)
    if st is None:
        hi, _lo = torch.cuda.Stream.priority_range()
        lo_num = min(hi, _lo)  # numerically lower = higher priority
        st = torch.cuda.Stream(device, priority=lo_num)
        _copy_streams[idx] = st
    return st


class StreamedRows:
    """Row-chunked asynchronous H2D of a host matrix that lets the first pass over the data run
    while the rest of it is still crossing PCIe.

    The copies are queued on a dedicated copy stream, one event per chunk (2048-row chunks of a
    1M x 3000 fp32 shard are 24 MB: ~0.4 ms of DMA each). ``chunks()`` makes the CURRENT stream
    wait for chunk i only, then yields its device view, so a per-chunk kernel (moments, SYRK
    Gram, X^T y, quantisation) overlaps the DMA of chunks i+1... . ``wait_all()`` orders the
    current stream after the whole transfer (no host synchronisation anywhere). Only for
    page-locked sources (pinned Arrow buffers); pageable ones take ``host_to_device``'s ring.
    """

    def __init__(self, host: np.ndarray, device: torch.device, dtype: Optional[torch.dtype] = None,
                 chunk_bytes: int = 0) -> None:
        if chunk_bytes <= 0:
            chunk_bytes = int(os.environ.get("SRML_INGEST_CHUNK_MB", "96")) << 20
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            t = torch.from_numpy(np.ascontiguousarray(host))
        if dtype is not None and t.dtype != dtype:
            t = t.to(dtype)
        if not t.is_pinned():
            raise ValueError("StreamedRows needs a page-locked source (use host_to_device otherwise)")
        self.host = t
        self.device = device
        m = t.shape[0]
        row_bytes = max(1, t[0].numel() * t.element_size()) if m else 1
        self.chunk_rows = max(256, int(chunk_bytes // row_bytes))
        cur = torch.cuda.current_stream(device)
        self.X = torch.empty(t.shape, dtype=t.dtype, device=device)
        self._copy = copy_stream(device)
        self._copy.wait_stream(cur)
        self.X.record_stream(self._copy)
        self.bounds = []
        self.events = []
        self._stalls: list = []
        self._t0 = torch.cuda.Event(enable_timing=True)
        self._t1 = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(self._copy):
            self._t0.record(self._copy)
            for r0 in range(0, m, self.chunk_rows):
                r1 = min(m, r0 + self.chunk_rows)
                self.X[r0:r1].copy_(t[r0:r1], non_blocking=True)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self._copy)
                self.bounds.append((r0, r1))
                self.events.append(ev)
            self._t1.record(self._copy)

    def h2d_seconds(self) -> float:
        """Copy-stream time of the whole transfer (synchronises on its end)."""
        self._t1.synchronize()
        return self._t0.elapsed_time(self._t1) / 1e3

    def chunks(self) -> Iterator[Any]:
        cur = torch.cuda.current_stream(self.device)
        for (r0, r1), ev in zip(self.bounds, self.events):
            _timed_wait(cur, ev, self._stalls)
            yield r0, r1, self.X[r0:r1]

    def wait_all(self) -> torch.Tensor:
        if self.events:
            _timed_wait(torch.cuda.current_stream(self.device), self.events[-1], self._stalls)
        return self.X

    def exposed_seconds(self) -> float:
        """Time the compute stream stood waiting for this transfer (the H2D NOT hidden under
        compute); call after the fit has synchronised."""
        return _stall_seconds(self._stalls)


class RingRows:
    """Row chunks of a page-locked host matrix through a ring of ``depth`` device buffers (a
    transform that consumes each chunk once: ~depth x chunk bytes of HBM instead of the whole
    matrix, and no large allocation per call). The copy of chunk c + depth - 1 is queued on the
    copy stream as soon as chunk c - 1 (the previous user of its buffer) is consumed, so up to
    depth - 1 chunks cross PCIe while the current one is processed. Iterate ``chunks()``: each
    yields (r0, r1, device view) valid until the next step of the iteration."""

    def __init__(self, host: Any, device: torch.device, dtype: Optional[torch.dtype] = None,
                 chunk_bytes: int = 256 << 20, depth: int = 3) -> None:
        # host: one page-locked matrix, or a multi-batch ``ChunkedRows`` (its per-batch views are
        # chunked separately: a chunk never spans two batches, so no host concatenation)
        parts = list(host.parts) if hasattr(host, "parts") else [host]
        ts = []
        for a in parts:
            with warnings.catch_warnings():
                warnings.simplefilter("ignore", UserWarning)
                t = torch.from_numpy(np.ascontiguousarray(a))
            if not t.is_pinned():
                raise ValueError("RingRows needs a page-locked source")
            if dtype is not None and t.dtype != dtype:
                raise ValueError("RingRows copies without a cast: the source must already be %s" % dtype)
            ts.append(t)
        t = ts[0]
        self.device = device
        row_bytes = max(1, t[0].numel() * t.element_size()) if t.shape[0] else 1
        self.chunk_rows = max(256, int(chunk_bytes // row_bytes))
        # bounds: global (r0, r1); _src: (host tensor, local row offset) of every chunk
        self.bounds, self._src = [], []
        g = 0
        for tp in ts:
            mp = int(tp.shape[0])
            for l0 in range(0, mp, self.chunk_rows):
                l1 = min(mp, l0 + self.chunk_rows)
                self.bounds.append((g + l0, g + l1))
                self._src.append((tp, l0))
            g += mp
        self.host = t if len(ts) == 1 else None
        self.depth = max(2, int(depth))
        nb = min(self.depth, len(self.bounds))
        self.bufs = [torch.empty((self.chunk_rows,) + tuple(t.shape[1:]), dtype=t.dtype, device=device)
                     for _ in range(nb)]
        self._copy = copy_stream(device)
        self._stalls: list = []

    def chunks(self) -> Iterator[Any]:
        cur = torch.cuda.current_stream(self.device)
        ready: list = [None] * len(self.bounds)
        done: list = [None] * len(self.bounds)
        nb = len(self.bufs)

        def issue(c: int) -> None:
            r0, r1 = self.bounds[c]
            if c >= nb:  # the buffer's previous chunk must be consumed first
                self._copy.wait_event(done[c - nb])
            else:
                self._copy.wait_stream(cur)
            src, l0 = self._src[c]
            with torch.cuda.stream(self._copy):
                self.bufs[c % nb][: r1 - r0].copy_(src[l0: l0 + r1 - r0], non_blocking=True)
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self._copy)
            ready[c] = ev

        for c in range(nb):  # every buffer's first chunk
            issue(c)
        for c, (r0, r1) in enumerate(self.bounds):
            if c >= 1 and c + nb - 1 < len(self.bounds):
                issue(c + nb - 1)  # into chunk c - 1's buffer: chunk c - 1 was consumed below
            _timed_wait(cur, ready[c], self._stalls)
            buf = self.bufs[c % nb]
            buf.record_stream(cur)
            yield r0, r1, buf[: r1 - r0]
            ev = torch.cuda.Event()
            ev.record(cur)
            done[c] = ev

    def exposed_seconds(self) -> float:
        return _stall_seconds(self._stalls)


def is_pinned(a: Any) -> bool:
    """Whether a numpy array's memory (every batch of a ``ChunkedRows``) is page-locked
    (registered with the HIP runtime)."""
    if hasattr(a, "parts") and not isinstance(a, np.ndarray):
        return bool(a.parts) and all(is_pinned(p) for p in a.parts)
    if not isinstance(a, np.ndarray) or not torch.cuda.is_available():
        return False
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        try:
            return bool(torch.from_numpy(a).is_pinned())
        except Exception:  # noqa: BLE001
            return False


# ------------------------------------------------------------------------------------------
# UVM (managed memory) mode: SRML_UVM=1 or Spark conf spark.rocm.ml.uvm.enabled=true
# ------------------------------------------------------------------------------------------
_TYPESTR = {torch.float32: "<f4", torch.float64: "<f8", torch.int32: "<i4", torch.int64: "<i8",
            torch.uint8: "|u1", torch.int8: "|i1", torch.float16: "<f2"}


def uvm_enabled() -> bool:
    import os

    return os.environ.get("SRML_UVM", "0").lower() in ("1", "true", "yes")


class _ManagedBuffer:
    """hipMallocManaged allocation (srml_managed_malloc) exposed through __cuda_array_interface__;
    torch keeps this object alive for the tensor's lifetime and the allocation is freed with it."""

    def __init__(self, shape: Any, dtype: torch.dtype, device: torch.device) -> None:
        import ctypes

        from . import native

        lib = native.lib()
        if not getattr(lib, "_srml_uvm_typed", False):
            lib.srml_managed_malloc.restype = ctypes.c_void_p
            lib.srml_managed_malloc.argtypes = [ctypes.c_ssize_t, ctypes.c_int, ctypes.c_void_p]
            lib.srml_managed_free.restype = None
            lib.srml_managed_free.argtypes = [ctypes.c_void_p, ctypes.c_ssize_t, ctypes.c_int, ctypes.c_void_p]
            lib._srml_uvm_typed = True
        self._lib = lib
        self.shape = tuple(int(d) for d in shape)
        n = 1
        for d in self.shape:
            n *= d
        self.nbytes = max(1, n * torch.empty((), dtype=dtype).element_size())
        self.device = device
        self.ptr = lib.srml_managed_malloc(self.nbytes, device.index or 0, None)
        if not self.ptr:
            raise MemoryError("hipMallocManaged(%d) failed" % self.nbytes)
        self.__cuda_array_interface__ = {"shape": self.shape, "typestr": _TYPESTR[dtype],
                                         "data": (self.ptr, False), "version": 3, "strides": None}

    def __del__(self) -> None:
        if getattr(self, "ptr", None):
            self._lib.srml_managed_free(self.ptr, self.nbytes, self.device.index or 0, None)
            self.ptr = None


def managed_empty(shape: Any, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    """Uninitialised tensor in managed (UVM) memory: pages live where the GPU touches them and can
    exceed HBM capacity (the reference's spark.rapids.ml.uvm.enabled)."""
    return torch.as_tensor(_ManagedBuffer(shape, dtype, device), device=device)
