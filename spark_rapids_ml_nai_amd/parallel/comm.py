"""Device collectives for the data-parallel solvers: RCCL (``torch.distributed`` backend
``"nccl"`` on ROCm) over xGMI between GPUs of a node, gloo for CPU ranks.

Replaces the reference's raft/NCCL comms injected into a cuML ``Handle`` plus the Spark
``BarrierTaskContext.allGather`` JSON side channel it uses for numeric payloads
(``common/cuml_context.py:35-193``; ``classification.py:1006-1033``; ``tree.py:337-378``).
Every numeric exchange here is a device collective on the compute stream:

* ``allreduce`` / ``allreduce_coalesced`` — sufficient statistics (Gram, centroid sums,
  gradients, histograms). Small, latency-bound payloads are packed into ONE flat buffer so a
  whole L-BFGS evaluation (loss + gradient) or a Lloyd iteration (sums + counts + inertia)
  costs one collective launch instead of several: on the point-to-point xGMI mesh small
  messages are latency-bound, large ones are per-link bandwidth-bound, so fewer/larger wins.
* ``allgather`` / ``allgatherv`` — ragged per-rank blocks (kNN partial results, RF forests).
* ``broadcast``, ``barrier``, object collectives for tiny bootstrap metadata only.

A world of size 1 short-circuits every call (no process group needed), unless
``SRML_COMM_FORCE_PG=1`` (test-only): then a size-1 communicator over an initialised process group
runs every collective through the backend, so the RCCL code paths (event-timed ``CommStats``,
``batch_isend_irecv``, ``allgatherv``, one-shot selection) execute on a one-GPU box.

Accounting: every collective is counted (calls, payload bytes) and timed into ``Communicator.stats``
(``CommStats``) — on RCCL by a pair of timing events on the compute stream around the call (so the
time includes waiting for the slowest peer: the rank's comm-wait), on gloo by host wall time. The
fit driver resets it per fit and reports it with the H2D and wall times as the per-rank breakdown
(reference logs each worker stage, ``core.py:720-770``).

Failure semantics (reference ``common/cuml_context.py:150-167``: ``nccl.destroy()`` on success,
``nccl.abort()`` on exception): ``abort()`` aborts the process group's communicators
(``ncclCommAbort`` for RCCL — non-blocking, in-flight collectives on every rank error out) and only
then destroys the group; ``destroy_process_group`` alone can block forever on a dead peer.
``watchdog(seconds)`` bounds a block of collectives: if it has not finished in time, a monitor
thread aborts the communicator, so a rank waiting on the device (RCCL collectives are
asynchronous; the host blocks in a stream sync) raises instead of hanging. gloo collectives block
the calling thread inside the transport and cannot be interrupted, so ``comm_timeout()`` also
becomes the process group's own per-operation timeout (``init_process_group(timeout=...)``);
either way the stage fails with ``CommTimeout`` well before the barrier-stage timeout.
"""
from __future__ import annotations

import contextlib
import os
import pickle
import threading
import time
from typing import Any, Iterator, List, Optional, Sequence

import torch
import torch.distributed as dist

_OPS = {
    "sum": dist.ReduceOp.SUM,
    "max": dist.ReduceOp.MAX,
    "min": dist.ReduceOp.MIN,
    "prod": dist.ReduceOp.PRODUCT,
}


class Communicator:
    def __init__(self, rank: int = 0, size: int = 1, device: Optional[torch.device] = None,
                 group: Any = None) -> None:
        self.rank = int(rank)
        self.size = int(size)
        self.device = device if device is not None else torch.device("cpu")
        self.group = group
        force = os.environ.get("SRML_COMM_FORCE_PG", "0") == "1" and dist.is_initialized()
        # _solo: no peers and no process group to exercise -> every collective is the identity
        self._solo = self.size == 1 and not force
        self._backend = dist.get_backend(group) if (not self._solo and dist.is_initialized()) else "none"
        self.aborted = False
        self.stats = CommStats()
        self._oneshot: Any = None
        self._oneshot_failed = False

    # -- helpers --------------------------------------------------------------------
    @property
    def backend(self) -> str:
        return self._backend

    def _comm_tensor(self, t: torch.Tensor) -> torch.Tensor:
        """gloo needs CPU tensors, nccl/RCCL device tensors."""
        if self._backend == "gloo" and t.is_cuda:
            return t.cpu()
        if self._backend == "nccl" and not t.is_cuda:
            return t.to(self.device)
        return t

    # -- collectives ----------------------------------------------------------------
    def _timed(self, t: torch.Tensor, wire: float = 1.0) -> Any:
        """Account one collective on payload ``t``; ``wire``: bytes this rank sends per payload byte
        under the ring algorithm (all-reduce 2 (W - 1) / W, reduce-scatter (W - 1) / W, all-gather
        W - 1 per input byte)."""
        nb = t.numel() * t.element_size()
        return self.stats.record(nb, self.device if self._backend == "nccl" else None, wire_bytes=nb * wire)

    def _ring(self, kind: str) -> float:
        W = max(1, self.size)
        return {"allreduce": 2.0 * (W - 1) / W, "reduce_scatter": (W - 1) / W, "allgather": float(W - 1)}[kind]

    def _oneshot_for(self, t: torch.Tensor, op: str) -> Any:
        """The peer-mapped one-shot path when it applies to this payload: ``SRML_COMM=oneshot``
        always, ``auto`` when every rank of the group lives on this node (peer-mappable memory)."""
        if op != "sum" or not t.is_cuda or self._backend != "nccl" or not t.is_contiguous():
            return None
        if t.dtype not in (torch.float32, torch.float64):
            return None
        from . import oneshot

        mode = oneshot.comm_mode()
        if mode not in ("oneshot", "auto") or t.numel() * 8 > oneshot.MAX_BYTES:
            return None
        if self._oneshot is None and not self._oneshot_failed:
            # every rank reaches this point for the same payload (all-reduce shapes agree), so the
            # set-up collectives line up; the constructor agrees on success across ranks itself
            if mode == "auto" and not oneshot.single_node(self):
                self._oneshot_failed = True
                return None
            os_ = oneshot.OneShotAllreduce(self, self.device)
            if os_.ok:
                self._oneshot = os_
            else:
                if mode == "oneshot":
                    import warnings

                    warnings.warn("one-shot all-reduce unavailable (%s); using RCCL" % os_.reason)
                self._oneshot_failed = True
        return self._oneshot

    def allreduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """In-place all-reduce; returns ``t``."""
        if self._solo:
            return t
        os_ = self._oneshot_for(t, op)
        with self._timed(t, self._ring("allreduce")):
            if os_ is not None:
                return os_.allreduce(t)
            ct = self._comm_tensor(t)
            dist.all_reduce(ct, op=_OPS[op], group=self.group)
            if ct is not t:
                t.copy_(ct)
        return t

    def poll(self) -> None:
        """Non-blocking error check for the asynchronous device paths (one-shot all-reduce): raises
        ``CommError`` (after aborting) if a call issued before the previous ``poll`` failed."""
        if self._oneshot is not None and self._oneshot.poll():
            self._fail_oneshot()

    def check(self) -> None:
        """Blocking error check before a fit's results are used: every rank's asynchronous collectives
        (one-shot) succeeded AND every rank issued the same number of them, else abort and raise
        ``CommError`` on every rank. A rank that made fewer calls than its peers cannot see the
        peer's timeout by itself, so the verdict is agreed over the group's own backend (one tiny
        MAX all-reduce of [error, calls, -calls]; only when the one-shot path is active)."""
        if self._oneshot is None:
            return
        v = torch.tensor([1.0 if self._oneshot.failed() else 0.0, float(self._oneshot.epoch),
                          -float(self._oneshot.epoch)], dtype=torch.float64, device=self.device)
        ct = self._comm_tensor(v)
        dist.all_reduce(ct, op=dist.ReduceOp.MAX, group=self.group)
        err, hi, lo = (float(a) for a in ct.cpu().tolist())
        if err > 0 or hi != -lo:
            self._fail_oneshot()

    def _fail_oneshot(self) -> None:
        from . import oneshot

        self.abort()
        raise CommError("one-shot all-reduce on rank %d: a peer did not arrive within %.1f s; communicator "
                        "aborted" % (self.rank, oneshot.TIMEOUT_S))

    def allreduce_coalesced(self, tensors: Sequence[torch.Tensor], op: str = "sum") -> List[torch.Tensor]:
        """Pack same-dtype tensors into one flat buffer -> one collective -> unpack (in place)."""
        if self._solo or not tensors:
            return list(tensors)
        dtype = tensors[0].dtype
        assert all(t.dtype == dtype for t in tensors), "coalesced all-reduce needs one dtype"
        flat = torch.cat([t.reshape(-1) for t in tensors])
        self.allreduce(flat, op)
        off = 0
        for t in tensors:
            n = t.numel()
            t.copy_(flat[off: off + n].view_as(t))
            off += n
        return list(tensors)

    def allgather(self, t: torch.Tensor) -> torch.Tensor:
        """Equal-shaped blocks -> concatenated along dim 0."""
        if self._solo:
            return t
        with self._timed(t, self._ring("allgather")):
            ct = self._comm_tensor(t.contiguous())
            out = [torch.empty_like(ct) for _ in range(self.size)]
            dist.all_gather(out, ct, group=self.group)
            res = torch.cat(out, 0)
        return res.to(t.device) if res.device != t.device else res

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """Sum over ranks of ``t`` (dim 0 divisible by the world size), of which this rank keeps
        block ``rank`` of dim 0: half the bytes of an all-reduce on a ring, for consumers that only
        need their own slice of the reduction (the data-parallel forest's node-partitioned split
        search)."""
        if self._solo:
            return t
        assert t.shape[0] % self.size == 0, "reduce_scatter: dim 0 must divide by the world size"
        rows = t.shape[0] // self.size
        with self._timed(t, self._ring("reduce_scatter")):
            ct = self._comm_tensor(t.contiguous())
            out = torch.empty((rows,) + tuple(ct.shape[1:]), dtype=ct.dtype, device=ct.device)
            dist.reduce_scatter_tensor(out, ct, op=_OPS[op], group=self.group)
        return out.to(t.device) if out.device != t.device else out

    def allgatherv(self, t: torch.Tensor) -> List[torch.Tensor]:
        """Ragged dim-0 blocks -> list of per-rank tensors. One implementation for every backend:
        the sizes are all-gathered, each block is padded to the largest and ONE equal-shaped
        all-gather moves them (a single ring pass on RCCL instead of W per-root broadcasts; the
        padding is bounded by the imbalance, which the row-balanced partitioning keeps small)."""
        if self._solo:
            return [t]
        n = torch.tensor([t.shape[0]], dtype=torch.int64, device=self.device)
        sizes = self.allgather(n).tolist()
        mx = max(sizes)
        tail = tuple(t.shape[1:])
        pad = torch.zeros((mx,) + tail, dtype=t.dtype, device=t.device)
        pad[: t.shape[0]] = t
        g = self.allgather(pad).view((self.size, mx) + tail)
        return [g[r, : sizes[r]] for r in range(self.size)]

    def isendrecv(self, send: torch.Tensor, dst: int, recv: torch.Tensor, src: int) -> Any:
        """Start a paired point-to-point exchange (send ``send`` to ``dst``, receive into ``recv``
        from ``src``; group-local ranks). Returns a handle for ``wait_sendrecv``. RCCL batches the
        pair into one group call (the ring steps of the kNN query pass); gloo stages through host."""
        if self._solo:
            recv.copy_(send)
            return None
        cs = self._comm_tensor(send.contiguous())
        cr = self._comm_tensor(recv)
        g = self.group
        gd = dist.get_global_rank(g, dst) if g is not None else dst
        gs = dist.get_global_rank(g, src) if g is not None else src
        self.stats.calls += 1
        self.stats.bytes += cs.numel() * cs.element_size()
        self.stats.wire_bytes += cs.numel() * cs.element_size()
        works = dist.batch_isend_irecv([dist.P2POp(dist.isend, cs, gd, group=g),
                                        dist.P2POp(dist.irecv, cr, gs, group=g)])
        return (works, cs, cr, recv)

    def wait_sendrecv(self, handle: Any) -> None:
        if handle is None:
            return
        works, _cs, cr, recv = handle
        with self.stats.record(0, self.device if self._backend == "nccl" else None, count=False):
            for w in works:
                w.wait()
        if cr is not recv:
            recv.copy_(cr)

    def sendrecv(self, send: torch.Tensor, dst: int, recv: torch.Tensor, src: int) -> torch.Tensor:
        self.wait_sendrecv(self.isendrecv(send, dst, recv, src))
        return recv

    def broadcast(self, t: torch.Tensor, src: int = 0) -> torch.Tensor:
        if self._solo:
            return t
        with self._timed(t, 1.0 if self.rank == src or self.size > 2 else 0.0):
            ct = self._comm_tensor(t)
            dist.broadcast(ct, src=src, group=self.group)
            if ct is not t:
                t.copy_(ct)
        return t

    def barrier(self) -> None:
        if self._solo:
            return
        if self._backend == "nccl":
            # a tiny all-reduce is the stream-ordered barrier for RCCL
            z = torch.zeros(1, device=self.device)
            dist.all_reduce(z, group=self.group)
            torch.cuda.synchronize(self.device)
        else:
            dist.barrier(group=self.group)

    def allgather_object(self, obj: Any) -> List[Any]:
        if self._solo:
            return [obj]
        out: List[Any] = [None] * self.size
        dist.all_gather_object(out, obj, group=self.group)
        return out

    def broadcast_object(self, obj: Any, src: int = 0) -> Any:
        if self._solo:
            return obj
        lst = [obj]
        dist.broadcast_object_list(lst, src=src, group=self.group)
        return lst[0]

    def allgather_bytes(self, payload: bytes) -> List[bytes]:
        """Device all-gather of opaque byte blobs (e.g. serialized forests) — no driver hop."""
        if self._solo:
            return [payload]
        buf = torch.frombuffer(bytearray(payload), dtype=torch.uint8) if payload else torch.zeros(0, dtype=torch.uint8)
        parts = self.allgatherv(buf.to(self.device))
        return [bytes(p.cpu().numpy().tobytes()) for p in parts]

    def abort(self) -> None:
        """Abort the communicators (``ncclCommAbort`` / gloo abort: pending collectives fail on
        every rank instead of waiting for a dead peer), then destroy the group."""
        if self.size <= 1 or not dist.is_initialized() or self.aborted:
            return
        self.aborted = True
        try:
            from torch.distributed import distributed_c10d as c10d

            c10d._abort_process_group(self.group if self.group is not None else c10d.GroupMember.WORLD)
        except Exception:  # noqa: BLE001 - fall back to the backend object's own abort
            try:
                pg = self.group if self.group is not None else dist.group.WORLD
                dev = self.device if self.device.type == "cuda" else torch.device("cpu")
                pg._get_backend(dev).abort()
            except Exception:  # noqa: BLE001
                pass
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass

    @contextlib.contextmanager
    def watchdog(self, seconds: Optional[float] = None, what: str = "collective") -> Iterator[None]:
        """Abort the communicator if the enclosed block runs longer than ``seconds``
        (default ``SRML_COMM_TIMEOUT``, 0/unset = off); the block then raises ``CommTimeout``."""
        if seconds is None:
            seconds = float(os.environ.get("SRML_COMM_TIMEOUT", "0") or 0)
        if self.size <= 1 or not seconds or seconds <= 0:
            yield
            return
        done = threading.Event()
        fired = threading.Event()

        def _monitor() -> None:
            if not done.wait(seconds):
                fired.set()
                self.abort()

        t = threading.Thread(target=_monitor, name="srml-comm-watchdog", daemon=True)
        t.start()
        try:
            yield
        except Exception as e:  # noqa: BLE001
            msg = str(e).lower()
            if fired.is_set() or "timed out" in msg or "timeout" in msg:
                done.set()
                self.abort()
                raise CommTimeout(f"{what} on rank {self.rank} exceeded {seconds:.0f}s; communicator aborted") from e
            raise
        finally:
            done.set()
        if fired.is_set():
            raise CommTimeout(f"{what} on rank {self.rank} exceeded {seconds:.0f}s; communicator aborted")


def comm_timeout(default_s: float) -> float:
    """Per-operation timeout for new process groups: ``SRML_COMM_TIMEOUT`` if set, else the default
    (the barrier-stage timeout)."""
    v = float(os.environ.get("SRML_COMM_TIMEOUT", "0") or 0)
    return v if v > 0 else float(default_s)


class CommError(RuntimeError):
    """A collective failed (a peer never arrived); the communicator was aborted."""


class CommTimeout(CommError):
    """A watched block of collectives overran its deadline and the communicator was aborted."""


def _rank_timers_enabled() -> bool:
    return os.environ.get("SRML_RANK_TIMERS", "1") == "1"


class CommStats:
    """Per-rank collective accounting: calls, payload bytes and time spent in collectives.

    Device collectives (RCCL) are timed by a pair of timing events on the current stream around
    the call: the span is how long the compute stream stood at that collective, i.e. the transfer
    plus the wait for the slowest peer. Host-blocking ones (gloo) add their wall time. ``seconds()``
    resolves the events (it synchronises on the last one), so call it after the fit."""

    def __init__(self) -> None:
        self.reset()

    def reset(self) -> None:
        self.calls = 0
        self.bytes = 0
        self.wire_bytes = 0.0  # bytes this rank sends (ring algorithms), see Communicator._timed
        self.host_s = 0.0
        self._dev_s = 0.0  # resolved device spans (folded out of _pairs)
        self._pairs: List[Any] = []

    _FOLD_AT = 256     # fold finished event pairs once this many are pending (non-blocking)
    _HARD_CAP = 4096   # beyond this, wait for the oldest ones (a long-lived communicator's jobs)

    def _fold(self) -> None:
        """Resolve finished timing pairs into ``_dev_s`` so a communicator that lives across many
        jobs (the SPMD context's transform / kneighbors / evaluate collectives) keeps a bounded
        list; never blocks unless more than ``_HARD_CAP`` pairs are still in flight."""
        i = 0
        while i < len(self._pairs) and (self._pairs[i][1].query() or len(self._pairs) - i > self._HARD_CAP):
            s, e = self._pairs[i]
            e.synchronize()
            self._dev_s += s.elapsed_time(e) / 1e3
            i += 1
        if i:
            del self._pairs[:i]

    @contextlib.contextmanager
    def record(self, nbytes: int, device: Optional[torch.device], count: bool = True,
               wire_bytes: Optional[float] = None) -> Iterator[None]:
        if count:
            self.calls += 1
            self.bytes += int(nbytes)
            self.wire_bytes += float(nbytes if wire_bytes is None else wire_bytes)
        if device is not None and device.type == "cuda" and torch.cuda.is_current_stream_capturing():
            yield  # recorded into a HIP graph (the QN batch): counted, not timed
            return
        if device is not None and device.type == "cuda" and _rank_timers_enabled():
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            try:
                yield
            finally:
                e.record()
                self._pairs.append((s, e))
                if len(self._pairs) >= self._FOLD_AT:
                    self._fold()
            return
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.host_s += time.perf_counter() - t0

    def seconds(self) -> float:
        if self._pairs:
            self._pairs[-1][1].synchronize()
            self._dev_s += sum(s.elapsed_time(e) for s, e in self._pairs) / 1e3
            self._pairs = []
        return self.host_s + self._dev_s

    def snapshot(self) -> dict:
        return {"comm_s": round(self.seconds(), 6), "comm_calls": self.calls, "comm_bytes": self.bytes,
                "comm_wire_bytes": int(self.wire_bytes)}


def pickle_obj(o: Any) -> bytes:
    return pickle.dumps(o, protocol=pickle.HIGHEST_PROTOCOL)
