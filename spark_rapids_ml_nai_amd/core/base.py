"""Estimator / Model base classes and the fit & transform drivers.

Re-design of the reference's framework core (``core.py:426-1647``):

* ``_Estimator._fit_internal`` = ``_CumlCaller._call_cuml_fit_func`` + ``_CumlEstimator._fit_internal``:
  validate params, select/cast feature columns (array, VectorUDT dense/sparse, multi-column),
  split the data into ``num_workers`` row partitions, run the algorithm's worker closure on
  every rank, build one model per param map (``fitMultiple`` single pass).
* Three execution backends for the same worker closure (``parallel/``):
  SPMD (caller already runs one process per GPU under torchrun: no data movement, RCCL
  group reused), LocalBarrierRunner (N spawned ranks, the Spark-free barrier stage) and
  in-process for ``num_workers == 1``; the Spark barrier path lives in ``parallel/spark.py``.
* The worker closure receives a ``FitInput`` with the partition already on the device
  (zero-copy Arrow view -> pinned staging -> async H2D) and a ``WorkerContext`` holding the
  rank's communicator — the analogue of the raft ``Handle`` the reference passes to cuML.
* ``_Model._transform`` runs the model's device predict function per partition and appends
  the output columns (prediction / probability / rawPrediction / outputCol).
"""
from __future__ import annotations

import os
import threading
import time
from abc import abstractmethod
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, Iterator, List, Optional, Sequence, Tuple, Union

import numpy as np
import torch

from ..parallel.context import (PartitionDescriptor, WorkerContext, current_context, spmd_active, spmd_context,
                                use_context)
from ..utils.log import get_logger
from ..utils.timer import PhaseTimer
import pyarrow as pa

from .dataframe import (
    ChunkedRows,
    DataFrame,
    array_column_chunks,
    as_dataframe,
    is_array_field,
    is_vector_field,
    restore_kind,
    vector_column_is_sparse,
    vector_column_to_csr,
    vector_column_to_dense,
    array_column_to_dense,
)
from .params import PYSPARK_PARAMS, Param, _BackendParams

if PYSPARK_PARAMS:  # estimators / models are genuine pyspark.ml stages (Pipeline, tuning, ...)
    from pyspark.ml import Estimator as _SparkEstimator  # type: ignore
    from pyspark.ml import Model as _SparkModel  # type: ignore

    _ESTIMATOR_BASES: Tuple[type, ...] = (_SparkEstimator,)
    _MODEL_BASES: Tuple[type, ...] = (_SparkModel,)
else:
    _ESTIMATOR_BASES = ()
    _MODEL_BASES = ()
from .persistence import (
    EstimatorReader,
    EstimatorWriter,
    MLReadable,
    MLWritable,
    ModelReader,
    ModelWriter,
)


# --------------------------------------------------------------------------------------
# Column aliases (reference core.py:122-156)
# --------------------------------------------------------------------------------------
class alias:
    data = "srml_values_c3BhcmtjdW1s"
    label = "srml_label_c3BhcmtjdW1s"
    row_number = "srml_row_number_c3BhcmtjdW1s"


class pred:
    prediction = "prediction"
    probability = "probability"
    model_index = "model_index"
    raw_prediction = "raw_prediction"


class param_alias:
    cuml_init = "cuml_init"
    handle = "handle"
    num_cols = "num_cols"
    part_sizes = "part_sizes"
    loop = "loop"
    fit_multiple_params = "fit_multiple_params"


# --------------------------------------------------------------------------------------
# Data carried to a worker and onto its device
# --------------------------------------------------------------------------------------
@dataclass
class CSR:
    """Device CSR matrix (row offsets int64, column indices int32, values)."""

    indptr: torch.Tensor
    indices: torch.Tensor
    data: torch.Tensor
    shape: Tuple[int, int]

    @property
    def device(self) -> torch.device:
        return self.data.device

    @property
    def dtype(self) -> torch.dtype:
        return self.data.dtype

    def to_dense(self) -> torch.Tensor:
        return torch.sparse_csr_tensor(self.indptr, self.indices.long(), self.data, self.shape).to_dense()


@dataclass
class HostPartition:
    X: Any  # np.ndarray (rows, n) | scipy.sparse.csr_matrix | None
    y: Optional[np.ndarray] = None
    cols: Dict[str, np.ndarray] = field(default_factory=dict)
    n_cols: int = 0

    @property
    def rows(self) -> int:
        if self.X is not None:
            return int(self.X.shape[0])
        if self.y is not None:
            return int(self.y.shape[0])
        return int(next(iter(self.cols.values())).shape[0]) if self.cols else 0


@dataclass
class FitInput:
    X: Union[torch.Tensor, CSR, None]
    y: Optional[torch.Tensor]
    cols: Dict[str, np.ndarray]
    desc: PartitionDescriptor
    host: HostPartition
    # set for estimators that opt into streaming ingest: X's H2D is still in flight and the
    # first pass must consume ``stream.chunks()`` (or call ``stream.wait_all()``) before using X
    stream: Any = None


def to_device(X: Any, device: torch.device, dtype: Optional[torch.dtype] = None) -> Any:
    """Host array -> device tensor through pinned staging (chunked, async H2D)."""
    from ..ops.ingest import host_to_device

    return host_to_device(X, device, dtype)


def _dense_from_df(df: DataFrame, col: Optional[str], cols: Optional[List[str]], np_dtype: Any,
                   chunked: bool = False) -> Any:
    """Features of a partition as a host matrix. ``chunked`` (fit ingest): a multi-batch array
    column stays a list of per-batch zero-copy views (``ChunkedRows``) for the streaming H2D."""
    if cols:
        mats = [df.to_numpy(c).reshape(-1, 1) for c in cols]
        return np.ascontiguousarray(np.hstack(mats).astype(np_dtype))
    f = df.schema.field(col)
    if is_vector_field(f):
        return vector_column_to_dense(df.column(col), np_dtype)
    if is_array_field(f):
        c = df.column(col)
        if chunked and isinstance(c, pa.ChunkedArray) and c.num_chunks > 1:
            return array_column_chunks(c, np_dtype)
        return array_column_to_dense(c, np_dtype)
    return df.to_numpy(col).astype(np_dtype).reshape(-1, 1)


# --------------------------------------------------------------------------------------
# Shared base
# --------------------------------------------------------------------------------------
class _CommonBase(_BackendParams, MLWritable, MLReadable):
    def __init__(self) -> None:
        super().__init__()
        self.logger = get_logger(self.__class__)

    @classmethod
    def _pyspark_class(cls) -> Optional[str]:
        """Fully-qualified pyspark.ml class this one mirrors (for ``cpu()``)."""
        return None

    def _verbose(self) -> Any:
        return self._backend_params.get("verbose", False)


def _split_rows(n: int, parts: int) -> List[Tuple[int, int]]:
    b = np.linspace(0, n, parts + 1).astype(np.int64)
    return [(int(b[i]), int(b[i + 1])) for i in range(parts)]


class _Estimator(_CommonBase, *_ESTIMATOR_BASES):  # type: ignore[misc]
    """Base of every estimator (reference ``_CumlEstimator`` + ``_CumlCaller``)."""

    def __init__(self) -> None:
        super().__init__()
        self._initialize_backend_params()

    # ---- hooks ------------------------------------------------------------------
    @abstractmethod
    def _get_fit_func(
        self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None
    ) -> Callable[[FitInput, WorkerContext, Dict[str, Any]], Union[Dict[str, Any], List[Dict[str, Any]]]]:
        """Return the worker closure ``fit(inp, ctx, params) -> attributes (or list for fitMultiple)``."""

    @abstractmethod
    def _create_model(self, result: Dict[str, Any]) -> "_Model":
        ...

    def _enable_fit_multiple_in_single_pass(self) -> bool:
        return False

    def _require_comm(self) -> bool:
        """Whether the fit needs a live communicator (False -> ranks never talk, e.g. RF ensemble)."""
        return True

    def _fit_uses_label(self) -> bool:
        return False

    def _fit_extra_cols(self) -> List[str]:
        return []

    def _fit_array_order(self) -> str:
        return "C"

    def _supports_sparse(self) -> bool:
        return False

    def _validate_parameters(self) -> None:
        pass

    def _label_dtype(self, float32: bool) -> Any:
        return np.float32 if float32 else np.float64

    def _supportsTransformEvaluate(self, evaluator: Any) -> bool:
        return False

    # ---- data preparation ----------------------------------------------------------
    def _use_sparse(self, df: DataFrame, col: Optional[str]) -> bool:
        if col is None or not df.is_vector(col) or not self._supports_sparse():
            return False
        flag = None
        if self.hasParam("enable_sparse_data_optim"):
            flag = self.getOrDefault("enable_sparse_data_optim")
        if flag is None:
            return vector_column_is_sparse(df.column(col))
        return bool(flag)

    def _host_partition(self, df: DataFrame) -> HostPartition:
        col, cols = self._get_input_columns()
        np_dtype = np.float32 if self._float32_inputs else np.float64
        if self._use_sparse(df, col):
            X = vector_column_to_csr(df.column(col), np_dtype)
        else:
            X = _dense_from_df(df, col, cols, np_dtype, chunked=True)
        y = None
        if self._fit_uses_label():
            lc = self.getOrDefault("labelCol")
            y = df.to_numpy(lc).astype(self._label_dtype(self._float32_inputs))
        extra = {c: df.to_numpy(c) for c in self._fit_extra_cols() if c in df.columns}
        return HostPartition(X=X, y=y, cols=extra, n_cols=int(X.shape[1]) if X is not None else 0)

    def _backend_param_maps(self, paramMaps: Optional[Sequence[Dict[Param, Any]]]) -> List[Dict[str, Any]]:
        out = []
        for pm in paramMaps or []:
            d = {}
            for k, v in pm.items():
                name = self._get_backend_param(k.name, False)
                if name is not None:
                    d[name] = self._get_backend_mapping_value(name, v)
            out.append(d)
        return out

    # ---- fit ----------------------------------------------------------------------
    def fit(self, dataset: Any, params: Any = None) -> Any:
        if params is None:
            return self._fit(dataset)
        if isinstance(params, dict):
            return self.copy(params)._fit(dataset)
        if isinstance(params, (list, tuple)):
            models: List[Any] = [None] * len(params)
            for idx, model in self.fitMultiple(dataset, params):
                models[idx] = model
            return models
        raise TypeError("Params must be either a param map or a list/tuple of param maps")

    def _fit(self, dataset: Any) -> "_Model":
        return self._fit_internal(dataset, None)[0]

    def fitMultiple(self, dataset: Any, paramMaps: Sequence[Dict[Param, Any]]) -> Iterator[Tuple[int, "_Model"]]:
        if self._enable_fit_multiple_in_single_pass():
            for pm in paramMaps:
                for p in pm:
                    self._get_backend_param(p.name, silent=False)
            return _FitMultipleIterator(lambda: self._fit_internal(dataset, paramMaps), len(paramMaps))

        est = self.copy()

        def _gen() -> Iterator[Tuple[int, "_Model"]]:
            for i, pm in enumerate(paramMaps):
                yield i, est.copy(pm)._fit(dataset)

        return _ThreadSafeIter(_gen())

    def _fit_internal(self, dataset: Any, paramMaps: Optional[Sequence[Dict[Param, Any]]]) -> List["_Model"]:
        self._validate_parameters()
        timer = PhaseTimer()
        fit_multiple = self._backend_param_maps(paramMaps)
        params = {
            param_alias.cuml_init: dict(self._backend_params),
            param_alias.fit_multiple_params: fit_multiple,
        }
        from ..parallel.spark import is_spark_dataframe, run_spark_fit

        if is_spark_dataframe(dataset):
            # Spark barrier stage: one task per GPU, RCCL bootstrapped through allGather
            fit_fn = self._get_fit_func(dataset, fit_multiple or None)
            with timer.phase("fit"):
                results = run_spark_fit(self, dataset, fit_fn, params)
            if isinstance(results, _FitOut):
                timer.rank_stats = results.ranks
                results = results.result
        else:
            df, _ = as_dataframe(dataset)
            fit_fn = self._get_fit_func(df, fit_multiple or None)
            results = run_fit_job(self, df, fit_fn, params, timer)
        if not isinstance(results, list):
            results = [results]
        log_rank_split(self.logger, self.__class__.__name__ + " fit", getattr(timer, "rank_stats", None))
        models = []
        for i, r in enumerate(results):
            model = self._create_model(r)
            model._num_workers = self._num_workers
            model._float32_inputs = self._float32_inputs
            self._copyValues(model)
            self._copy_backend_params(model)
            if paramMaps is not None:
                est_i = self.copy(paramMaps[i])
                est_i._copyValues(model)
                est_i._copy_backend_params(model)
            model._fit_timings = dict(timer.times)
            model._rank_stats = getattr(timer, "rank_stats", None)
            models.append(model)
        return models

    def write(self) -> EstimatorWriter:
        return EstimatorWriter(self)

    @classmethod
    def read(cls) -> EstimatorReader:
        return EstimatorReader(cls)


class _EstimatorSupervised(_Estimator):
    def _fit_uses_label(self) -> bool:
        return True


class _FitOut:
    """A worker's fit result plus the per-rank time split of that fit (every rank's, all-gathered
    at the end of a multi-rank fit): what ``_fit_worker`` hands back to the driver side."""

    def __init__(self, result: Any, ranks: List[Dict[str, Any]]) -> None:
        self.result = result
        self.ranks = ranks


_worker_log = get_logger("worker")


def _fit_worker(ctx: WorkerContext, payload: Tuple[HostPartition, Callable, Dict[str, Any], bool]) -> _FitOut:
    """Body of one barrier task: ingest to device, describe partitions, run the fit closure.

    Logs the reference's worker stages (``core.py:720-770``) and returns the rank's time split:
    ``h2d_exposed_s`` (the compute stream waiting for the host->device copy; a streamed ingest's
    chunks hidden under compute are not counted), ``comm_s`` (collectives, event-timed on RCCL),
    ``compute_s`` = wall - h2d_exposed - comm, plus ``h2d_s`` (the copy stream's whole span)."""
    hp, fit_fn, params, float32 = payload
    t_start = time.perf_counter()
    ctx.comm.stats.reset()
    tag = "rank %d/%d" % (ctx.rank, ctx.world_size)
    _worker_log.info("%s: Loading data (%d rows x %d cols) onto %s", tag, hp.rows, hp.n_cols, ctx.device)
    _maybe_inject_fault(ctx, "ingest")
    desc = None
    if ctx.world_size > 1:
        # the partition descriptor's one all-gather of row counts, BEFORE any numeric collective:
        # every rank learns which ranks are empty and raises the same error together, instead of
        # the empty rank raising alone while its peers block in their first all-reduce
        desc = PartitionDescriptor.build(ctx, hp.rows, hp.n_cols)
        empty = [r for r, n in desc.parts_rank_size if n == 0]
        if empty:
            raise RuntimeError("A worker received no data. Please increase amount of data or use fewer workers. "
                               "(ranks with no rows: %s of %d)" % (empty, ctx.world_size))
    elif hp.rows == 0:
        raise RuntimeError("A worker received no data. Please increase amount of data or use fewer workers.")
    dtype = torch.float32 if float32 else torch.float64
    streamed = None
    # the copy alone: the descriptor's all-gather above is already in comm_s (counting it here too
    # double-counts the wait for a slower peer)
    t_h2d = time.perf_counter()
    from ..ops.ingest import StreamedParts, StreamedRows, is_pinned, uvm_enabled

    stream_ok = (ctx.is_gpu and getattr(fit_fn, "streaming_ingest", False) and not uvm_enabled()
                 and os.environ.get("SRML_STREAM_INGEST", "1") == "1")
    if (stream_ok and isinstance(hp.X, np.ndarray) and hp.X.ndim == 2 and hp.X.shape[0] > 0
            and hp.X.dtype == (np.float32 if float32 else np.float64) and hp.X.flags.c_contiguous
            and is_pinned(hp.X)):
        # the fit's preferred chunk (bytes) unless SRML_INGEST_CHUNK_MB overrides it
        chunk_mb = 0 if "SRML_INGEST_CHUNK_MB" in os.environ else int(getattr(fit_fn, "ingest_chunk_mb", 0))
        streamed = StreamedRows(hp.X, ctx.device, dtype, chunk_bytes=chunk_mb << 20)
        X = streamed.X
    elif stream_ok and isinstance(hp.X, ChunkedRows) and hp.X.shape[0] > 0:
        streamed = StreamedParts(hp.X, ctx.device, dtype)  # Spark batches: fill/DMA/compute pipelined
        X = streamed.X
    else:
        h2d_ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)] if ctx.is_gpu else None
        if h2d_ev:
            h2d_ev[0].record()
        X = to_device(hp.X, ctx.device, dtype) if hp.X is not None else None
        if h2d_ev:
            h2d_ev[1].record()  # pinned sources are queued asynchronously: time them on the stream
    h2d_host_s = time.perf_counter() - t_h2d
    y = to_device(hp.y, ctx.device) if hp.y is not None else None
    _worker_log.info("%s: Initializing context (partition descriptor, %s communicator)", tag,
                     ctx.comm.backend if hasattr(ctx.comm, "backend") else "local")
    if desc is None:
        desc = PartitionDescriptor.build(ctx, hp.rows, hp.n_cols)
    inp = FitInput(X=X, y=y, cols=hp.cols, desc=desc, host=hp, stream=streamed)
    _maybe_inject_fault(ctx, "fit")
    _worker_log.info("%s: Invoking fit (%d global rows)", tag, desc.m)
    with ctx.comm.watchdog(what="fit"):  # SRML_COMM_TIMEOUT: abort the communicator on a stuck collective
        out = fit_fn(inp, ctx, params)
        ctx.comm.check()  # asynchronous collectives (one-shot) all succeeded, else CommError
    if ctx.is_gpu and os.environ.get("SRML_FIT_DEVICE_SYNC", "1") == "1":
        # leave the device idle (copy stream included) before the task returns
        torch.cuda.synchronize(ctx.device)
    wall = time.perf_counter() - t_start
    if streamed is not None:
        h2d = streamed.h2d_seconds()
        exposed = min(streamed.exposed_seconds(), h2d)
    elif ctx.is_gpu and h2d_ev:
        h2d_ev[1].synchronize()
        h2d = max(h2d_host_s, h2d_ev[0].elapsed_time(h2d_ev[1]) / 1e3)
        exposed = h2d  # copied before any compute was queued: none of it is hidden
    else:
        h2d = exposed = h2d_host_s
    st = ctx.comm.stats.snapshot()
    exposed = min(exposed, wall)
    mine = dict(rank=ctx.rank, wall_s=round(wall, 6), h2d_s=round(h2d, 6), h2d_exposed_s=round(exposed, 6),
                compute_s=round(max(0.0, wall - exposed - st["comm_s"]), 6), **st)
    ctx.timers["rank"] = mine
    ranks = [mine]
    if ctx.world_size > 1:
        # one small all-gather at the end of the fit: every rank (and the driver, through rank 0's
        # result) sees the whole split and the skew
        import pickle

        from ..parallel.comm import pickle_obj

        ranks = [pickle.loads(b) for b in ctx.comm.allgather_bytes(pickle_obj(mine))]
    ctx.timers["ranks"] = ranks
    _worker_log.info("%s: Fit complete in %.4f s (h2d exposed %.4f, compute %.4f, comm %.4f)", tag, wall,
                     mine["h2d_exposed_s"], mine["compute_s"], mine["comm_s"])
    return _FitOut(out, ranks)


def log_rank_split(logger: Any, what: str, ranks: Optional[List[Dict[str, Any]]]) -> None:
    """One line per rank of a fit's time split plus the rank skew (max / min wall), from the driver
    (or rank 0 of an SPMD job, whose every rank holds the gathered split)."""
    if not ranks:
        return
    if spmd_active() and torch.distributed.get_rank() != 0:
        return
    for r in ranks:
        logger.info("%s rank %d: wall %.4f s = h2d_exposed %.4f + compute %.4f + comm %.4f (h2d span %.4f, "
                    "%d collectives, %d bytes)", what, r.get("rank", -1), r.get("wall_s", 0.0),
                    r.get("h2d_exposed_s", 0.0), r.get("compute_s", 0.0), r.get("comm_s", 0.0), r.get("h2d_s", 0.0),
                    r.get("comm_calls", 0), r.get("comm_bytes", 0))
    walls = [float(r.get("wall_s", 0.0)) for r in ranks]
    if len(walls) > 1:
        logger.info("%s rank skew: max/min wall %.4f / %.4f s (%.3fx)", what, max(walls), min(walls),
                    max(walls) / max(min(walls), 1e-12))


def _maybe_inject_fault(ctx: WorkerContext, stage: str) -> None:
    """Fault injection for failure-path tests: ``SRML_FAULT_RANK=<r>`` (``all`` for every rank),
    ``SRML_FAULT_STAGE=ingest|fit`` (default fit), ``SRML_FAULT_MODE=raise|exit|hang``."""
    import os

    who = os.environ.get("SRML_FAULT_RANK")
    if who is None or os.environ.get("SRML_FAULT_STAGE", "fit") != stage:
        return
    if who != "all" and int(who) != ctx.rank:
        return
    mode = os.environ.get("SRML_FAULT_MODE", "raise")
    if mode == "exit":
        os._exit(17)
    if mode == "hang":
        import time

        time.sleep(float(os.environ.get("SRML_FAULT_HANG_S", "3600")))
    raise RuntimeError("injected fault on rank %d at %s" % (ctx.rank, stage))


def run_fit_job(est: _Estimator, df: DataFrame, fit_fn: Callable, params: Dict[str, Any],
                timer: Optional[PhaseTimer] = None) -> Any:
    """Dispatch the worker closure to SPMD / in-process / LocalBarrierRunner (or Spark)."""
    timer = timer or PhaseTimer()
    float32 = est._float32_inputs
    if spmd_active() or est.num_workers <= 1:
        ctx = current_context() or (spmd_context() if spmd_active() else WorkerContext.single())
        with timer.phase("ingest"):
            hp = est._host_partition(df)
        with use_context(ctx), timer.phase("fit"):
            res = _fit_worker(ctx, (hp, fit_fn, params, float32))
        timer.rank_stats = res.ranks
        return res.result
    nw = est.num_workers
    from ..parallel.launcher import run_barrier_job

    with timer.phase("ingest"):
        if df.getNumPartitions() != nw:
            df = df.repartition(nw)
        hps = [est._host_partition(DataFrame([p])) for p in df.partitions]
    with timer.phase("fit"):
        results = run_barrier_job(_fit_worker, [(hp, fit_fn, params, float32) for hp in hps])
    timer.rank_stats = results[0].ranks
    return results[0].result


def run_worker_job(fn: Callable[[WorkerContext, Any], Any], payloads: Sequence[Any]) -> List[Any]:
    """Run ``fn(ctx, payload)`` once per worker and return every rank's result.

    SPMD (torch.distributed already initialised): this process is one rank and ``payloads``
    holds only its own entry. Otherwise one payload runs in-process and several run as a
    LocalBarrierRunner stage (one process per GPU).
    """
    if spmd_active():
        ctx = current_context() or spmd_context()
        with use_context(ctx):
            return [fn(ctx, payloads[0])]
    if len(payloads) <= 1:
        ctx = current_context() or WorkerContext.single()
        with use_context(ctx):
            return [fn(ctx, payloads[0])]
    from ..parallel.launcher import run_barrier_job

    return run_barrier_job(fn, list(payloads))


class _FitMultipleIterator:
    """Thread-safe iterator that fits every param map in ONE job on first ``next()``."""

    def __init__(self, fitMultipleModels: Callable[[], List["_Model"]], numModels: int) -> None:
        self.fitMultipleModels = fitMultipleModels
        self.numModels = numModels
        self.counter = 0
        self.lock = threading.Lock()
        self.models: Optional[List["_Model"]] = None

    def __iter__(self) -> Iterator[Tuple[int, "_Model"]]:
        return self

    def __next__(self) -> Tuple[int, "_Model"]:
        with self.lock:
            index = self.counter
            if index >= self.numModels:
                raise StopIteration("No models remaining.")
            if index == 0:
                self.models = self.fitMultipleModels()
                assert len(self.models) == self.numModels
            self.counter += 1
        assert self.models is not None
        return index, self.models[index]

    next = __next__


class _ThreadSafeIter:
    def __init__(self, it: Iterator) -> None:
        self.it = it
        self.lock = threading.Lock()

    def __iter__(self) -> "_ThreadSafeIter":
        return self

    def __next__(self) -> Any:
        with self.lock:
            return next(self.it)


# --------------------------------------------------------------------------------------
# Models
# --------------------------------------------------------------------------------------
TransformFn = Callable[[Any, Any, WorkerContext], Dict[str, np.ndarray]]


class _Model(_CommonBase, *_MODEL_BASES):  # type: ignore[misc]
    """Base of every fitted model (reference ``_CumlModel``)."""

    def __init__(self, **model_attributes: Any) -> None:
        super().__init__()
        self._model_attributes = model_attributes
        self._fit_timings: Dict[str, float] = {}
        self._device_state_cache: Dict[Any, Any] = {}
        self._initialize_backend_params()

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {}

    def _get_model_attributes(self) -> Dict[str, Any]:
        return self._model_attributes

    @classmethod
    def _from_row(cls, model_attributes: Any) -> "_Model":
        d = model_attributes.asDict() if hasattr(model_attributes, "asDict") else dict(model_attributes)
        return cls(**d)

    def cpu(self) -> Any:
        raise NotImplementedError("cpu() needs pyspark; it is not installed" if not _have_pyspark() else "")

    # ---- transform hooks -------------------------------------------------------------
    @abstractmethod
    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable[[WorkerContext], Any], TransformFn]:
        """Return (construct(ctx) -> device state, predict(state, X, ctx) -> {col: ndarray})."""

    def _transform_input_cols(self) -> Tuple[Optional[str], Optional[List[str]]]:
        return self._get_input_columns()

    def _transform_supports_sparse(self) -> bool:
        return False

    def _transform_dtype(self) -> Any:
        return np.float32 if self._float32_inputs else np.float64

    def _transform_features(self, part: DataFrame) -> Any:
        col, cols = self._transform_input_cols()
        dt = self._transform_dtype()
        if (col is not None and part.is_vector(col) and self._transform_supports_sparse()
                and vector_column_is_sparse(part.column(col))):
            return vector_column_to_csr(part.column(col), dt)
        # a multi-batch array column stays per-batch views (ChunkedRows): ``to_device`` streams
        # them without a host concatenation (1M x 3000 = a 12 GB copy before any PCIe transfer)
        return _dense_from_df(part, col, cols, dt, chunked=True)

    def _output_is_vector(self, df: DataFrame, out_col: str) -> bool:
        """probability/rawPrediction are vectors; array outputs mirror a vector input column."""
        return out_col in self._vector_output_cols()

    def _vector_output_cols(self) -> List[str]:
        return []

    def _spark_vector_output_cols(self, input_is_vector: bool) -> List[str]:
        """Output columns a Spark transform returns as VectorUDT (reference ``core.py:1559-1610``:
        probability / rawPrediction always; array outputs mirror a vector input column)."""
        return [c for c in self._vector_output_cols() if c]

    def _spark_output_fields(self, sdf: Any) -> List[Any]:
        """Spark schema of the columns ``transform`` appends (prediction double, array outputs)."""
        from pyspark.sql.types import ArrayType, DoubleType, StructField  # type: ignore

        out = []
        for pname, arr in (("predictionCol", False), ("probabilityCol", True), ("rawPredictionCol", True),
                           ("outputCol", True)):
            if self.hasParam(pname) and self.isDefined(pname) and self.getOrDefault(pname):
                out.append(StructField(self.getOrDefault(pname), ArrayType(DoubleType()) if arr else DoubleType()))
        return out

    def _device(self) -> torch.device:
        ctx = current_context()
        if ctx is not None:
            return ctx.device
        from ..parallel.context import local_device

        return local_device()

    def transform(self, dataset: Any, params: Optional[Dict[Param, Any]] = None) -> Any:
        if params:
            return self.copy(params)._transform(dataset)
        return self._transform(dataset)

    def _transform(self, dataset: Any) -> Any:
        from ..parallel.spark import is_spark_dataframe, spark_transform

        if is_spark_dataframe(dataset):
            return spark_transform(self, dataset)
        df, kind = as_dataframe(dataset)
        out = self._transform_df(df)
        return restore_kind(out, kind)

    def _transform_df(self, df: DataFrame) -> DataFrame:
        construct, predict = self._get_transform_func(df)
        ctx = current_context() or WorkerContext.single(self._device())
        state = construct(ctx)
        results: List[Dict[str, np.ndarray]] = []
        for p in df.partitions:
            part = DataFrame([p])
            if p.num_rows == 0:
                results.append({})
                continue
            X = self._transform_features(part)
            results.append(predict(state, X, ctx))
        names = [k for r in results for k in r.keys()]
        names = list(dict.fromkeys(names))
        out_parts = []
        vec_cols = set(self._vector_output_cols())
        for p, r in zip(df.partitions, results):
            part = DataFrame([p])
            for name in names:
                v = r.get(name)
                if v is None:
                    v = np.zeros((0,), dtype=np.float64)
                if isinstance(v, np.ndarray) and v.ndim == 2 and name in vec_cols:
                    from .dataframe import dense_to_vector_array

                    part = part.withColumn(name, dense_to_vector_array(v), vector=True)
                else:
                    part = part.withColumn(name, v)
            out_parts.append(part.partitions[0])
        return DataFrame(out_parts)

    # ---- evaluation in the transform pass (CrossValidator fast path) ----------------------
    def _transformEvaluate(self, dataset: Any, evaluator: Any, num_models: int = 1, params: Any = None) -> List[float]:
        """Transform + evaluate every combined model in ONE pass over ``dataset`` (reference
        ``core.py:1318-1468``). Each partition's features are moved to the device once, all models
        predict from that copy, and the partition emits only mergeable sufficient statistics per
        model (``metrics.ClassificationSummary`` — per-class tp / fp / label counts + log-loss
        sum — or ``RegressionSummary`` — moments of [label, label - prediction, prediction]); the
        predictions themselves never leave the worker. Partitions run where the data lives: Spark
        tasks (``mapInArrow``), the ranks of an SPMD job (summaries all-gathered, every rank gets
        the metrics) or LocalBarrierRunner workers; the driver merges the records (Chan merges)
        and applies Spark's formulas."""
        models = getattr(self, "_combined_models", None) or [self]
        if params:
            models = [m.copy(params) for m in models]
        info = _eval_info(evaluator)
        label_col = evaluator.getLabelCol()
        from ..parallel.spark import is_spark_dataframe

        if is_spark_dataframe(dataset):
            if label_col not in dataset.columns:
                raise RuntimeError("Label column is not existing.")
            partials = _spark_eval_partials(models, dataset, label_col, info)
        else:
            df, _ = as_dataframe(dataset)
            if label_col not in df.columns:
                raise RuntimeError("Label column is not existing.")
            if spmd_active():
                ctx = current_context() or spmd_context()
                mine = _eval_worker(ctx, (models, df.partitions, label_col, info))
                partials = [p for r in ctx.comm.allgather_object(mine) for p in r]
            elif self.num_workers > 1 and df.getNumPartitions() > 1:
                nw = min(self.num_workers, df.getNumPartitions())
                parts = df.repartition(nw).partitions if df.getNumPartitions() != nw else df.partitions
                res = run_worker_job(_eval_worker, [(models, [p], label_col, info) for p in parts])
                partials = [p for r in res for p in r]
            else:
                ctx = current_context() or WorkerContext.single(self._device())
                partials = _eval_worker(ctx, (models, df.partitions, label_col, info))
        return [_metric_from_partials([p[i] for p in partials], info, evaluator) for i in range(len(models))]

    @classmethod
    def _combine(cls, models: List["_Model"]) -> "_Model":
        raise NotImplementedError()

    def write(self) -> ModelWriter:
        return ModelWriter(self)

    @classmethod
    def read(cls) -> ModelReader:
        return ModelReader(cls)


class _ModelWithPredictionCol(_Model):
    @property
    def numFeatures(self) -> int:
        n = self._model_attributes.get("n_cols")
        return int(n) if n else -1


def _have_pyspark() -> bool:
    try:
        import pyspark  # noqa: F401

        return True
    except Exception:  # noqa: BLE001
        return False


# --------------------------------------------------------------------------------------
# single-pass transform-evaluate helpers
# --------------------------------------------------------------------------------------
def _eval_info(evaluator: Any) -> Tuple[str, bool, float]:
    """(kind, needs probabilities, eps) of a supported evaluator (pyspark's or ours)."""
    name = type(evaluator).__name__
    if name == "RegressionEvaluator":
        return "regression", False, 0.0
    if name == "MulticlassClassificationEvaluator":
        logloss = evaluator.getMetricName() == "logLoss"
        eps = float(evaluator.getOrDefault("eps")) if evaluator.hasParam("eps") else 1e-15
        return "classification", logloss, eps
    raise ValueError("transform-evaluate does not support %s" % name)


def _eval_worker(ctx: WorkerContext, payload: Tuple[Any, ...]) -> List[List[Any]]:
    """Per-partition summaries of every model: [[summary of model i] for each non-empty partition].

    The predictions stay on the device (``ctx.device_outputs``): the confusion counts, the log-loss
    sum and the regression moments are reduced there (``ops.confusion_counts`` / ``logloss_sum`` /
    ``reg_moments``, reference classification.py:113-155 / regression.py:144-173) and only those
    C x C / 12-double partials come to the host."""
    from .. import ops
    from ..metrics import ClassificationSummary, RegressionSummary

    models, tables, label_col, (kind, need_prob, eps) = payload
    fns = [m._get_transform_func(None) for m in models]
    states = [c(ctx) for c, _ in fns]
    dt = torch.float32 if models[0]._transform_dtype() == np.float32 else torch.float64
    out = []
    prev = ctx.device_outputs
    ctx.device_outputs = True
    try:
        for t in tables:
            if t is None or t.num_rows == 0:
                continue
            part = DataFrame([t])
            Xd = to_device(models[0]._transform_features(part), ctx.device, dt)
            y = part.to_numpy(label_col, np.float64)
            yd = torch.from_numpy(y).to(ctx.device)
            row = []
            for m, (_, predict), st in zip(models, fns, states):
                res = predict(st, Xd, ctx)
                p = res[m.getOrDefault("predictionCol")]
                if not isinstance(p, torch.Tensor):  # a model without device outputs: host summary
                    p = np.asarray(p, np.float64)
                    if kind == "regression":
                        row.append(RegressionSummary.from_arrays(y, p))
                    else:
                        prob = np.asarray(res[m.getOrDefault("probabilityCol")]) if need_prob else None
                        row.append(ClassificationSummary.from_arrays(y, p, prob, eps))
                    continue
                if kind == "regression":
                    row.append(RegressionSummary.from_moments(len(y), ops.reg_moments(yd, p)))
                    continue
                prob = res.get(m.getOrDefault("probabilityCol"))
                width = int(prob.shape[1]) if isinstance(prob, torch.Tensor) and prob.dim() == 2 else 0
                finite = bool(np.isfinite(y).all()) if len(y) else True
                C = max(width, int(y.max()) + 1 if len(y) and finite else 1, 1)
                # the device C x C histogram takes C <= CONFUSION_MAX_CLASSES and finite labels
                cm = ops.confusion_counts(yd, p, C) if finite and C <= ops.CONFUSION_MAX_CLASSES else None
                if cm is None:  # a label / prediction outside [0, C): the host path handles any values
                    ph = p.double().cpu().numpy()
                    row.append(ClassificationSummary.from_arrays(
                        y, ph, prob.cpu().numpy() if need_prob and prob is not None else None, eps))
                    continue
                ll = ops.logloss_sum(prob, yd, eps) if need_prob and prob is not None else 0.0
                row.append(ClassificationSummary.from_confusion(cm, len(y), ll))
            out.append(row)
    finally:
        ctx.device_outputs = prev
    return out


def _eval_task(ctx: WorkerContext, table: Any, extra: Tuple[Any, ...]) -> Iterator[Any]:
    """Spark partition -> one row holding the pickled per-model summaries (nothing else leaves)."""
    import cloudpickle

    models, label_col, info = extra
    rows = _eval_worker(ctx, (models, [table], label_col, info))
    yield pa.RecordBatch.from_pydict({"result": pa.array([cloudpickle.dumps(rows)], type=pa.binary())})


def _spark_eval_partials(models: List[Any], sdf: Any, label_col: str, info: Tuple[str, bool, float]) -> List[Any]:
    import cloudpickle

    from ..parallel.spark import spark_map_partitions

    col, cols = models[0]._transform_input_cols()
    sel = ([col] if col else list(cols)) + [label_col]
    out = spark_map_partitions(sdf.select(*sel), _eval_task, (models, label_col, info), "result binary")
    return [p for r in out.collect() for p in cloudpickle.loads(r["result"])]


def _metric_from_partials(parts: List[Any], info: Tuple[str, bool, float], evaluator: Any) -> float:
    from ..metrics import ClassificationSummary, MulticlassMetrics, RegressionMetrics, RegressionSummary

    if info[0] == "regression":
        s = RegressionSummary()
        for p in parts:
            s = s.merge(p)
        return float(RegressionMetrics(s).evaluate(evaluator))
    c = ClassificationSummary()
    for p in parts:
        c = c.merge(p)
    return float(MulticlassMetrics(c).evaluate(evaluator))
