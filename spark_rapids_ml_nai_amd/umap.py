"""``umap.UMAP`` / ``UMAPModel`` (reference ``umap.py:90-1327``).

Like the reference, the fit runs on ONE device over the whole (optionally ``sample_fraction``
sampled) dataset and the model keeps ``embedding_`` (N x n_components) and ``raw_data_``
(N x n_features); ``transform`` is data-parallel over partitions and outputs only the features
and the embedding columns (``umap.py:1149-1241``). Persistence writes the two matrices as
``.npy`` files next to the JSON metadata (``umap.py:1262-1327``).

Supported: euclidean / l2 / sqeuclidean / cosine / correlation metrics, ``init`` spectral or
random, supervised fits through ``labelCol`` (categorical target intersection), ``a``/``b``
overrides, ``precomputed_knn`` (indices, distances), ``random_state``.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .core.base import _dense_from_df, _Estimator, _Model, run_worker_job
from .core.dataframe import DataFrame, as_dataframe
from .core.params import (
    HasFeaturesCol,
    HasFeaturesCols,
    HasLabelCol,
    HasOutputCol,
    Param,
    Params,
    TypeConverters,
    _BackendClass,
    _BackendParams,
    _FeaturesColMixin,
    keyword_only,
)
from .parallel.context import WorkerContext

_UMAP_KEYS = ("n_neighbors", "n_components", "metric", "n_epochs", "learning_rate", "init", "min_dist", "spread",
              "set_op_mix_ratio", "local_connectivity", "repulsion_strength", "negative_sample_rate",
              "transform_queue_size", "a", "b", "precomputed_knn", "random_state", "build_algo", "build_kwds")


class UMAPClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {k: k for k in _UMAP_KEYS}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {
            "n_neighbors": 15, "n_components": 2, "metric": "euclidean", "n_epochs": None, "learning_rate": 1.0,
            "init": "spectral", "min_dist": 0.1, "spread": 1.0, "set_op_mix_ratio": 1.0, "local_connectivity": 1.0,
            "repulsion_strength": 1.0, "negative_sample_rate": 5, "transform_queue_size": 4.0, "a": None, "b": None,
            "precomputed_knn": None, "random_state": None, "build_algo": "auto", "build_kwds": None,
            "verbose": False,
        }


def _p(name: str, doc: str, conv: Callable) -> Param:
    return Param(Params._dummy(), name, doc, typeConverter=conv)


class _UMAPParams(_FeaturesColMixin, _BackendParams, HasFeaturesCol, HasFeaturesCols, HasLabelCol, HasOutputCol):
    n_neighbors = _p("n_neighbors", "The size of local neighborhood used for manifold approximation.",
                     TypeConverters.toFloat)
    n_components = _p("n_components", "The dimension of the space to embed into.", TypeConverters.toInt)
    metric = _p("metric", "Distance metric (euclidean, l2, sqeuclidean, cosine, correlation).", TypeConverters.toString)
    n_epochs = _p("n_epochs", "The number of training epochs (None: 500 for small, 200 for large datasets).",
                  TypeConverters.identity)
    learning_rate = _p("learning_rate", "The initial learning rate for the embedding optimization.",
                       TypeConverters.toFloat)
    init = _p("init", "How to initialize the low dimensional embedding: 'spectral' or 'random'.",
              TypeConverters.toString)
    min_dist = _p("min_dist", "The effective minimum distance between embedded points.", TypeConverters.toFloat)
    spread = _p("spread", "The effective scale of embedded points.", TypeConverters.toFloat)
    set_op_mix_ratio = _p("set_op_mix_ratio", "Interpolate between fuzzy union (1.0) and intersection (0.0).",
                          TypeConverters.toFloat)
    local_connectivity = _p("local_connectivity", "The local connectivity required.", TypeConverters.toFloat)
    repulsion_strength = _p("repulsion_strength", "Weighting applied to negative samples.", TypeConverters.toFloat)
    negative_sample_rate = _p("negative_sample_rate", "Negative samples per positive sample.", TypeConverters.toInt)
    transform_queue_size = _p("transform_queue_size", "Accepted for compatibility (exact kNN is used).",
                              TypeConverters.toFloat)
    a = _p("a", "More specific parameters controlling the embedding.", TypeConverters.identity)
    b = _p("b", "More specific parameters controlling the embedding.", TypeConverters.identity)
    precomputed_knn = _p("precomputed_knn", "(indices, distances) of a precomputed kNN graph.",
                         TypeConverters.identity)
    random_state = _p("random_state", "Seed of the pseudo random number generator.", TypeConverters.identity)
    sample_fraction = _p("sample_fraction", "Fraction of the dataset used for fitting.", TypeConverters.toFloat)
    build_algo = _p("build_algo", "kNN graph construction: 'auto' (exact up to 100k rows, IVF lists beyond), "
                    "'brute_force_knn', 'ivf' (per-query IVF probing) or 'nn_descent' (the IVF graph refined by "
                    "NN-descent rounds).", TypeConverters.toString)
    build_kwds = _p("build_kwds", "kNN graph options, e.g. {'nlist': ..., 'nprobe': ..., 'probe': 'query' | 'list', "
                    "'nnd_iters': ...} for build_algo='ivf' / 'nn_descent'.", TypeConverters.identity)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(n_neighbors=15, n_components=2, metric="euclidean", n_epochs=None, learning_rate=1.0,
                         init="spectral", min_dist=0.1, spread=1.0, set_op_mix_ratio=1.0, local_connectivity=1.0,
                         repulsion_strength=1.0, negative_sample_rate=5, transform_queue_size=4.0, a=None, b=None,
                         precomputed_knn=None, random_state=None, sample_fraction=1.0, outputCol="embedding",
                         featuresCol="features", build_algo="auto", build_kwds=None)

    def getSampleFraction(self) -> float:
        return self.getOrDefault(self.sample_fraction)

    def setSampleFraction(self, value: float) -> Any:
        return self._set_params(sample_fraction=value)

    def setOutputCol(self, value: str) -> Any:
        return self._set_params(outputCol=value)

    def _umap_params(self) -> Dict[str, Any]:
        d = {k: self._backend_params.get(k) for k in _UMAP_KEYS}
        d["n_neighbors"] = int(d["n_neighbors"]) if d["n_neighbors"] is not None else 15
        return d

    def _features(self, df: DataFrame) -> np.ndarray:
        fc = self.getFeaturesCol()
        col, cols = (fc, None) if isinstance(fc, str) else (None, list(fc))
        return _dense_from_df(df, col, cols, np.float32)


for _n in _UMAP_KEYS:
    _cap = "".join(p.capitalize() for p in _n.split("_"))
    _cap = _cap[0].lower() + _cap[1:]
    if not hasattr(_UMAPParams, "get" + _cap[0].upper() + _cap[1:]):
        setattr(_UMAPParams, "get" + _cap[0].upper() + _cap[1:], lambda self, _k=_n: self.getOrDefault(_k))
    if not hasattr(_UMAPParams, "set" + _cap[0].upper() + _cap[1:]):
        setattr(_UMAPParams, "set" + _cap[0].upper() + _cap[1:], lambda self, v, _k=_n: self._set_params(**{_k: v}))


def _umap_fit_worker(ctx: WorkerContext, payload: Tuple[Any, ...]) -> Tuple[np.ndarray, np.ndarray]:
    from .core.base import to_device
    from .models.umap import umap_fit

    X, y, params = payload[:3]
    every_rank = len(payload) > 3 and bool(payload[3])
    Xh = np.ascontiguousarray(X, dtype=np.float32)
    Xd = to_device(Xh, ctx.device, torch.float32)
    yd = torch.as_tensor(np.asarray(y), device=ctx.device) if y is not None else None
    if ctx.world_size > 1:
        # every rank holds the whole (sampled) training set: device all-gather over RCCL
        Xd = torch.cat([p.to(ctx.device) for p in ctx.comm.allgatherv(Xd)], 0)
        if yd is not None:
            yd = torch.cat([p.to(ctx.device) for p in ctx.comm.allgatherv(yd)], 0)
    emb = umap_fit(Xd, params, yd, ctx=ctx)
    # in-process / Spark jobs build the model from rank 0's result only; an SPMD (torchrun) fit
    # asks every rank for its own model (the layouts are identical: one all-reduce per epoch)
    if ctx.rank != 0 and not every_rank:
        return None, None
    # the model's raw_data_: one rank already holds all rows on the host (no 4 B x N x n copy back
    # from the device: ~0.5 s at 20M x 128); several ranks return the device-gathered rows
    return emb, (Xh if ctx.world_size == 1 else Xd.cpu().numpy())


def _spark_umap_task(ctx: WorkerContext, table: Any, extra: Tuple[Any, ...]) -> Any:
    """One rank of the Spark UMAP fit (barrier job): the ranks' rows are device-gathered and fitted
    together (``_umap_fit_worker``); rank 0 then YIELDS the result as Arrow record batches of at most
    ``maxRecordsPerBatch`` rows — one row per training sample, ``embedding_`` and ``raw_data_`` as
    float lists — so no Arrow cell / task result holds the whole model (the reference streams
    ``maxRecordsPerBatch``-row sections, ``umap.py:1060-1073``). The reference fits in ONE
    non-barrier task on one GPU (``umap.py:830-909``); ``num_workers=1`` gives exactly that."""
    col, cols, label_col, params, rows_per_batch = extra
    if table is not None and table.num_rows:
        part = DataFrame([table])
        X = _dense_from_df(part, col, cols, np.float32)
        y = part.to_numpy(label_col).astype(np.int64) if label_col else None
    else:
        X, y = None, (np.zeros(0, np.int64) if label_col else None)
    nt = torch.tensor([float(X.shape[1] if X is not None else 0)], dtype=torch.float64, device=ctx.device)
    ctx.comm.allreduce(nt, op="max")
    if X is None:
        X = np.zeros((0, int(nt.item())), np.float32)
    emb, Xall = _umap_fit_worker(ctx, (X, y, params))
    if emb is None:
        return
    import pyarrow as pa

    from .core.dataframe import dense_to_list_array

    step = max(1, int(rows_per_batch))
    for r0 in range(0, emb.shape[0], step):
        yield pa.RecordBatch.from_arrays([dense_to_list_array(np.ascontiguousarray(emb[r0: r0 + step])),
                                          dense_to_list_array(np.ascontiguousarray(Xall[r0: r0 + step]))],
                                         names=["embedding_", "raw_data_"])


def _chunk_rows(arr: np.ndarray, limit: int) -> List[np.ndarray]:
    """Row slices of ``arr`` of at most ``limit`` bytes each (one row at least): the pieces that
    are broadcast separately (reference ``_chunk_arr``, ``umap.py:873-885``)."""
    if arr.nbytes <= limit or arr.shape[0] <= 1:
        return [arr]
    row_bytes = max(1, arr.nbytes // arr.shape[0])
    step = max(1, int(limit) // row_bytes)
    return [arr[i: i + step] for i in range(0, arr.shape[0], step)]


class _BroadcastChunks:
    """A driver array shipped to Spark tasks as a list of broadcasts (each <= BROADCAST_LIMIT);
    ``value()`` reassembles it once per executor process. The cache holds every array of ONE model
    (``group``: its embedding and its raw rows side by side); loading an array of another model
    evicts the previous model's arrays only."""

    _cache: Dict[Tuple[str, str], np.ndarray] = {}

    def __init__(self, spark: Any, arr: np.ndarray, limit: int, group: str, name: str) -> None:
        self.group = group
        self.key = (group, name)
        self.shape = tuple(arr.shape)
        self.chunks = [spark.sparkContext.broadcast(c) for c in _chunk_rows(arr, limit)]

    def __len__(self) -> int:
        return len(self.chunks)

    def value(self) -> np.ndarray:
        cache = _BroadcastChunks._cache
        v = cache.get(self.key)
        if v is None:
            parts = [np.asarray(b.value) for b in self.chunks]
            v = parts[0] if len(parts) == 1 else np.concatenate(parts, 0)
            for k in [k for k in cache if k[0] != self.group]:
                del cache[k]  # keep one model's training data per executor process
            cache[self.key] = v
        return v

    def unpersist(self) -> None:
        for b in self.chunks:
            try:
                b.unpersist()
            except Exception:  # noqa: BLE001
                pass


class UMAP(UMAPClass, _Estimator, _UMAPParams):
    """Uniform Manifold Approximation and Projection.

    ``BROADCAST_LIMIT`` (bytes, default 8 GiB like the reference): the fitted embedding and raw
    rows reach Spark transform tasks as broadcasts of at most this size each.

    >>> from spark_rapids_ml_nai_amd.umap import UMAP
    >>> model = UMAP(n_neighbors=15, n_components=2, random_state=1).fit(df)  # doctest: +SKIP
    >>> model.transform(df).select("embedding")  # doctest: +SKIP
    """

    @keyword_only
    def __init__(self, *, n_neighbors: Optional[float] = 15, n_components: Optional[int] = 2,
                 metric: str = "euclidean", n_epochs: Optional[int] = None, learning_rate: Optional[float] = 1.0,
                 init: Optional[str] = "spectral", min_dist: Optional[float] = 0.1, spread: Optional[float] = 1.0,
                 set_op_mix_ratio: Optional[float] = 1.0, local_connectivity: Optional[float] = 1.0,
                 repulsion_strength: Optional[float] = 1.0, negative_sample_rate: Optional[int] = 5,
                 transform_queue_size: Optional[float] = 4.0, a: Optional[float] = None, b: Optional[float] = None,
                 precomputed_knn: Optional[Any] = None, random_state: Optional[int] = None,
                 sample_fraction: Optional[float] = 1.0, featuresCol: Optional[Union[str, List[str]]] = None,
                 labelCol: Optional[str] = None, outputCol: Optional[str] = None, num_workers: Optional[int] = None,
                 verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._set_params(**self._input_kwargs)

    BROADCAST_LIMIT = 8 << 30

    def _get_fit_func(self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        raise NotImplementedError("UMAP fits through _fit")

    def _create_model(self, result: Dict[str, Any]) -> "UMAPModel":
        return UMAPModel._from_row(result)

    def _spark_fit(self, sdf: Any) -> Tuple[np.ndarray, np.ndarray]:
        from .parallel.spark import spark_barrier_job

        frac = self.getSampleFraction()
        if frac is not None and frac < 1.0:
            sdf = sdf.sample(False, frac, seed=self._backend_params.get("random_state"))
        fc = self.getFeaturesCol()
        col, cols = (fc, None) if isinstance(fc, str) else (None, list(fc))
        label = self.getLabelCol() if self.isDefined("labelCol") and self.getLabelCol() in sdf.columns else None
        sel = ([col] if col else list(cols)) + ([label] if label else [])
        from pyspark.sql.types import ArrayType, FloatType, StructField, StructType  # type: ignore

        from .parallel.spark import collect_arrow

        rows = int(sdf.sparkSession.conf.get("spark.sql.execution.arrow.maxRecordsPerBatch", "10000"))
        if rows <= 0:  # Spark reads <= 0 as "no limit": one batch per 10k rows, not one per row
            rows = 10000
        schema = StructType([StructField("embedding_", ArrayType(FloatType(), False), False),
                             StructField("raw_data_", ArrayType(FloatType(), False), False)])
        out = spark_barrier_job(sdf.select(*sel).repartition(max(1, self.num_workers)), _spark_umap_task,
                                (col, cols, label, self._umap_params(), rows), out_schema=schema)
        t = collect_arrow(out)
        from .core.dataframe import array_column_to_dense

        self._fit_result_batches = int(sum(c.num_chunks for c in t.columns[:1]))
        return (array_column_to_dense(t.column("embedding_"), np.float32),
                array_column_to_dense(t.column("raw_data_"), np.float32))

    def _fit(self, dataset: Any) -> "UMAPModel":
        from .parallel.spark import is_spark_dataframe

        if is_spark_dataframe(dataset):
            emb, Xall = self._spark_fit(dataset)
            return self._make_model(emb, Xall)
        df, _ = as_dataframe(dataset)
        frac = self.getSampleFraction()
        if frac is not None and frac < 1.0:
            seed = self._backend_params.get("random_state")
            df = df.sample(frac, seed=seed)
        y = None
        if self.isDefined("labelCol") and self.getLabelCol() in df.columns:
            y = df.to_numpy(self.getLabelCol()).astype(np.int64)
        params = self._umap_params()
        # The reference fits on ONE device (umap.py:840-850). Here num_workers > 1 (or SPMD)
        # fits on all ranks: replicated rows, distributed kNN graph, edge-parallel SGD.
        from .core.base import spmd_active

        nw = self.num_workers
        if spmd_active() or nw <= 1:
            payloads = [(self._features(df), y, params, spmd_active())]
        else:
            if df.getNumPartitions() != nw:
                df = df.repartition(nw)
            payloads = []
            for p in df.partitions:
                part = DataFrame([p])
                yp = part.to_numpy(self.getLabelCol()).astype(np.int64) if y is not None else None
                payloads.append((self._features(part), yp, params))
        emb, Xall = run_worker_job(_umap_fit_worker, payloads)[0]
        return self._make_model(emb, Xall)

    def _make_model(self, emb: np.ndarray, Xall: np.ndarray) -> "UMAPModel":
        model = UMAPModel(embedding_=emb, raw_data_=Xall, n_cols=int(Xall.shape[1]), dtype="float32")
        model.BROADCAST_LIMIT = int(self.BROADCAST_LIMIT)
        model._num_workers = self._num_workers
        model._float32_inputs = True
        self._copyValues(model)
        self._copy_backend_params(model)
        return model


class UMAPModel(UMAPClass, _Model, _UMAPParams):
    BROADCAST_LIMIT = 8 << 30

    def __init__(self, embedding_: Any, raw_data_: Any, n_cols: int, dtype: str) -> None:
        emb = np.asarray(embedding_, dtype=np.float32)
        raw = np.asarray(raw_data_, dtype=np.float32)
        super().__init__(embedding_=emb, raw_data_=raw, n_cols=n_cols, dtype=dtype)
        self.embedding_ = emb
        self.raw_data_ = raw
        self.n_cols = int(n_cols)
        self.dtype = dtype

    @property
    def embedding(self) -> List[List[float]]:
        return self.embedding_.tolist()

    @property
    def raw_data(self) -> List[List[float]]:
        return self.raw_data_.tolist()

    def _spark_task_model(self, spark: Any) -> "UMAPModel":
        """The copy of this model that Spark transform tasks unpickle: embedding and raw rows as
        chunked broadcasts (<= BROADCAST_LIMIT bytes each, reference ``umap.py:873-895``), created
        once per model and reused by later transforms; nothing large is pickled into the closure."""
        import copy
        import uuid

        bc = getattr(self, "_broadcasts", None)
        if bc is None or bc[0] != int(self.BROADCAST_LIMIT):
            key = uuid.uuid4().hex
            bc = (int(self.BROADCAST_LIMIT),
                  _BroadcastChunks(spark, self.embedding_, self.BROADCAST_LIMIT, key, "e"),
                  _BroadcastChunks(spark, self.raw_data_, self.BROADCAST_LIMIT, key, "r"))
            self._broadcasts = bc
        light = copy.copy(self)
        light.embedding_ = np.zeros((0,) + self.embedding_.shape[1:], np.float32)
        light.raw_data_ = np.zeros((0,) + self.raw_data_.shape[1:], np.float32)
        light._model_attributes = {k: v for k, v in self._model_attributes.items()
                                   if k not in ("embedding_", "raw_data_")}
        light._device_state_cache = {}
        light._broadcasts = None
        light._sources = (bc[1], bc[2])
        return light

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        params = self._umap_params()
        out_col = self.getOutputCol()
        src = getattr(self, "_sources", None)
        emb, raw = (self.embedding_, self.raw_data_) if src is None else src

        def construct(ctx: WorkerContext) -> Tuple[torch.Tensor, torch.Tensor]:
            e, r = (emb, raw) if src is None else (emb.value(), raw.value())
            return torch.from_numpy(r).to(ctx.device), torch.from_numpy(e).to(ctx.device)

        def predict(state: Tuple[torch.Tensor, torch.Tensor], X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            from .core.base import to_device
            from .models.umap import umap_transform

            Rd, Ed = state
            Xd = to_device(np.asarray(X, dtype=np.float32), ctx.device, torch.float32)
            return {out_col: umap_transform(Xd, Rd, Ed, params)}

        return construct, predict

    def _transform(self, dataset: Any) -> Any:
        from .parallel.spark import is_spark_dataframe, spark_transform

        if is_spark_dataframe(dataset):
            # per-partition transform (kNN to the training rows + SGD placement); like the reference
            # the output holds the features and the embedding only (umap.py:1149-1241)
            fc = self.getFeaturesCol()
            out = spark_transform(self, dataset)
            return out.select(*(([fc] if isinstance(fc, str) else list(fc)) + [self.getOutputCol()]))
        return super()._transform(dataset)

    def _transform_df(self, df: DataFrame) -> DataFrame:
        out = super()._transform_df(df)
        fc = self.getFeaturesCol()
        if isinstance(fc, str):
            return out.select(fc, self.getOutputCol())
        # multi-column input: emit one "features" array column like the reference
        from .core.dataframe import dense_to_list_array

        parts = []
        for p in out.partitions:
            part = DataFrame([p])
            X = _dense_from_df(part, None, list(fc), np.float32)
            part = part.withColumn("features", dense_to_list_array(X))
            parts.append(part.select("features", self.getOutputCol()).partitions[0])
        return DataFrame(parts)
