"""Exact and approximate nearest neighbours — ``NearestNeighbors`` / ``ApproximateNearestNeighbors``.

API parity with the reference ``knn.py``:
* ``NearestNeighbors`` (``knn.py:188-392``): ``fit(item_df)`` only remembers the items (with an id
  column); ``NearestNeighborsModel.kneighbors(query_df)`` (558-624) returns
  ``(item_df_withid, query_df_withid, knn_df[query_<id>, indices, distances])``;
  ``exactNearestNeighborsJoin(query_df, distCol)`` (419-466, 753-782). Euclidean distances.
* ``ApproximateNearestNeighbors`` (``knn.py:889-1118``): ``algorithm="ivfflat"`` (plus ``"brute"``),
  ``algoParams={"nlist", "nprobe"}``, metrics euclidean / l2 / sqeuclidean / inner_product
  (1307-1312); ``kneighbors`` and ``approxSimilarityJoin`` (1398-1427). One IVF index per item
  partition, as in the reference.
* No persistence (``write/read/save/load`` raise — ``knn.py:368-392, 468-492, 1093-1118``).

Distances: ``euclidean``/``l2`` are true L2 distances, ``sqeuclidean`` squared L2 and
``inner_product`` the dot product (neighbours ordered by descending similarity).

Execution: items and queries are split over ``num_workers`` ranks; each rank all-gathers the
queries over RCCL, searches its local items with the MFMA kernels and the partial top-k lists are
merged on device (``models/knn.py``). Unlike the reference no item ids travel through a driver.
On a Spark DataFrame the same rank code runs as ONE barrier job over the tagged item u query
union for both classes (the reference's ANN instead broadcasts the queries to a non-barrier job
and merges with a SQL ``groupBy``; here the IVF partial lists are merged on the device); the join
methods use Spark SQL explode + joins on the ids.
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import pyarrow as pa

from .core.base import _dense_from_df, run_worker_job
from .core.dataframe import DataFrame, as_dataframe
from .core.params import (
    HasIDCol,
    HasInputCol,
    HasInputCols,
    Param,
    Params,
    TypeConverters,
    _BackendClass,
    _BackendParams,
    keyword_only,
)
from .core.persistence import MLReadable, MLWritable
from .parallel.context import WorkerContext, spmd_active

_DEFAULT_ID = "unique_id"


# ------------------------------------------------------------------------------------------
# worker closures (module level so cloudpickle ships them by reference)
# ------------------------------------------------------------------------------------------
def _agree_ncols(ctx: WorkerContext, items: np.ndarray, queries: np.ndarray) -> int:
    """Feature count every rank agrees on: a rank holding no items and no queries (an empty
    shard) learns it from the others, so it still joins every collective with the right shapes."""
    import torch

    n = items.shape[1] if items.ndim == 2 and items.shape[1] else (queries.shape[1] if queries.ndim == 2 else 0)
    if ctx.world_size > 1:
        nt = torch.tensor([float(n)], dtype=torch.float64, device=ctx.device)
        ctx.comm.allreduce(nt, op="max")
        n = int(nt.item())
    return n


def _exact_worker(ctx: WorkerContext, payload: Tuple[Any, ...]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    import torch

    from .core.base import to_device
    from .models.knn import exact_knn

    items, item_ids, queries, query_ids, k, metric = payload
    n = _agree_ncols(ctx, items, queries)
    X = to_device(items.reshape(-1, n), ctx.device, torch.float32)
    ids = torch.as_tensor(item_ids, dtype=torch.int64).to(ctx.device)
    Q = to_device(queries.reshape(-1, n), ctx.device, torch.float32)
    d, i = exact_knn(X, ids, Q, k, ctx, metric)
    return query_ids, i, d


def _ivf_worker(ctx: WorkerContext, payload: Tuple[Any, ...]) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    import torch

    from .core.base import to_device
    from .models.knn import build_ivf, exact_knn, ivf_knn

    items, item_ids, queries, query_ids, k, metric, algorithm, nlist, nprobe, seed, cache = payload
    n = _agree_ncols(ctx, items, queries)
    Q = to_device(queries.reshape(-1, n), ctx.device, torch.float32)
    X = to_device(items.reshape(-1, n), ctx.device, torch.float32)
    ids = torch.as_tensor(item_ids, dtype=torch.int64).to(ctx.device)
    if algorithm == "brute":
        d, i = exact_knn(X, ids, Q, k, ctx, metric)
        return query_ids, i, d
    index = None
    if X.shape[0] > 0:
        index = cache.get("index") if cache is not None else None
        if index is None or index.items.device != X.device:
            nl = nlist if nlist else _default_nlist(X.shape[0])
            index = build_ivf(X, ids, nl, seed)
            if cache is not None:
                cache["index"] = index
    npb = nprobe if nprobe else _default_nprobe(index.centroids.shape[0] if index is not None else 1)
    d, i = ivf_knn(index, Q, k, npb, ctx, metric)
    return query_ids, i, d


_TAG = "__srml_is_query"
_ITEM_KEY = "__srml_item_id"


def _spark_knn_task(ctx: WorkerContext, table: Any, extra: Tuple[Any, ...]) -> Any:
    """One rank of the Spark kNN barrier job over the item u query union (reference
    ``knn.py:638-749``): split the partition by the query tag, search this rank's items for every
    rank's queries (device ring over RCCL), emit (query id, indices, distances) for this rank's
    queries. Item ids stay on the device: no id list travels through the driver."""
    col, cols, id_col, qname, k, metric, ivf = extra
    if table is not None and table.num_rows:
        part = DataFrame([table])
        tag = np.asarray(part.to_numpy(_TAG)).astype(bool)
        ids = np.asarray(part.to_numpy(id_col)).astype(np.int64)
        X = _dense_from_df(part, col, cols, np.float32)
        items, item_ids, queries, query_ids = X[~tag], ids[~tag], X[tag], ids[tag]
    else:  # an empty rank still takes part in every collective (the workers agree on n)
        items, queries = np.zeros((0, 0), np.float32), np.zeros((0, 0), np.float32)
        item_ids, query_ids = np.zeros(0, np.int64), np.zeros(0, np.int64)
    if ivf is None:
        qid, ind, dist = _exact_worker(ctx, (items, item_ids, queries, query_ids, k, metric))
    else:
        qid, ind, dist = _ivf_worker(ctx, (items, item_ids, queries, query_ids, k, metric) + tuple(ivf) + (None,))
    yield _knn_batch(qname, np.asarray(qid, np.int64), np.asarray(ind), np.asarray(dist))


def _knn_batch(qname: str, qid: np.ndarray, ind: np.ndarray, dist: np.ndarray) -> Any:
    """(query id, indices list<int64>, distances list<float>) record batch; neighbours padded with
    -1 (k > number of items) are dropped from their row."""
    m = qid.shape[0]
    kk = ind.shape[1] if ind.ndim == 2 else 0
    valid = ind >= 0 if m else np.zeros((0, kk), bool)
    counts = valid.sum(1).astype(np.int32) if m else np.zeros(0, np.int32)
    offsets = pa.array(np.concatenate([[0], np.cumsum(counts)]).astype(np.int32))
    ind_a = pa.ListArray.from_arrays(offsets, pa.array(ind[valid].astype(np.int64) if m else np.zeros(0, np.int64)))
    dist_a = pa.ListArray.from_arrays(offsets, pa.array(dist[valid].astype(np.float32) if m else np.zeros(0, np.float32)))
    return pa.RecordBatch.from_arrays([pa.array(qid), ind_a, dist_a], names=[qname, "indices", "distances"])


def _default_nlist(m: int) -> int:
    return int(max(1, min(1024, round(np.sqrt(m)))))


def _default_nprobe(nlist: int) -> int:
    return int(max(1, min(nlist, 20)))


# ------------------------------------------------------------------------------------------
# params
# ------------------------------------------------------------------------------------------
class NearestNeighborsClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {"k": "n_neighbors"}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {"n_neighbors": 5, "verbose": False, "batch_size": 2000000}


class _NNParams(_BackendParams, HasInputCol, HasInputCols, HasIDCol):
    k = Param(Params._dummy(), "k", "The number nearest neighbors to retrieve. Must be >= 1.",
              typeConverter=TypeConverters.toInt)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(k=5, idCol=_DEFAULT_ID)

    def setK(self, value: int) -> Any:
        return self._set_params(k=value)

    def getK(self) -> int:
        return self.getOrDefault(self.k)

    def setInputCol(self, value: Union[str, List[str]]) -> Any:
        if isinstance(value, str):
            return self._set_params(inputCol=value)
        return self._set_params(inputCols=value)

    def setInputCols(self, value: List[str]) -> Any:
        return self._set_params(inputCols=value)

    def setIdCol(self, value: str) -> Any:
        return self._set_params(idCol=value)

    def _getIdColOrDefault(self) -> str:
        return self.getOrDefault("idCol")

    def _features(self, df: DataFrame) -> np.ndarray:
        col, cols = self._get_input_columns()
        if col is None and not cols:
            col = "features" if "features" in df.columns else None
        if col is None and not cols:
            raise ValueError("set inputCol or inputCols")
        if df.count() == 0:
            return np.zeros((0, 0), dtype=np.float32)
        return _dense_from_df(df, col, cols, np.float32)


class _NoPersistence(MLWritable, MLReadable):
    def write(self) -> Any:
        raise NotImplementedError("%s does not support saving/loading, just re-fit the estimator to re-create a model."
                                  % self.__class__.__name__)

    @classmethod
    def read(cls) -> Any:
        raise NotImplementedError("%s does not support saving/loading, just re-fit the estimator to re-create a model."
                                  % cls.__name__)

    def save(self, path: str) -> None:
        raise NotImplementedError("%s does not support saving/loading, just re-create the estimator."
                                  % self.__class__.__name__)

    @classmethod
    def load(cls, path: str) -> Any:
        raise NotImplementedError("%s does not support saving/loading, just re-create the estimator." % cls.__name__)


def _split(df: DataFrame, parts: int) -> List[DataFrame]:
    if df.getNumPartitions() != parts:
        df = df.repartition(parts)
    return [DataFrame([p]) for p in df.partitions]


class _NNModelBase(_NoPersistence, _NNParams):
    _item_df_withid: DataFrame

    def _transform(self, dataset: Any) -> Any:
        raise NotImplementedError("%s does not provide a transform function. Use 'kneighbors' instead."
                                  % self.__class__.__name__)

    transform = _transform  # type: ignore[assignment]

    def _metric(self) -> str:
        return "euclidean"

    def _payload_extra(self) -> Tuple[Any, ...]:
        return ()

    def _worker(self) -> Any:
        return _exact_worker

    def _ivf_args(self) -> Optional[Tuple[Any, ...]]:
        return None

    def _feature_spec(self) -> Tuple[Optional[str], Optional[List[str]]]:
        col, cols = self._get_input_columns()
        if col is None and not cols:
            col = "features"
        return col, cols

    def _spark_kneighbors(self, query_df: Any, sort_knn_df_by_query_id: bool) -> Tuple[Any, Any, Any]:
        """Spark path: ONE barrier job over items u queries (tagged), like the reference
        (``knn.py:558-624``); the result is a lazily computed Spark DataFrame."""
        from pyspark.sql import functions as F  # type: ignore
        from pyspark.sql.types import ArrayType, FloatType, LongType, StructField, StructType  # type: ignore

        from .parallel.spark import spark_barrier_job

        query_df_withid = self._ensureIdCol(query_df)
        id_col = self._getIdColOrDefault()
        col, cols = self._feature_spec()
        sel = ([col] if col else list(cols)) + [id_col]
        union = self._item_df_withid.select(*sel).withColumn(_TAG, F.lit(0)).union(
            query_df_withid.select(*sel).withColumn(_TAG, F.lit(1)))
        nw = max(1, self.num_workers)
        union = union.repartition(nw)
        qname = "query_%s" % id_col
        schema = StructType([StructField(qname, LongType()), StructField("indices", ArrayType(LongType())),
                             StructField("distances", ArrayType(FloatType()))])
        k = self.getK()
        if k < 1:
            raise ValueError("k must be >= 1")
        knn_df = spark_barrier_job(union, _spark_knn_task, (col, cols, id_col, qname, k, self._metric(),
                                                            self._ivf_args()), schema)
        if sort_knn_df_by_query_id:
            knn_df = knn_df.sort(qname)
        return self._item_df_withid, query_df_withid, knn_df

    def _spark_join(self, query_df: Any, distCol: str) -> Any:
        """Every (query, neighbour) pair as ``item_df`` / ``query_df`` structs + distance, with Spark
        SQL explode + joins on the ids (reference ``knn.py:419-466``)."""
        from pyspark.sql import functions as F  # type: ignore

        id_col = self._getIdColOrDefault()
        item_df, query_df_withid, knn_df = self._spark_kneighbors(query_df, False)
        qname = "query_%s" % id_col
        pairs = knn_df.select(F.col(qname), F.explode(F.arrays_zip("indices", "distances")).alias("__z"))
        pairs = pairs.select(F.col(qname), F.col("__z.indices").alias(_ITEM_KEY), F.col("__z.distances").alias(distCol))
        keep_id = self.isSet("idCol")
        icols = [c for c in item_df.columns if keep_id or c != id_col]
        qcols = [c for c in query_df_withid.columns if keep_id or c != id_col]
        items = item_df.select(F.struct(*icols).alias("item_df"), F.col(id_col).alias(_ITEM_KEY))
        queries = query_df_withid.select(F.struct(*qcols).alias("query_df"), F.col(id_col).alias(qname))
        return pairs.join(items, on=_ITEM_KEY).join(queries, on=qname).select("item_df", "query_df", distCol)

    def kneighbors(self, query_df: Any, sort_knn_df_by_query_id: bool = True) -> Tuple[DataFrame, DataFrame, DataFrame]:
        """Return ``(item_df_withid, query_df_withid, knn_df)``; knn_df has one row per query:
        ``query_<idCol>``, ``indices`` (array of item ids) and ``distances`` (array<float>)."""
        from .parallel.spark import is_spark_dataframe

        if is_spark_dataframe(self._item_df_withid) or is_spark_dataframe(query_df):
            return self._spark_kneighbors(query_df, sort_knn_df_by_query_id)
        query_df, _ = as_dataframe(query_df)
        query_df_withid = self._ensureIdCol(query_df)
        id_col = self._getIdColOrDefault()
        k = self.getK()
        if k < 1:
            raise ValueError("k must be >= 1")
        if spmd_active():
            # torchrun: this process is one rank and its frames are its whole shard (ids already
            # global from _ensureIdCol); the rank returns the neighbours of its own queries
            items, queries = [self._item_df_withid], [query_df_withid]
        else:
            nw = max(1, self.num_workers)
            items = _split(self._item_df_withid, nw)
            queries = _split(query_df_withid, nw)
        payloads = []
        for it, q in zip(items, queries):
            payloads.append((self._features(it), it.to_numpy(id_col).astype(np.int64), self._features(q),
                             q.to_numpy(id_col), k, self._metric()) + self._payload_extra())
        results = run_worker_job(self._worker(), payloads)
        qid = np.concatenate([r[0] for r in results])
        ind = np.concatenate([r[1] for r in results]) if results else np.zeros((0, k), np.int64)
        dist = np.concatenate([r[2] for r in results]) if results else np.zeros((0, k), np.float32)
        # drop padding of k > number of items
        valid = ind >= 0
        if not valid.all():
            ind_l = [row[v].tolist() for row, v in zip(ind, valid)]
            dist_l = [row[v].astype(np.float32).tolist() for row, v in zip(dist, valid)]
            ind_a, dist_a = pa.array(ind_l, pa.list_(pa.int64())), pa.array(dist_l, pa.list_(pa.float32()))
        else:
            ind_a = pa.ListArray.from_arrays(pa.array(np.arange(0, ind.size + 1, max(ind.shape[1], 1), dtype=np.int32)
                                                      if ind.size else np.zeros(ind.shape[0] + 1, np.int32)),
                                             pa.array(ind.reshape(-1).astype(np.int64)))
            dist_a = pa.ListArray.from_arrays(pa.array(np.arange(0, dist.size + 1, max(dist.shape[1], 1), dtype=np.int32)
                                                       if dist.size else np.zeros(dist.shape[0] + 1, np.int32)),
                                              pa.array(dist.reshape(-1).astype(np.float32)))
        qname = "query_%s" % id_col
        table = pa.table({qname: pa.array(qid), "indices": ind_a, "distances": dist_a})
        knn_df = DataFrame([table])
        if sort_knn_df_by_query_id:
            knn_df = knn_df.sort(qname)
        knn_df = knn_df.repartition(query_df.getNumPartitions())
        return self._item_df_withid, query_df_withid, knn_df

    def _nearest_neighbors_join(self, query_df: Any, distCol: str = "distCol") -> DataFrame:
        from .parallel.spark import is_spark_dataframe

        if is_spark_dataframe(self._item_df_withid) or is_spark_dataframe(query_df):
            return self._spark_join(query_df, distCol)
        id_col = self._getIdColOrDefault()
        item_df, query_df_withid, knn_df = self.kneighbors(query_df, sort_knn_df_by_query_id=False)
        knn = knn_df._concat()
        qids = knn.column("query_%s" % id_col).to_numpy()
        lens = np.asarray(pa.compute.list_value_length(knn.column("indices").combine_chunks()).to_numpy(
            zero_copy_only=False), dtype=np.int64)
        inds = pa.compute.list_flatten(knn.column("indices").combine_chunks()).to_numpy(zero_copy_only=False)
        dists = pa.compute.list_flatten(knn.column("distances").combine_chunks()).to_numpy(zero_copy_only=False)
        q_rep = np.repeat(qids, lens)
        items_t = item_df._concat()
        query_t = query_df_withid._concat()
        item_pos = _positions(items_t.column(id_col).to_numpy(), inds)
        query_pos = _positions(query_t.column(id_col).to_numpy(), q_rep)
        keep_id = self.isSet("idCol")
        it = items_t if keep_id else items_t.drop([id_col])
        qt = query_t if keep_id else query_t.drop([id_col])
        item_struct = pa.StructArray.from_arrays([c.combine_chunks().take(pa.array(item_pos)) for c in it.columns],
                                                 fields=list(it.schema))
        query_struct = pa.StructArray.from_arrays([c.combine_chunks().take(pa.array(query_pos)) for c in qt.columns],
                                                  fields=list(qt.schema))
        out = pa.table({"item_df": item_struct, "query_df": query_struct, distCol: pa.array(dists.astype(np.float32))})
        return DataFrame([out])


def _positions(keys: np.ndarray, wanted: np.ndarray) -> np.ndarray:
    order = np.argsort(keys, kind="stable")
    pos = np.searchsorted(keys[order], wanted)
    pos = np.clip(pos, 0, max(len(keys) - 1, 0))
    return order[pos].astype(np.int64)


# ------------------------------------------------------------------------------------------
# exact
# ------------------------------------------------------------------------------------------
class NearestNeighbors(NearestNeighborsClass, _NoPersistence, _NNParams):
    """Exact k-nearest-neighbour search (brute force on MFMA, distributed over ranks).

    >>> from spark_rapids_ml_nai_amd.knn import NearestNeighbors
    >>> items = DataFrame.createDataFrame([(0, [1.0, 1.0]), (1, [2.0, 2.0]), (2, [3.0, 3.0])], ["id", "features"])
    >>> model = NearestNeighbors(k=2, inputCol="features", idCol="id").fit(items)
    >>> _, _, knn_df = model.kneighbors(items)
    """

    @keyword_only
    def __init__(self, *, k: Optional[int] = None, inputCol: Optional[Union[str, List[str]]] = None,
                 idCol: Optional[str] = None, num_workers: Optional[int] = None,
                 verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._initialize_backend_params()
        self._set_params(**self._input_kwargs)

    def setK(self, value: int) -> "NearestNeighbors":
        return self._set_params(k=value)

    def fit(self, dataset: Any, params: Any = None) -> "NearestNeighborsModel":
        est = self.copy(params) if isinstance(params, dict) else self
        return est._fit(dataset)

    def _fit(self, dataset: Any) -> "NearestNeighborsModel":
        from .parallel.spark import is_spark_dataframe

        df = dataset if is_spark_dataframe(dataset) else as_dataframe(dataset)[0]
        item_df_withid = self._ensureIdCol(df)
        model = NearestNeighborsModel(item_df_withid)
        model._num_workers = self._num_workers
        model._float32_inputs = True
        self._copyValues(model)
        self._copy_backend_params(model)
        return model


class NearestNeighborsModel(NearestNeighborsClass, _NNModelBase):
    def __init__(self, item_df_withid: DataFrame) -> None:
        super().__init__()
        self._initialize_backend_params()
        self._item_df_withid = item_df_withid

    def exactNearestNeighborsJoin(self, query_df: Any, distCol: str = "distCol") -> DataFrame:
        """``(item_df struct, query_df struct, distCol)`` for every (query, neighbour) pair."""
        return self._nearest_neighbors_join(query_df, distCol)


# ------------------------------------------------------------------------------------------
# approximate (IVF-Flat)
# ------------------------------------------------------------------------------------------
class ApproximateNearestNeighborsClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {"k": "n_neighbors", "algorithm": "algorithm", "metric": "metric", "algoParams": "algo_params"}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {"n_neighbors": 5, "verbose": False, "algorithm": "ivfflat", "metric": "euclidean", "algo_params": None}


class _ANNParams(_NNParams):
    algorithm = Param(Params._dummy(), "algorithm", "The algorithm to use for approximate nearest neighbors search.",
                      typeConverter=TypeConverters.toString)
    algoParams = Param(Params._dummy(), "algoParams", "The parameters to use to set up a neighbor algorithm.",
                       typeConverter=TypeConverters.identity)
    metric = Param(Params._dummy(), "metric", "The distance metric to use.", typeConverter=TypeConverters.toString)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(algorithm="ivfflat", algoParams=None, metric="euclidean")

    def setAlgorithm(self, value: str) -> Any:
        return self._set_params(algorithm=value)

    def getAlgorithm(self) -> str:
        return self.getOrDefault(self.algorithm)

    def setAlgoParams(self, value: Dict[str, Any]) -> Any:
        return self._set_params(algoParams=value)

    def getAlgoParams(self) -> Dict[str, Any]:
        return self.getOrDefault(self.algoParams)

    def setMetric(self, value: str) -> Any:
        return self._set_params(metric=value)

    def getMetric(self) -> str:
        return self.getOrDefault(self.metric)


_SUPPORTED_ALGOS = ("ivfflat", "brute")
_SUPPORTED_METRICS = ("euclidean", "sqeuclidean", "l2", "inner_product")


class ApproximateNearestNeighbors(ApproximateNearestNeighborsClass, _NoPersistence, _ANNParams):
    """IVF-Flat approximate kNN (``algoParams={"nlist": .., "nprobe": ..}``), one index per item partition.

    >>> from spark_rapids_ml_nai_amd.knn import ApproximateNearestNeighbors
    >>> ann = ApproximateNearestNeighbors(k=2, algoParams={"nlist": 2, "nprobe": 2}, inputCol="features")
    """

    @keyword_only
    def __init__(self, *, k: Optional[int] = None, algorithm: str = "ivfflat", metric: str = "euclidean",
                 algoParams: Optional[Dict[str, Any]] = None, inputCol: Optional[Union[str, List[str]]] = None,
                 idCol: Optional[str] = None, num_workers: Optional[int] = None,
                 verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._initialize_backend_params()
        self._set_params(**self._input_kwargs)

    def _validate(self) -> None:
        if self.getAlgorithm() not in _SUPPORTED_ALGOS:
            raise ValueError("algorithm %r is not supported; expected one of %s" % (self.getAlgorithm(), _SUPPORTED_ALGOS))
        if self.getMetric() not in _SUPPORTED_METRICS:
            raise ValueError("metric %r is not supported; expected one of %s" % (self.getMetric(), _SUPPORTED_METRICS))

    def fit(self, dataset: Any, params: Any = None) -> "ApproximateNearestNeighborsModel":
        est = self.copy(params) if isinstance(params, dict) else self
        return est._fit(dataset)

    def _fit(self, dataset: Any) -> "ApproximateNearestNeighborsModel":
        self._validate()
        from .parallel.spark import is_spark_dataframe

        df = dataset if is_spark_dataframe(dataset) else as_dataframe(dataset)[0]
        item_df_withid = self._ensureIdCol(df).coalesce(max(1, self.num_workers))
        model = ApproximateNearestNeighborsModel(item_df_withid)
        model._num_workers = self._num_workers
        model._float32_inputs = True
        self._copyValues(model)
        self._copy_backend_params(model)
        return model


class ApproximateNearestNeighborsModel(ApproximateNearestNeighborsClass, _NNModelBase, _ANNParams):
    def __init__(self, item_df_withid: DataFrame) -> None:
        super().__init__()
        self._initialize_backend_params()
        self._item_df_withid = item_df_withid
        self._index_cache: Dict[str, Any] = {}

    def _metric(self) -> str:
        return self.getMetric()

    def _worker(self) -> Any:
        return _ivf_worker

    def _ivf_args(self) -> Optional[Tuple[Any, ...]]:
        ap = dict(self.getAlgoParams() or {})
        return (self.getAlgorithm(), ap.get("nlist", ap.get("n_lists")), ap.get("nprobe", ap.get("n_probes")),
                int(ap.get("seed", 1)))

    def _payload_extra(self) -> Tuple[Any, ...]:
        ap = dict(self.getAlgoParams() or {})
        nlist = ap.get("nlist", ap.get("n_lists"))
        nprobe = ap.get("nprobe", ap.get("n_probes"))
        # the built index is reusable across kneighbors calls only when the search runs in-process
        # (one worker, or one SPMD rank over its own item shard)
        cache = self._index_cache if (spmd_active() or max(1, self.num_workers) == 1) else None
        return (self.getAlgorithm(), nlist, nprobe, int(ap.get("seed", 1)), cache)

    def kneighbors(self, query_df: Any, sort_knn_df_by_query_id: bool = True) -> Tuple[DataFrame, DataFrame, DataFrame]:
        """Approximate k nearest items of every query (see ``NearestNeighborsModel.kneighbors``)."""
        return super().kneighbors(query_df, sort_knn_df_by_query_id)

    def approxSimilarityJoin(self, query_df: Any, distCol: str = "distCol") -> DataFrame:
        """``(item_df struct, query_df struct, distCol)`` for every (query, approximate neighbour)."""
        return self._nearest_neighbors_join(query_df, distCol)
