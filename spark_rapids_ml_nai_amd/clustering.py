"""``clustering.KMeans`` / ``KMeansModel`` (reference ``clustering.py:67-499``) and
``clustering.DBSCAN`` / ``DBSCANModel`` (``clustering.py:502-1100``).

KMeans param mapping: ``initMode -> init`` ("k-means||" -> scalable-k-means++), ``k ->
n_clusters``, ``maxIter -> max_iter``, ``seed -> random_state``, ``tol -> tol`` (0 mapped to
float32 tiny with a warning), ``distanceMeasure``/``weightCol`` unsupported, ``initSteps``,
``solver``, ``maxBlockSizeInMB`` ignored. Default seed: a stable 31-bit hash of the class name.
"""
from __future__ import annotations

import warnings
import zlib
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .core.base import FitInput, _Estimator, _ModelWithPredictionCol
from .core.dataframe import DataFrame
from .core.linalg import as_dense_array
from .core.params import (
    HasDistanceMeasure,
    HasFeaturesCol,
    HasFeaturesCols,
    HasIDCol,
    HasMaxBlockSizeInMB,
    HasMaxIter,
    HasPredictionCol,
    HasSeed,
    HasSolver,
    HasTol,
    HasWeightCol,
    Param,
    Params,
    TypeConverters,
    _BackendClass,
    _BackendParams,
    keyword_only,
)
from .parallel.context import WorkerContext
from .core.params import _FeaturesColMixin


def _stable_seed(name: str) -> int:
    return zlib.crc32(name.encode()) & 0x7FFFFFFF


class KMeansClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {
            "distanceMeasure": None,
            "initMode": "init",
            "k": "n_clusters",
            "initSteps": "",
            "maxIter": "max_iter",
            "seed": "random_state",
            "tol": "tol",
            "weightCol": None,
            "solver": "",
            "maxBlockSizeInMB": "",
        }

    @classmethod
    def _param_value_mapping(cls) -> Dict[str, Callable[[Any], Any]]:
        def tol_map(x: float) -> float:
            if x == 0.0:
                warnings.warn("tol=0 is mapped to the smallest positive float32 (numpy.finfo('float32').tiny).")
                return float(np.finfo("float32").tiny)
            return x

        def init_map(x: str) -> Optional[str]:
            return {"k-means||": "scalable-k-means++", "random": "random",
                    "scalable-k-means++": "scalable-k-means++", "k-means++": "k-means++"}.get(x)

        return {"tol": tol_map, "init": init_map}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {
            "n_clusters": 8, "max_iter": 300, "tol": 0.0001, "verbose": False, "random_state": 1,
            "init": "scalable-k-means++", "n_init": 1, "oversampling_factor": 2.0, "max_samples_per_batch": 32768,
        }


class _KMeansParams(_BackendParams, HasFeaturesCol, HasFeaturesCols, HasPredictionCol, HasMaxIter, HasTol,
                    HasSeed, HasDistanceMeasure, HasWeightCol, HasSolver, HasMaxBlockSizeInMB, _FeaturesColMixin):
    k = Param(Params._dummy(), "k", "The number of clusters to create. Must be > 1.", typeConverter=TypeConverters.toInt)
    initMode = Param(Params._dummy(), "initMode", 'The initialization algorithm: "random" or "k-means||".',
                     typeConverter=TypeConverters.toString)
    initSteps = Param(Params._dummy(), "initSteps", "The number of steps for k-means|| initialization mode.",
                      typeConverter=TypeConverters.toInt)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(k=2, initMode="k-means||", initSteps=2, tol=1e-4, maxIter=20, distanceMeasure="euclidean",
                         solver="auto", maxBlockSizeInMB=0.0, featuresCol="features", predictionCol="prediction",
                         seed=_stable_seed(type(self).__name__))

    def getK(self) -> int:
        return self.getOrDefault("k")

    def getInitMode(self) -> str:
        return self.getOrDefault("initMode")

    def getInitSteps(self) -> int:
        return self.getOrDefault("initSteps")


class KMeans(KMeansClass, _Estimator, _KMeansParams):
    """Distributed KMeans (fused MFMA distance+argmin kernel, RCCL centroid all-reduce)."""

    @keyword_only
    def __init__(self, *, featuresCol: Union[str, List[str]] = "features", predictionCol: str = "prediction",
                 k: int = 2, initMode: str = "k-means||", tol: float = 0.0001, maxIter: int = 20,
                 seed: Optional[int] = None, num_workers: Optional[int] = None, verbose: Union[int, bool] = False,
                 **kwargs: Any) -> None:
        super().__init__()
        self._set_params(**self._input_kwargs)

    def setK(self, value: int) -> "KMeans":
        return self._set_params(k=value)

    def setMaxIter(self, value: int) -> "KMeans":
        return self._set_params(maxIter=value)

    def setSeed(self, value: int) -> "KMeans":
        if value > 0x07FFFFFFF:
            raise ValueError("seed value must be a 32-bit integer.")
        return self._set_params(seed=value)

    def setTol(self, value: float) -> "KMeans":
        return self._set_params(tol=value)

    def setInitMode(self, value: str) -> "KMeans":
        return self._set_params(initMode=value)

    def setWeightCol(self, value: str) -> "KMeans":
        raise ValueError("'weightCol' is not supported.")

    def _get_fit_func(self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        init_steps = self.getOrDefault("initSteps")

        def _fit(inp: FitInput, ctx: WorkerContext, params: Dict[str, Any]) -> Dict[str, Any]:
            from .models.kmeans import kmeans_fit

            p = params["cuml_init"]
            return kmeans_fit(inp.X, inp.desc, ctx, int(p["n_clusters"]), int(p["max_iter"]), float(p["tol"]),
                              int(p["random_state"]), p["init"], float(p.get("oversampling_factor", 2.0)), init_steps)

        return _fit

    def _create_model(self, result: Dict[str, Any]) -> "KMeansModel":
        return KMeansModel._from_row(result)


class KMeansModel(KMeansClass, _ModelWithPredictionCol, _KMeansParams):
    def __init__(self, cluster_centers_: List[List[float]], n_cols: int, dtype: str, n_iter: int = 0,
                 refined_frac: Optional[float] = None, delta_iters: Optional[int] = None,
                 phase_s: Optional[List[float]] = None) -> None:
        super().__init__(cluster_centers_=cluster_centers_, n_cols=n_cols, dtype=dtype, n_iter=n_iter,
                         refined_frac=refined_frac, delta_iters=delta_iters, phase_s=phase_s)
        self.cluster_centers_ = cluster_centers_
        self.n_cols = n_cols
        self.dtype = dtype

    def clusterCenters(self) -> List[np.ndarray]:
        return [np.array(x) for x in self.cluster_centers_]

    @property
    def hasSummary(self) -> bool:
        return False

    @property
    def summary(self) -> Any:
        raise RuntimeError("No training summary available for this KMeansModel")

    def predict(self, value: Any) -> int:
        x = as_dense_array(value)
        C = np.asarray(self.cluster_centers_, dtype=np.float64)
        return int(np.argmin(((C - x) ** 2).sum(1)))

    def cpu(self) -> Any:
        from .utils.spark_compat import to_spark_kmeans_model

        return to_spark_kmeans_model(self)

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        C = np.asarray(self.cluster_centers_, dtype=np.float32)
        pred_col = self.getPredictionCol()

        def construct(ctx: WorkerContext) -> torch.Tensor:
            return torch.from_numpy(C).to(ctx.device)

        def predict(Cd: torch.Tensor, X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            from .core.base import to_device
            from .models.kmeans import kmeans_predict, kmeans_predict_streamed, predict_streams

            if ctx.device.type == "cuda" and predict_streams(X, Cd.shape[0]):  # H2D under the search
                return {pred_col: kmeans_predict_streamed(X, Cd, ctx.device).cpu().numpy().astype(np.int32)}
            Xd = to_device(X, ctx.device, torch.float32)
            return {pred_col: kmeans_predict(Xd, Cd).cpu().numpy().astype(np.int32)}

        return construct, predict


# ------------------------------------------------------------------------------------------
# DBSCAN
# ------------------------------------------------------------------------------------------
class DBSCANClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        # Spark params carry the backend names (reference mapping is empty for the same reason)
        return {k: k for k in ("eps", "min_samples", "metric", "algorithm", "max_mbytes_per_batch",
                               "calc_core_sample_indices")}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {
            "eps": 0.5,
            "min_samples": 5,
            "metric": "euclidean",
            "algorithm": "brute",
            "verbose": False,
            "max_mbytes_per_batch": None,
            "calc_core_sample_indices": False,
        }


class _DBSCANParams(_FeaturesColMixin, _BackendParams, HasFeaturesCol, HasFeaturesCols, HasPredictionCol, HasIDCol):
    eps = Param(Params._dummy(), "eps",
                "The maximum distance between 2 points such they reside in the same neighborhood.",
                typeConverter=TypeConverters.toFloat)
    min_samples = Param(Params._dummy(), "min_samples",
                        "The number of samples in a neighborhood such that this group can be considered as an "
                        "important core point (including the point itself).", typeConverter=TypeConverters.toInt)
    metric = Param(Params._dummy(), "metric", "The metric to use when calculating distances between points "
                   "('euclidean' or 'cosine'; 'precomputed' is not supported).", typeConverter=TypeConverters.toString)
    algorithm = Param(Params._dummy(), "algorithm", "The algorithm to be used by for nearest neighbor computations "
                      "('brute' or 'rbc'; both run the fused brute-force tile sweep).",
                      typeConverter=TypeConverters.toString)
    max_mbytes_per_batch = Param(Params._dummy(), "max_mbytes_per_batch",
                                 "Accepted for compatibility; the tiled kernels never materialise the N x N "
                                 "distance matrix, so no batching is needed.", typeConverter=TypeConverters.toInt)
    calc_core_sample_indices = Param(Params._dummy(), "calc_core_sample_indices",
                                     "Indicates whether the indices of the core samples should be calculated.",
                                     typeConverter=TypeConverters.toBoolean)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(eps=0.5, min_samples=5, metric="euclidean", algorithm="brute", max_mbytes_per_batch=None,
                         calc_core_sample_indices=True, idCol="unique_id", predictionCol="prediction",
                         featuresCol="features")

    def setEps(self, value: float) -> Any:
        return self._set_params(eps=value)

    def getEps(self) -> float:
        return self.getOrDefault(self.eps)

    def setMinSamples(self, value: int) -> Any:
        return self._set_params(min_samples=value)

    def getMinSamples(self) -> int:
        return self.getOrDefault(self.min_samples)

    def setMetric(self, value: str) -> Any:
        return self._set_params(metric=value)

    def getMetric(self) -> str:
        return self.getOrDefault(self.metric)

    def setAlgorithm(self, value: str) -> Any:
        return self._set_params(algorithm=value)

    def getAlgorithm(self) -> str:
        return self.getOrDefault(self.algorithm)

    def setMaxMbytesPerBatch(self, value: Optional[int]) -> Any:
        return self._set_params(max_mbytes_per_batch=value)

    def getMaxMbytesPerBatch(self) -> Optional[int]:
        return self.getOrDefault(self.max_mbytes_per_batch)

    def setCalcCoreSampleIndices(self, value: bool) -> Any:
        return self._set_params(calc_core_sample_indices=value)

    def getCalcCoreSampleIndices(self) -> bool:
        return self.getOrDefault(self.calc_core_sample_indices)

    def setIdCol(self, value: str) -> Any:
        return self._set_params(idCol=value)


def _dbscan_worker(ctx: WorkerContext, payload: Tuple[Any, ...]) -> Tuple[np.ndarray, np.ndarray]:
    from .core.base import to_device
    from .models.dbscan import dbscan_fit_predict

    X, eps, min_samples, metric = payload
    if ctx.world_size > 1:  # an empty shard learns the feature count from the other ranks
        nt = torch.tensor([float(X.shape[1] if X.ndim == 2 else 0)], dtype=torch.float64, device=ctx.device)
        ctx.comm.allreduce(nt, op="max")
        X = np.asarray(X, np.float32).reshape(-1, int(nt.item())) if X.size == 0 else X
    Xd = to_device(X, ctx.device, torch.float32)
    return dbscan_fit_predict(Xd, ctx, eps, min_samples, metric)


def _spark_dbscan_task(ctx: WorkerContext, table: Any, extra: Tuple[Any, ...]) -> Any:
    """One rank of the Spark DBSCAN barrier job: this rank's rows are clustered together with every
    other rank's (device-gathered over RCCL, ``models/dbscan.py``) and it emits (id, label) for its
    own rows. Replaces the reference's driver ``toPandas`` + <= 8 GiB broadcasts of the whole
    dataset (``clustering.py:1013-1069``)."""
    import pyarrow as pa

    from .core.base import _dense_from_df
    from .core.dataframe import DataFrame as _DF

    col, cols, id_col, pred_col, eps, min_samples, metric = extra
    if table is not None and table.num_rows:
        part = _DF([table])
        X = _dense_from_df(part, col, cols, np.float32)
        ids = np.asarray(part.to_numpy(id_col)).astype(np.int64)
    else:  # an empty rank still joins every collective (the worker agrees on n)
        X, ids = np.zeros((0, 0), np.float32), np.zeros(0, np.int64)
    labels, _core = _dbscan_worker(ctx, (X, eps, min_samples, metric))
    yield pa.RecordBatch.from_arrays([pa.array(ids), pa.array(np.asarray(labels).astype(np.int32))],
                                     names=[id_col, pred_col])


class DBSCAN(DBSCANClass, _Estimator, _DBSCANParams):
    """Density-based clustering. Like the reference, ``fit`` does no work: it returns a
    ``DBSCANModel`` whose ``transform`` clusters the dataset it is given (``clustering.py:820-833``).

    >>> from spark_rapids_ml_nai_amd.clustering import DBSCAN
    >>> df = DataFrame.createDataFrame([([0.0, 0.0],), ([1.0, 1.0],), ([9.0, 8.0],), ([8.0, 9.0],)], ["features"])
    >>> model = DBSCAN(eps=2.0, min_samples=2).setFeaturesCol("features").fit(df)
    >>> [r.prediction for r in model.transform(df).collect()]
    [0, 0, 1, 1]
    """

    @keyword_only
    def __init__(self, *, featuresCol: Union[str, List[str]] = "features", predictionCol: str = "prediction",
                 eps: float = 0.5, min_samples: int = 5, metric: str = "euclidean", algorithm: str = "brute",
                 max_mbytes_per_batch: Optional[int] = None, calc_core_sample_indices: bool = True,
                 idCol: Optional[str] = None, num_workers: Optional[int] = None,
                 verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._set_params(**self._input_kwargs)

    def _get_fit_func(self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        raise NotImplementedError("DBSCAN does not fit and generate model")

    def _create_model(self, result: Dict[str, Any]) -> "DBSCANModel":
        raise NotImplementedError("DBSCAN does not support model creation from Row")

    def _fit(self, dataset: Any) -> "DBSCANModel":
        if self.getMetric() == "precomputed":
            raise ValueError("The 'precomputed' metric of sklearn/cuML is not supported; use those libraries instead")
        if self.getMetric() not in ("euclidean", "cosine", "l2"):
            raise ValueError("Unsupported metric %r" % self.getMetric())
        model = DBSCANModel(n_cols=0, dtype="", verbose=self._backend_params.get("verbose", False))
        model._num_workers = self._num_workers
        model._float32_inputs = self._float32_inputs
        self._copyValues(model)
        self._copy_backend_params(model)
        return model


class DBSCANModel(DBSCANClass, _ModelWithPredictionCol, _DBSCANParams):
    def __init__(self, n_cols: int = 0, dtype: str = "", verbose: Union[int, bool] = False) -> None:
        super().__init__(n_cols=n_cols, dtype=dtype, verbose=verbose)
        self.n_cols = n_cols
        self.dtype = dtype
        self.verbose = verbose
        self.core_sample_indices_: Optional[np.ndarray] = None

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        raise NotImplementedError("DBSCANModel clusters the whole dataset in transform()")

    def _transform(self, dataset: Any) -> Any:
        from .parallel.spark import is_spark_dataframe

        if is_spark_dataframe(dataset):
            return self._spark_transform(dataset)
        return super()._transform(dataset)

    def _spark_transform(self, sdf: Any) -> Any:
        """Spark DataFrame: an id column is ensured, ONE barrier job labels every row and the labels
        are joined back on the id (reference ``clustering.py:1013-1091``; output keeps the id)."""
        from pyspark.sql.types import IntegerType, LongType, StructField, StructType  # type: ignore

        from .parallel.spark import spark_barrier_job

        df_withid = self._ensureIdCol(sdf)
        id_col = self.getIdCol()
        fc = self.getFeaturesCol()
        col, cols = (fc, None) if isinstance(fc, str) else (None, list(fc))
        sel = ([col] if col else list(cols)) + [id_col]
        job_in = df_withid.select(*sel).repartition(max(1, self.num_workers))
        pred = self.getPredictionCol()
        schema = StructType([StructField(id_col, LongType()), StructField(pred, IntegerType())])
        labels = spark_barrier_job(job_in, _spark_dbscan_task, (col, cols, id_col, pred, self.getEps(),
                                                                self.getMinSamples(), self.getMetric()), schema)
        return df_withid.join(labels, on=id_col)

    def _features_all(self, df: DataFrame) -> np.ndarray:
        from .core.base import _dense_from_df

        fc = self.getFeaturesCol()
        col, cols = (fc, None) if isinstance(fc, str) else (None, list(fc))
        return _dense_from_df(df, col, cols, np.float32)

    def _transform_df(self, df: DataFrame) -> DataFrame:
        from .core.base import run_worker_job
        from .parallel.context import spmd_active

        if spmd_active():
            # torchrun: the frame is this rank's whole shard; the rank labels its own rows (global
            # cluster numbering, every rank's rows clustered together) and core_sample_indices_
            # index into this rank's frame
            parts = df.partitions
            X = self._features_all(df) if df.count() else np.zeros((0, 0), np.float32)
            payloads = [(X, self.getEps(), self.getMinSamples(), self.getMetric())]
        else:
            nw = max(1, self.num_workers)
            parts = df.repartition(nw).partitions if df.getNumPartitions() != nw else df.partitions
            payloads = [(self._features_all(DataFrame([p])), self.getEps(), self.getMinSamples(), self.getMetric())
                        for p in parts]
        res = run_worker_job(_dbscan_worker, payloads)
        labels = np.concatenate([r[0] for r in res]).astype(np.int32)
        core = np.concatenate([r[1] for r in res])
        if self.getCalcCoreSampleIndices():
            self.core_sample_indices_ = np.nonzero(core)[0]
        out = DataFrame(parts) if len(parts) != df.getNumPartitions() else df
        return out.withColumn(self.getPredictionCol(), labels)
