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

from .core.base import FitInput, _Estimator, _ModelWithPredictionCol, _Model
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
    def __init__(self, cluster_centers_: List[List[float]], n_cols: int, dtype: str, n_iter: int = 0) -> None:
        super().__init__(cluster_centers_=cluster_centers_, n_cols=n_cols, dtype=dtype, n_iter=n_iter)
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
            from .models.kmeans import kmeans_predict

            Xd = to_device(X, ctx.device, torch.float32)
            return {pred_col: kmeans_predict(Xd, Cd).cpu().numpy().astype(np.int32)}

        return construct, predict
