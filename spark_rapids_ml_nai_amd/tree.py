"""Shared RandomForest estimator/model machinery (reference ``tree.py:80-636``).

Param mapping (reference ``tree.py:82-124``): ``maxBins -> n_bins``, ``maxDepth -> max_depth``,
``numTrees -> n_estimators``, ``impurity -> split_criterion``, ``featureSubsetStrategy ->
max_features`` (onethird -> 1/3, all -> 1.0, sqrt, log2, auto, numeric), ``bootstrap``,
``seed -> random_state``, ``minInstancesPerNode -> min_samples_leaf``. Unlike the reference
(which ignores them), ``minInfoGain`` and ``subsamplingRate`` are honoured
(``min_impurity_decrease`` / bootstrap rate ``max_samples``). Trees are stored in a portable JSON
form (flat breadth-first node arrays) instead of a pickled treelite handle.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, List, Optional, Union

import numpy as np
import torch

from .core.base import FitInput, _EstimatorSupervised, _ModelWithPredictionCol
from .core.dataframe import DataFrame
from .core.linalg import Vectors, as_dense_array
from .core.params import (
    HasCheckpointInterval,
    HasFeaturesCol,
    HasFeaturesCols,
    HasLabelCol,
    HasLeafCol,
    HasPredictionCol,
    HasSeed,
    HasWeightCol,
    Param,
    Params,
    TypeConverters,
    _BackendClass,
    _BackendParams,
)
from .parallel.context import WorkerContext
from .core.params import _FeaturesColMixin


def _str_or_numerical(v: str) -> Union[str, int, float]:
    try:
        return int(v)
    except (ValueError, TypeError):
        try:
            return float(v)
        except (ValueError, TypeError):
            return v


class _RandomForestClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {
            "maxBins": "n_bins",
            "maxDepth": "max_depth",
            "numTrees": "n_estimators",
            "impurity": "split_criterion",
            "featureSubsetStrategy": "max_features",
            "bootstrap": "bootstrap",
            "seed": "random_state",
            "minInstancesPerNode": "min_samples_leaf",
            "minInfoGain": "min_impurity_decrease",
            "maxMemoryInMB": "",
            "cacheNodeIds": "",
            "checkpointInterval": "",
            "subsamplingRate": "max_samples",
            "minWeightFractionPerNode": "",
            "weightCol": None,
            "leafCol": None,
        }

    @classmethod
    def _param_value_mapping(cls) -> Dict[str, Callable[[Any], Any]]:
        def tree_mapping(feature_subset: Any) -> Any:
            v = _str_or_numerical(feature_subset)
            if isinstance(v, (int, float)):
                return v
            return {"onethird": 1 / 3.0, "all": 1.0, "auto": "auto", "sqrt": "sqrt", "log2": "log2"}.get(v)

        return {"max_features": tree_mapping}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {
            "n_streams": 1, "n_estimators": 100, "max_depth": 16, "max_features": "auto", "n_bins": 128,
            "bootstrap": True, "verbose": False, "min_samples_leaf": 1, "min_samples_split": 2, "max_samples": 1.0,
            "max_leaves": -1, "min_impurity_decrease": 0.0, "random_state": None, "max_batch_size": 4096,
            "split_mode": "ensemble",
        }


class _RandomForestParams(_BackendParams, HasFeaturesCol, HasFeaturesCols, HasLabelCol, HasPredictionCol, HasSeed,
                          HasWeightCol, HasCheckpointInterval, HasLeafCol, _FeaturesColMixin):
    maxDepth = Param(Params._dummy(), "maxDepth", "Maximum depth of the tree (>= 0).", typeConverter=TypeConverters.toInt)
    maxBins = Param(Params._dummy(), "maxBins", "Max number of bins for discretizing continuous features (>= 2).",
                    typeConverter=TypeConverters.toInt)
    minInstancesPerNode = Param(Params._dummy(), "minInstancesPerNode",
                                "Minimum number of instances each child must have after split.",
                                typeConverter=TypeConverters.toInt)
    minWeightFractionPerNode = Param(Params._dummy(), "minWeightFractionPerNode",
                                     "Minimum fraction of the weighted sample count per child.",
                                     typeConverter=TypeConverters.toFloat)
    minInfoGain = Param(Params._dummy(), "minInfoGain", "Minimum information gain for a split.",
                        typeConverter=TypeConverters.toFloat)
    maxMemoryInMB = Param(Params._dummy(), "maxMemoryInMB", "Maximum memory in MB for histogram aggregation.",
                          typeConverter=TypeConverters.toInt)
    cacheNodeIds = Param(Params._dummy(), "cacheNodeIds", "Cache node IDs per instance.",
                         typeConverter=TypeConverters.toBoolean)
    impurity = Param(Params._dummy(), "impurity", "Criterion used for information gain calculation.",
                     typeConverter=TypeConverters.toString)
    numTrees = Param(Params._dummy(), "numTrees", "Number of trees to train (>= 1).", typeConverter=TypeConverters.toInt)
    subsamplingRate = Param(Params._dummy(), "subsamplingRate", "Fraction of the training data used per tree.",
                            typeConverter=TypeConverters.toFloat)
    featureSubsetStrategy = Param(Params._dummy(), "featureSubsetStrategy",
                                  "The number of features to consider for splits at each tree node.",
                                  typeConverter=TypeConverters.toString)
    bootstrap = Param(Params._dummy(), "bootstrap", "Whether bootstrap samples are used when building trees.",
                      typeConverter=TypeConverters.toBoolean)

    def __init__(self) -> None:
        super().__init__()
        self._setDefault(maxDepth=5, maxBins=32, minInstancesPerNode=1, minWeightFractionPerNode=0.0, minInfoGain=0.0,
                         maxMemoryInMB=256, cacheNodeIds=False, checkpointInterval=10, numTrees=20,
                         subsamplingRate=1.0, featureSubsetStrategy="auto", bootstrap=True, leafCol="",
                         featuresCol="features", labelCol="label", predictionCol="prediction",
                         seed=_stable_seed(type(self).__name__))

    def getMaxDepth(self) -> int:
        return self.getOrDefault("maxDepth")

    def getMaxBins(self) -> int:
        return self.getOrDefault("maxBins")

    def getNumTrees(self) -> int:
        return self.getOrDefault("numTrees")

    def getImpurity(self) -> str:
        return self.getOrDefault("impurity")

    def getFeatureSubsetStrategy(self) -> str:
        return self.getOrDefault("featureSubsetStrategy")

    def getMinInstancesPerNode(self) -> int:
        return self.getOrDefault("minInstancesPerNode")

    def getBootstrap(self) -> bool:
        return self.getOrDefault("bootstrap")

    def getSubsamplingRate(self) -> float:
        return self.getOrDefault("subsamplingRate")

    def getMinInfoGain(self) -> float:
        return self.getOrDefault("minInfoGain")

    def getMinWeightFractionPerNode(self) -> float:
        return self.getOrDefault("minWeightFractionPerNode")

    def getMaxMemoryInMB(self) -> int:
        return self.getOrDefault("maxMemoryInMB")

    def getCacheNodeIds(self) -> bool:
        return self.getOrDefault("cacheNodeIds")

    def setLeafCol(self, value: str) -> Any:
        """Records the Spark Param only: like the reference (tests/test_random_forest.py:573-628),
        leaf-index output is not produced by transform (no backend mapping)."""
        self._set(leafCol=value)
        return self


def _stable_seed(name: str) -> int:
    import zlib

    return zlib.crc32(name.encode()) & 0x7FFFFFFF


class _RandomForestEstimator(_RandomForestClass, _EstimatorSupervised, _RandomForestParams):
    _is_classification = True

    def setBootstrap(self, value: bool) -> Any:
        return self._set_params(bootstrap=value)

    def setFeatureSubsetStrategy(self, value: str) -> Any:
        return self._set_params(featureSubsetStrategy=value)

    def setImpurity(self, value: str) -> Any:
        return self._set_params(impurity=value)

    def setMaxBins(self, value: int) -> Any:
        return self._set_params(maxBins=value)

    def setMaxDepth(self, value: int) -> Any:
        return self._set_params(maxDepth=value)

    def setMinInstancesPerNode(self, value: int) -> Any:
        return self._set_params(minInstancesPerNode=value)

    def setNumTrees(self, value: int) -> Any:
        return self._set_params(numTrees=value)

    def setSubsamplingRate(self, value: float) -> Any:
        return self._set_params(subsamplingRate=value)

    def setMinInfoGain(self, value: float) -> Any:
        return self._set_params(minInfoGain=value)

    def setSeed(self, value: int) -> Any:
        if value > 0x07FFFFFFF:
            raise ValueError("seed value must be a 32-bit integer.")
        return self._set_params(seed=value)

    def setWeightCol(self, value: str) -> Any:
        raise ValueError("'weightCol' is not supported.")

    def _enable_fit_multiple_in_single_pass(self) -> bool:
        return True

    def _require_comm(self) -> bool:
        return self._backend_params.get("split_mode", "ensemble") == "data_parallel"

    def _label_dtype(self, float32: bool) -> Any:
        return np.float32

    def _get_fit_func(self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        classification = self._is_classification
        nw = self.num_workers

        def _fit(inp: FitInput, ctx: WorkerContext, params: Dict[str, Any]) -> Any:
            from .models.forest import feature_subset_size, fit_forest, quantize_features

            X, y = inp.X, inp.y
            n = inp.desc.n
            num_classes = 0
            if classification:
                if torch.any(y < 0) or torch.any(y != torch.floor(y)):
                    raise RuntimeError("Labels MUST be non-negative integers for classification")
                mx = torch.tensor([float(y.max().item())], dtype=torch.float64, device=y.device)
                ctx.comm.allreduce(mx, op="max")
                num_classes = max(2, int(mx.item()) + 1)
                if num_classes > 32:
                    raise ValueError("RandomForestClassifier supports at most 32 classes")
            maps = params["fit_multiple_params"] or [{}]
            outs = []
            # hyper-parameter batching: param maps with the same (maxBins, seed) share one quantile
            # binning of the shard (bin edges + uint8 matrix), the per-fit pass over X
            binned: Dict[Any, Any] = {}
            streamed = inp.stream  # streamed ingest: the first binning consumes the row chunks as they land
            for mp in maps:
                p = dict(params["cuml_init"], **mp)
                mode = p.get("split_mode", "ensemble")
                data_parallel = mode == "data_parallel"  # world 1: the same path, its all-reduces are no-ops
                n_est = int(p["n_estimators"])
                if data_parallel:
                    n_local = n_est
                else:
                    share = n_est // ctx.world_size + (1 if ctx.rank < n_est % ctx.world_size else 0)
                    n_local = share
                mf = p["max_features"]
                p["_nf"] = feature_subset_size(mf, n, n_est, classification)
                crit = p["split_criterion"]
                if crit in ("variance", "mse"):
                    p["split_criterion"] = "variance"
                seed = int(p["random_state"]) if p.get("random_state") is not None else 0
                key = (int(p["n_bins"]), seed)
                if key not in binned:
                    binned[key] = quantize_features(X, key[0], ctx, inp.desc.m, seed, stream=streamed,
                                                    defer=True)
                    streamed = None  # the whole shard is ordered before everything queued after it
                trees = fit_forest(X, y, ctx, inp.desc.m, p, n_local, classification, num_classes, data_parallel,
                                   rank_seed=seed * 1000003 + ctx.rank, binned=binned[key])
                binned[key] = binned[key][:2]  # its pending chunks (if any) are binned by now
                if not data_parallel and ctx.world_size > 1:
                    # forests of peer ranks of this same job (numpy node arrays), device all-gather
                    import pickle

                    from .parallel.comm import pickle_obj

                    blobs = ctx.comm.allgather_bytes(pickle_obj(trees))
                    trees = [t for b in blobs for t in pickle.loads(b)]
                res = {"trees": trees, "n_cols": int(n), "dtype": "float32", "num_classes": num_classes}
                outs.append(res)
            return outs if params["fit_multiple_params"] else outs[0]

        _fit.streaming_ingest = True  # type: ignore[attr-defined]
        # binning trails each chunk by one quantise launch: fewer, larger DMA chunks (measured -3 ms
        # per fit at 384 MB vs the 96 MB default, profiles/bench_r3_ingest_chunk_ab.txt)
        _fit.ingest_chunk_mb = 384  # type: ignore[attr-defined]
        return _fit


class _RandomForestModel(_RandomForestClass, _ModelWithPredictionCol, _RandomForestParams):
    _is_classification = True

    def __init__(self, trees: List[Dict[str, Any]], n_cols: int, dtype: str = "float32", num_classes: int = 0) -> None:
        super().__init__(trees=trees, n_cols=n_cols, dtype=dtype, num_classes=num_classes)
        self._trees = trees
        self.n_cols = int(n_cols)
        self.dtype = dtype
        self._num_classes = int(num_classes)
        self._packed: Dict[Any, Any] = {}

    @property
    def _S(self) -> int:
        return self._num_classes if self._is_classification else 1

    def _pack(self, device: torch.device) -> Dict[str, torch.Tensor]:
        from .models.forest import pack_forest

        key = str(device)
        if key not in self._packed:
            self._packed[key] = pack_forest(self._trees, self._S, device)
        return self._packed[key]

    # ---- Spark model surface -----------------------------------------------------------
    @property
    def getNumTrees(self) -> int:  # type: ignore[override]
        """Number of trees (a property on Spark's tree-ensemble models)."""
        return len(self._trees)

    @property
    def treeWeights(self) -> List[float]:
        return [1.0] * len(self._trees)

    @property
    def totalNumNodes(self) -> int:
        return sum(len(t["feature"]) for t in self._trees)

    @property
    def featureImportances(self) -> Any:
        from .core.linalg import compressed_vector
        from .models.forest import feature_importances

        return compressed_vector(feature_importances(self._trees, self.n_cols))

    @property
    def trees(self) -> List["DecisionTreeModel"]:
        return [DecisionTreeModel(t, self.n_cols, self._S, self._is_classification) for t in self._trees]

    @property
    def toDebugString(self) -> str:
        kind = "RandomForestClassificationModel" if self._is_classification else "RandomForestRegressionModel"
        s = "%s: uid=%s, numTrees=%d, numFeatures=%d\n" % (kind, self.uid, len(self._trees), self.n_cols)
        for i, t in enumerate(self.trees):
            s += "  Tree %d (weight 1.0):\n%s" % (i, t.toDebugString)
        return s

    def predictLeaf(self, value: Any) -> Any:
        x = torch.from_numpy(as_dense_array(value).astype(np.float32)).view(1, -1)
        from .models.forest import forest_predict

        _, leaves = forest_predict(x, self._pack(torch.device("cpu")), self._S, want_leaves=True)
        return Vectors.dense(leaves[0].double().numpy())

    def _raw_sum(self, X: Any, device: torch.device) -> torch.Tensor:
        from .core.base import to_device
        from .models.forest import forest_predict

        Xd = to_device(X, device, torch.float32)
        out, _ = forest_predict(Xd, self._pack(device), self._S)
        return out.double()

    def cpu(self) -> Any:
        from .utils.spark_compat import to_spark_random_forest_model

        return to_spark_random_forest_model(self)

    @classmethod
    def _combine(cls, models: List["_RandomForestModel"]) -> "_RandomForestModel":
        first = models[0]
        out = cls(**first._get_model_attributes())
        first._copyValues(out)
        first._copy_backend_params(out)
        out._combined_models = list(models)
        return out


class DecisionTreeModel:
    """Read-only view of one tree of a forest (Spark ``DecisionTree*Model`` surface)."""

    def __init__(self, tree: Dict[str, Any], n_cols: int, S: int, classification: bool) -> None:
        self._t = tree
        self.numFeatures = n_cols
        self._S = S
        self._classification = classification

    @property
    def numNodes(self) -> int:
        return len(self._t["feature"])

    @property
    def depth(self) -> int:
        return int(self._t.get("depth", 0))

    def predict(self, value: Any) -> float:
        x = as_dense_array(value)
        node = 0
        t = self._t
        while t["feature"][node] >= 0:
            node = t["left"][node] if x[t["feature"][node]] <= t["threshold"][node] else t["right"][node]
        v = t["value"][node]
        return float(np.argmax(v)) if self._classification else float(v[0])

    @property
    def toDebugString(self) -> str:
        t = self._t
        lines: List[str] = []

        def rec(node: int, indent: int) -> None:
            pad = "  " * (indent + 2)
            if t["feature"][node] < 0:
                v = t["value"][node]
                pred = float(np.argmax(v)) if self._classification else float(v[0])
                lines.append("%sPredict: %s" % (pad, pred))
                return
            f, thr = t["feature"][node], t["threshold"][node]
            lines.append("%sIf (feature %d <= %s)" % (pad, f, thr))
            rec(t["left"][node], indent + 1)
            lines.append("%sElse (feature %d > %s)" % (pad, f, thr))
            rec(t["right"][node], indent + 1)

        rec(0, 0)
        return "\n".join(lines) + "\n"
