"""``feature.PCA`` / ``PCAModel`` — PySpark-ML compatible API (reference ``feature.py:61-447``).

Param mapping ``k -> n_components``; backend defaults ``n_components=None, svd_solver="auto",
whiten=False``. ``PCAModel.transform`` follows Spark: rows are projected without centring
(the reference gets there by adding ``mean·Cᵀ`` back after cuML's centred transform).
Output column type mirrors the input: ``array<float|double>``, or a vector for VectorUDT input.
"""
from __future__ import annotations

import itertools
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import torch

from .core.base import FitInput, _Estimator, _Model
from .core.dataframe import DataFrame
from .core.linalg import DenseMatrix, DenseVector
from .core.params import (
    HasInputCol,
    HasInputCols,
    HasOutputCol,
    Param,
    Params,
    TypeConverters,
    _BackendClass,
    _BackendParams,
    keyword_only,
)
from .parallel.context import WorkerContext


class PCAClass(_BackendClass):
    @classmethod
    def _param_mapping(cls) -> Dict[str, Optional[str]]:
        return {"k": "n_components"}

    def _get_backend_params_default(self) -> Dict[str, Any]:
        return {"n_components": None, "svd_solver": "auto", "verbose": False, "whiten": False}


class _PCAParams(_BackendParams, HasInputCol, HasInputCols, HasOutputCol):
    k = Param(Params._dummy(), "k", "the number of principal components (> 0)", typeConverter=TypeConverters.toInt)

    def getK(self) -> int:
        return self.getOrDefault(self.k)

    def setInputCol(self, value: Union[str, List[str]]) -> Any:
        if isinstance(value, str):
            return self._set_params(inputCol=value)
        return self._set_params(inputCols=value)

    def setInputCols(self, value: List[str]) -> Any:
        return self._set_params(inputCols=value)

    def setOutputCol(self, value: str) -> Any:
        return self._set_params(outputCol=value)


class PCA(PCAClass, _Estimator, _PCAParams):
    """GPU-accelerated distributed PCA (mean + covariance all-reduce, top-k eigensolver).

    >>> from spark_rapids_ml_nai_amd.feature import PCA
    >>> df = DataFrame.createDataFrame([([1.0, 1.0],), ([2.0, 2.0],), ([3.0, 3.0],)], ["features"])
    >>> model = PCA(k=1, inputCol="features").fit(df)
    >>> model.mean
    [2.0, 2.0]
    """

    @keyword_only
    def __init__(self, *, k: Optional[int] = None, inputCol: Optional[Union[str, List[str]]] = None,
                 outputCol: Optional[str] = None, num_workers: Optional[int] = None,
                 verbose: Union[int, bool] = False, **kwargs: Any) -> None:
        super().__init__()
        self._setDefault(outputCol=self.uid + "__output")
        self._set_params(**self._input_kwargs)

    def setK(self, value: int) -> "PCA":
        return self._set_params(k=value)

    def _get_fit_func(self, dataset: DataFrame, extra_params: Optional[List[Dict[str, Any]]] = None) -> Callable:
        def _fit(inp: FitInput, ctx: WorkerContext, params: Dict[str, Any]) -> Dict[str, Any]:
            from .models.pca import pca_fit

            init = params["cuml_init"]
            return pca_fit(inp.X, inp.desc.m, ctx, init.get("n_components"), stream=inp.stream)

        _fit.streaming_ingest = True  # type: ignore[attr-defined]
        return _fit

    def _create_model(self, result: Dict[str, Any]) -> "PCAModel":
        return PCAModel._from_row(result)


class PCAModel(PCAClass, _Model, _PCAParams):
    def __init__(self, mean_: List[float], components_: List[List[float]], explained_variance_ratio_: List[float],
                 singular_values_: List[float], n_cols: int, dtype: str) -> None:
        super().__init__(mean_=mean_, components_=components_, explained_variance_ratio_=explained_variance_ratio_,
                         singular_values_=singular_values_, n_cols=n_cols, dtype=dtype)
        self.mean_ = list(mean_)
        self.components_ = [list(c) for c in components_]
        self.explained_variance_ratio_ = list(explained_variance_ratio_)
        self.singular_values_ = list(singular_values_)
        self.n_cols = int(n_cols)
        self.dtype = dtype
        self._setDefault(outputCol=self.uid + "__output")
        self._set_params(n_components=len(self.components_))

    @property
    def mean(self) -> List[float]:
        return self.mean_

    @property
    def pc(self) -> DenseMatrix:
        """Principal components, one per column (n_cols x k, column-major)."""
        values = list(itertools.chain.from_iterable(self.components_))
        return DenseMatrix(self.n_cols, len(self.components_), values, False)

    @property
    def explainedVariance(self) -> DenseVector:
        return DenseVector(self.explained_variance_ratio_)

    @property
    def explained_variance(self) -> List[float]:
        return self.explained_variance_ratio_

    def getK(self) -> int:
        return len(self.components_)

    def cpu(self) -> Any:
        from .utils.spark_compat import to_spark_pca_model

        return to_spark_pca_model(self)

    def _get_transform_func(self, dataset: DataFrame) -> Tuple[Callable, Callable]:
        comps = np.asarray(self.components_, dtype=np.float64)
        out_col = self.getOrDefault("outputCol")
        np_dt = np.float32 if self.dtype == "float32" else np.float64

        def construct(ctx: WorkerContext) -> torch.Tensor:
            return torch.from_numpy(comps.astype(np_dt)).to(ctx.device)

        def predict(C: torch.Tensor, X: Any, ctx: WorkerContext) -> Dict[str, np.ndarray]:
            from .core.base import to_device
            from .models.pca import pca_transform

            Xd = to_device(X, ctx.device, C.dtype)
            return {out_col: pca_transform(Xd, C).cpu().numpy().astype(np_dt)}

        return construct, predict

    def _vector_output_cols(self) -> List[str]:
        return []

    def _spark_vector_output_cols(self, input_is_vector: bool) -> List[str]:
        return [self.getOrDefault("outputCol")] if input_is_vector else []

    def _transform_df(self, df: DataFrame) -> DataFrame:
        out = super()._transform_df(df)
        col, _ = self._get_input_columns()
        oc = self.getOrDefault("outputCol")
        if col is not None and df.is_vector(col):
            X = out.to_numpy(oc, np.float64)
            from .core.dataframe import dense_to_vector_array

            out = out.withColumn(oc, dense_to_vector_array(X), vector=True)
        return out
