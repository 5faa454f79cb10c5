"""Distributed PCA solver (Spark-free; runs on one rank per MI355X).

Reference behaviour: cuML ``PCAMG.fit`` called from ``feature.py:216-257`` — column means and
covariance reduced over NCCL, eigendecomposition, sign flip, explained-variance ratio, singular
values. MI355X pipeline per rank:

1-2. one pass (``models/stats.py``; chunk by chunk while the shard's H2D is still in flight):
   ``col_moments`` column sums + the ``gram`` MFMA SYRK about a shift estimated from the first
   chunk, exactly re-centred in fp64 -> RCCL all-reduce of the sums (n) and of the scatter (n^2)
3. top-k eigensolver on the replicated covariance (``models/eig.py``), sign-fixed on device
4. attributes exactly as the reference persists them (mean_, components_ k x n,
   explained_variance_ratio_ = λ/trace, singular_values_ = sqrt((m-1) λ), n_cols, dtype)
"""
from __future__ import annotations

from typing import Any, Dict

import numpy as np
import torch

from .. import ops
from ..parallel.context import WorkerContext
from .eig import topk_eigh


def pca_fit(X: torch.Tensor, m_total: int, ctx: WorkerContext, n_components: Any, timer: Any = None,
            stream: Any = None) -> Dict[str, Any]:
    from .stats import scatter_stats

    n = X.shape[1]
    k = n if n_components is None else int(n_components)
    if k > n:
        raise ValueError("k (%d) must be <= number of features (%d)" % (k, n))
    st = scatter_stats(X, ctx, m_total, stream=stream, need_sq=False)
    mean, G = st.mean, st.scatter
    denom = float(max(m_total - 1, 1))
    cov = G / denom
    total_var = float(torch.trace(cov).item())
    vals, vecs = topk_eigh(cov, k)
    vals = np.maximum(vals, 0.0)
    ratio = vals / total_var if total_var > 0 else np.zeros_like(vals)
    sing = np.sqrt(vals * denom)
    return {
        "mean_": mean.cpu().numpy().tolist(),
        "components_": vecs.T.tolist(),
        "explained_variance_ratio_": ratio.tolist(),
        "singular_values_": sing.tolist(),
        "n_cols": int(n),
        "dtype": "float32" if X.dtype == torch.float32 else "float64",
    }


def pca_transform(X: torch.Tensor, components: torch.Tensor) -> torch.Tensor:
    """Spark semantics: project the *uncentred* rows, out = X @ components^T (one pass over X)."""
    return ops.xw(X, components.T.contiguous())
