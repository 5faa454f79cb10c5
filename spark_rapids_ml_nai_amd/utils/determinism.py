"""Seeded deterministic mode (SURVEY §5 "Sanitizers / deterministic mode").

The fast reductions accumulate with fp64/fp32 atomics (block partials folded in arrival order), so
their last bits can differ run to run. ``SRML_DETERMINISTIC=1`` (or ``set_deterministic(True)``,
or the Spark conf ``spark.rocm.ml.deterministic=true`` forwarded to the workers as the env var)
switches the affected kernels to fixed-order variants:

* KMeans cluster sums -> label-sorted segment sums, one block per (cluster, column chunk), no
  atomics (``srml_kmeans_segment_sums_*``);
* Gram / covariance (PCA, LinearRegression normal equations) -> each row chunk stores its
  partial tiles into a workspace (<= 64 chunks, <= 1 GB) folded in chunk order, instead of
  fp64 atomics (same fp32-per-chunk / fp64-across-chunk precision);
* fp64 GEMMs (``ops.dgemm``: X^T V, Krylov products) always fold split-K partials in index
  order, deterministic in either mode;
* LogisticRegression -> the two-pass path (residual stage + MFMA X^T R) with ordered block-partial
  folds instead of the fused atomics kernel;
* RandomForest regression histograms -> the cross-chunk fold adds exact i64 fixed-point integers
  (order-independent) converted to fp64 once (``srml_rf_hist_fixed``), node statistics one block
  per segment with a fixed-order reduction (``srml_rf_node_stats_det``); classification histograms
  are integer counts, exact in any order.

Device RNG streams are counter-based and seeded
(k-means|| sampling, bootstrap, k-means++ draws), so PCA, LinearRegression, KMeans,
LogisticRegression and RandomForestRegressor fits on the same data and partitioning are
bit-reproducible with the flag on.
"""
from __future__ import annotations

import os
from typing import Optional

_override: Optional[bool] = None


def deterministic() -> bool:
    if _override is not None:
        return _override
    return os.environ.get("SRML_DETERMINISTIC", "0") == "1"


def set_deterministic(flag: Optional[bool]) -> None:
    """Force the mode on/off for this process (None: follow ``SRML_DETERMINISTIC``)."""
    global _override
    _override = flag
