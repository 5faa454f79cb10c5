"""spark_rapids_ml_nai_amd — MI355X-native distributed ML with a PySpark-ML-compatible API.

Capabilities of spark-rapids-ml (PCA, KMeans, DBSCAN, exact/approximate kNN, Linear/Logistic
Regression, RandomForest, UMAP, CrossValidator) re-designed for AMD Instinct MI355X:
hand-written gfx950 HIP kernels (MFMA/LDS) for every hot primitive, one process per GPU with
RCCL collectives over xGMI, and a Spark-free columnar (Arrow) data plane with an optional
Spark barrier-mode adapter.
"""
__version__ = "24.06.0"

from .core.dataframe import DataFrame, Row  # noqa: E402,F401
