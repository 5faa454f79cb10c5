"""Test-only stand-in for the slice of the pyspark API this library calls (pyspark is not
installable in this environment). It executes the library's REAL Spark glue — the barrier
``mapInArrow`` fit stage with ``BarrierTaskContext.allGather`` bootstrap (one spawned process per
partition), the per-partition ``mapInArrow`` transform, VectorUDT unwrapping, pyspark-based Param /
Estimator / Model classes — against in-memory Arrow partitions. Spark's planner, scheduler, JVM and
Arrow IPC are not modelled: behaviour that depends on them stays "parity unpinned"."""
from spark_rapids_ml_nai_amd.core._params_builtin import keyword_only  # noqa: F401

from .taskcontext import BarrierTaskContext, TaskContext  # noqa: F401

__version__ = "3.5.1+fake"
