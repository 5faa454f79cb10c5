"""In-memory DataFrame over Arrow partitions with the calls the library's Spark glue makes:
select / repartition / withColumn(unwrap_udt) / schema / rdd.getNumPartitions and the two
execution shapes it uses:

* ``mapInArrow(f).rdd.barrier().mapPartitions(identity).collect()`` — one spawned process per
  partition, ``BarrierTaskContext`` (allGather / barrier) backed by a shared board, exactly one
  task per rank (the fit stage);
* ``mapInArrow(f)`` then ``collect()`` / ``toArrow()`` — per-partition, in-process, TaskContext set.

Batches are cut at ``spark.sql.execution.arrow.maxRecordsPerBatch`` rows like Spark's Arrow path."""
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import pyarrow as pa

from .. import taskcontext
from ..ml.linalg import VectorUDT
from .types import ArrayType, BinaryType, DoubleType, FloatType, LongType, StructField, StructType


def _spark_type(field: pa.Field):
    meta = field.metadata or {}
    if b"srml.vector" in meta or (pa.types.is_struct(field.type) and field.type.num_fields == 4):
        return VectorUDT()
    t = field.type
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        return ArrayType(FloatType() if pa.types.is_float32(t.value_type) else DoubleType())
    if pa.types.is_binary(t):
        return BinaryType()
    if pa.types.is_integer(t):
        return LongType()
    return DoubleType()


class _Conf:
    def __init__(self, d: Dict[str, str]):
        self._d = d

    def get(self, k: str, default: Optional[str] = None):
        return self._d.get(k, default)

    def set(self, k: str, v: Any):
        self._d[k] = str(v)


class _SparkContext:
    def __init__(self, conf: _Conf, master: str):
        self._conf, self.master = conf, master

    def getConf(self):
        return self._conf


class SparkSession:
    _active: Optional["SparkSession"] = None

    def __init__(self, master: str = "local[2]", conf: Optional[Dict[str, str]] = None):
        self.conf = _Conf(dict(conf or {}))
        self.sparkContext = _SparkContext(self.conf, master)
        self.version = "3.5.1"
        SparkSession._active = self

    @classmethod
    def getActiveSession(cls):
        return cls._active

    def createDataFrame(self, table: pa.Table, num_partitions: int = 1) -> "DataFrame":
        return DataFrame(self, _split(table, num_partitions))


def _split(table: pa.Table, n: int) -> List[pa.Table]:
    b = np.linspace(0, table.num_rows, n + 1).astype(np.int64)
    return [table.slice(int(b[i]), int(b[i + 1] - b[i])) for i in range(n)]


def _batches(t: pa.Table, session: SparkSession):
    mx = int(session.conf.get("spark.sql.execution.arrow.maxRecordsPerBatch", "10000"))
    return iter(t.to_batches(max_chunksize=mx) or [pa.RecordBatch.from_pydict({n: [] for n in t.schema.names})])


class DataFrame:
    def __init__(self, session: SparkSession, parts: List[pa.Table], mapper: Optional[Callable] = None,
                 parent: Optional["DataFrame"] = None, out_schema: Any = None):
        self.sparkSession = session
        self._parts = parts
        self._mapper, self._parent, self._out_schema = mapper, parent, out_schema

    # ---- schema -----------------------------------------------------------------
    @property
    def schema(self) -> StructType:
        if self._mapper is not None:
            s = self._out_schema
            return s if isinstance(s, StructType) else StructType([StructField("result", BinaryType())])
        return StructType([StructField(f.name, _spark_type(f)) for f in self._parts[0].schema])

    def _materialized(self) -> "DataFrame":
        return self if self._mapper is None else DataFrame(self.sparkSession, self._eager())

    @property
    def columns(self) -> List[str]:
        return self.schema.names

    # ---- transformations ----------------------------------------------------------
    def _eager(self) -> List[pa.Table]:
        """Partitions as tables (a mapInArrow result is materialised partition by partition)."""
        if self._mapper is None:
            return self._parts
        out = []
        for pid, t in enumerate(self._parts):
            taskcontext._install(taskcontext.TaskContext(pid))
            try:
                rbs = list(self._mapper(_batches(t, self.sparkSession)))
            finally:
                taskcontext._install(None)
            out.append(pa.Table.from_batches(rbs))
        return out

    def select(self, *cols: str) -> "DataFrame":
        return DataFrame(self.sparkSession, [t.select(list(cols)) for t in self._eager()])

    def mapInPandas(self, f: Callable, schema: Any) -> "DataFrame":
        raise AssertionError("the library must use mapInArrow (zero-copy Arrow batches), not mapInPandas")

    def repartition(self, n: int) -> "DataFrame":
        whole = pa.concat_tables(self._eager())
        return DataFrame(self.sparkSession, _split(whole, n))

    def withColumn(self, name: str, c: Any) -> "DataFrame":
        assert getattr(c, "op", None) == "unwrap_udt", "fake DataFrame models withColumn(unwrap_udt) only"
        return self  # vector columns are stored as their unwrapped struct already

    def mapInArrow(self, f: Callable, schema: Any) -> "DataFrame":
        base = self._materialized()
        return DataFrame(self.sparkSession, base._parts, mapper=f, parent=base, out_schema=schema)

    @property
    def rdd(self) -> "_RDD":
        return _RDD(self)

    # ---- actions ------------------------------------------------------------------
    def toArrow(self) -> pa.Table:
        return pa.concat_tables(self._eager())

    def collect(self) -> List[Dict[str, Any]]:
        return self.toArrow().to_pylist()

    def count(self) -> int:
        return self.toArrow().num_rows


class _RDD:
    def __init__(self, df: DataFrame, barrier: bool = False):
        self._df, self._barrier = df, barrier

    def getNumPartitions(self) -> int:
        return len(self._df._parts)

    def barrier(self) -> "_RDD":
        return _RDD(self._df, True)

    def mapPartitions(self, f: Callable) -> "_RDD":
        return self  # identity in the library's use

    def withResources(self, profile: Any) -> "_RDD":
        return self

    def collect(self) -> List[Dict[str, Any]]:
        if not self._barrier:
            return self._df.collect()
        from spark_rapids_ml_nai_amd.parallel.testing import run_fake_barrier_stage

        df, session = self._df, self._df.sparkSession
        mx = int(session.conf.get("spark.sql.execution.arrow.maxRecordsPerBatch", "10000"))

        def task(ctx: Any, batches: Any) -> Any:
            from pyspark import taskcontext as tcm

            tcm._install(ctx)
            for rb in df._mapper(batches):
                yield from pa.Table.from_batches([rb]).to_pylist()

        parts = [t.to_batches(max_chunksize=mx) for t in df._parts]
        return run_fake_barrier_stage(task, parts)
