"""In-memory DataFrame over Arrow partitions with the calls the library's Spark glue makes:
select / withColumn / filter / union / join / sort / coalesce / repartition / sample, column
expressions (``functions.py``) and the execution shapes it uses:

* ``mapInArrow(f, schema, barrier=True)`` and ``mapInArrow(f).rdd.barrier().mapPartitions(identity)``
  — one spawned process per partition, ``BarrierTaskContext`` (allGather / barrier) backed by a
  shared board, exactly one task per rank (fit stages, kNN / DBSCAN / UMAP barrier jobs);
* ``mapInArrow(f)`` then an action — per-partition, in-process, TaskContext set.

Batches are cut at ``spark.sql.execution.arrow.maxRecordsPerBatch`` rows like Spark's Arrow path.
DataFrames are lazy like Spark's: a mapped frame re-runs its function on every action."""
from typing import Any, Callable, Dict, List, Optional

import numpy as np
import pyarrow as pa

from .. import taskcontext
from ..ml.linalg import VectorUDT
from .functions import Column, _c
from .types import (ArrayType, BinaryType, DoubleType, FloatType, IntegerType, LongType, StructField, StructType,
                    to_arrow_type)


def _spark_type(field: pa.Field):
    meta = field.metadata or {}
    if b"srml.vector" in meta or (pa.types.is_struct(field.type) and field.type.num_fields == 4
                                  and field.type[0].name == "type"):
        return VectorUDT()
    t = field.type
    if pa.types.is_list(t) or pa.types.is_large_list(t):
        v = t.value_type
        return ArrayType(FloatType() if pa.types.is_float32(v) else LongType() if pa.types.is_integer(v)
                         else DoubleType())
    if pa.types.is_struct(t):
        return StructType([_spark_field(f) for f in t])
    if pa.types.is_binary(t):
        return BinaryType()
    if pa.types.is_int32(t):
        return IntegerType()
    if pa.types.is_integer(t):
        return LongType()
    if pa.types.is_float32(t):
        return FloatType()
    return DoubleType()


def _spark_field(f: pa.Field) -> StructField:
    return StructField(f.name, _spark_type(f))


class _Conf:
    def __init__(self, d: Dict[str, str]):
        self._d = d

    def get(self, k: str, default: Optional[str] = None):
        return self._d.get(k, default)

    def set(self, k: str, v: Any):
        self._d[k] = str(v)


_BROADCASTS: Dict[int, Any] = {}


def _broadcast_lookup(bid: int) -> "Broadcast":
    return _BROADCASTS[bid]


class Broadcast:
    """Like Spark's: pickles as a reference to the driver-registered value (a task closure that
    holds one stays small); ``value`` resolves it where the task runs (in process here)."""

    def __init__(self, value: Any):
        self.id = len(_BROADCASTS)
        self._value = value
        _BROADCASTS[self.id] = self

    @property
    def value(self) -> Any:
        return self._value

    def unpersist(self, blocking: bool = False) -> None:
        pass

    def __reduce__(self):
        return (_broadcast_lookup, (self.id,))


class _SparkContext:
    def __init__(self, conf: _Conf, master: str):
        self._conf, self.master = conf, master
        self.broadcasts: List[Broadcast] = []

    def broadcast(self, value: Any) -> Broadcast:
        b = Broadcast(value)
        self.broadcasts.append(b)
        return b

    def getConf(self):
        return self._conf

    @property
    def defaultParallelism(self) -> int:
        return 2


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

    def createDataFrame(self, data: Any, schema: Any = None, num_partitions: int = 1) -> "DataFrame":
        if isinstance(data, pa.Table):
            return DataFrame(self, _split(data, num_partitions))
        if isinstance(data, _RDD):  # rows of a (barrier) RDD
            tables = data._tables()
            return DataFrame(self, [_conform(t, schema) for t in tables])
        rows = [r if isinstance(r, dict) else r.asDict() for r in data]
        fields = schema.fields if isinstance(schema, StructType) else None
        if fields is None:
            return DataFrame(self, _split(pa.Table.from_pylist(rows), num_partitions))
        sch = pa.schema([pa.field(f.name, to_arrow_type(f.dataType)) for f in fields])
        return DataFrame(self, _split(pa.Table.from_pylist(rows, schema=sch), num_partitions))


def _conform(t: pa.Table, schema: Any) -> pa.Table:
    if not isinstance(schema, StructType) or t.num_columns == 0:
        return t
    return t.select(schema.names)


def _split(table: pa.Table, n: int) -> List[pa.Table]:
    b = np.linspace(0, table.num_rows, n + 1).astype(np.int64)
    return [table.slice(int(b[i]), int(b[i + 1] - b[i])) for i in range(n)]


def _batches(t: pa.Table, session: SparkSession):
    mx = int(session.conf.get("spark.sql.execution.arrow.maxRecordsPerBatch", "10000"))
    return iter(t.to_batches(max_chunksize=mx))


def _ipc(tables: List[pa.Table]) -> bytes:
    sink = pa.BufferOutputStream()
    for t in tables:
        with pa.ipc.new_stream(sink, t.schema) as w:
            w.write_table(t)
    return sink.getvalue().to_pybytes()


class DataFrame:
    def __init__(self, session: SparkSession, parts: List[pa.Table], mapper: Optional[Callable] = None,
                 parent: Optional["DataFrame"] = None, out_schema: Any = None, barrier: bool = False):
        self.sparkSession = session
        self._parts = parts
        self._mapper, self._parent, self._out_schema, self._barrier = mapper, parent, out_schema, barrier

    # ---- schema -----------------------------------------------------------------
    @property
    def schema(self) -> StructType:
        if self._mapper is not None:
            s = self._out_schema
            return s if isinstance(s, StructType) else StructType([StructField("result", BinaryType())])
        return StructType([_spark_field(f) for f in self._parts[0].schema])

    def _materialized(self) -> "DataFrame":
        return self if self._mapper is None else DataFrame(self.sparkSession, self._eager())

    @property
    def columns(self) -> List[str]:
        return self.schema.names

    @property
    def dtypes(self) -> List[Any]:
        return [(f.name, repr(f.dataType)) for f in self.schema.fields]

    def __getitem__(self, name: str) -> Column:
        return Column(name)

    # ---- transformations ----------------------------------------------------------
    def _eager(self) -> List[pa.Table]:
        """Partitions as tables (a mapInArrow result is materialised partition by partition)."""
        if self._mapper is None:
            return self._parts
        if self._barrier:
            return _run_barrier(self)
        out = []
        for pid, t in enumerate(self._parts):
            taskcontext._install(taskcontext.TaskContext(pid))
            try:
                rbs = list(self._mapper(_batches(t, self.sparkSession)))
            finally:
                taskcontext._install(None)
            out.append(pa.Table.from_batches(rbs) if rbs else _empty(self._out_schema))
        return out

    def _new(self, parts: List[pa.Table]) -> "DataFrame":
        return DataFrame(self.sparkSession, parts)

    def select(self, *cols: Any) -> "DataFrame":
        if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
            cols = tuple(cols[0])
        cs = [_c(c) for c in cols]
        out = []
        for pid, t in enumerate(self._eager()):
            arrays = [c.eval(t, pid) for c in cs]
            names = [c.name for c in cs]
            ex = [i for i, c in enumerate(cs) if c.explode]
            if ex:
                i = ex[0]
                lst = arrays[i]
                lens = np.asarray(pa.compute.list_value_length(lst).fill_null(0).to_numpy(zero_copy_only=False),
                                  dtype=np.int64)
                rep = np.repeat(np.arange(t.num_rows), lens)
                arrays = [pa.compute.list_flatten(a) if j == i else a.take(pa.array(rep)) for j, a in enumerate(arrays)]
            fields = []
            for n, a in zip(names, arrays):
                src = t.schema.field(n) if n in t.schema.names and t.column(n).type == a.type else None
                fields.append(src if src is not None else pa.field(n, a.type))
            out.append(pa.Table.from_arrays(arrays, schema=pa.schema(fields)))
        return self._new(out)

    def withColumn(self, name: str, c: Any) -> "DataFrame":
        if getattr(c, "op", None) == "unwrap_udt":
            return self  # vector columns are stored as their unwrapped struct already
        out = []
        for pid, t in enumerate(self._eager()):
            a = c.eval(t, pid)
            field = c._field(name) if hasattr(c, "_field") else pa.field(name, a.type)
            if name in t.schema.names:
                t = t.set_column(t.schema.names.index(name), field, a)
            else:
                t = t.append_column(field, a)
            out.append(t)
        return self._new(out)

    def withColumnRenamed(self, old: str, new: str) -> "DataFrame":
        return self._new([t.rename_columns([new if n == old else n for n in t.schema.names]) for t in self._eager()])

    def drop(self, *names: str) -> "DataFrame":
        return self._new([t.drop([n for n in names if n in t.schema.names]) for t in self._eager()])

    def filter(self, cond: Column) -> "DataFrame":
        return self._new([t.filter(cond.eval(t, pid)) for pid, t in enumerate(self._eager())])

    where = filter

    def union(self, other: "DataFrame") -> "DataFrame":
        a, b = self._eager(), other._eager()
        names = a[0].schema.names
        return self._new(list(a) + [t.select(names).cast(a[0].schema) for t in b])

    unionAll = union

    def sample(self, withReplacement: Any = None, fraction: Optional[float] = None, seed: Optional[int] = None):
        if fraction is None:
            withReplacement, fraction = False, withReplacement
        out = []
        for pid, t in enumerate(self._eager()):
            u = np.random.default_rng((seed or 0) * 31 + pid).random(t.num_rows)
            out.append(t.filter(pa.array(u < fraction)))
        return self._new(out)

    def repartition(self, n: int, *cols: Any) -> "DataFrame":
        whole = pa.concat_tables(self._eager())
        return self._new(_split(whole, n))

    def coalesce(self, n: int) -> "DataFrame":
        parts = self._eager()
        if n >= len(parts):
            return self
        groups = np.array_split(np.arange(len(parts)), n)
        return self._new([pa.concat_tables([parts[i] for i in g]) for g in groups])

    def sort(self, *cols: Any, **kw: Any) -> "DataFrame":
        parts = self._eager()
        whole = pa.concat_tables(parts)
        keys = [(_c(c).name, "ascending") for c in cols]
        return self._new(_split(whole.sort_by(keys), len(parts)))

    orderBy = sort

    def join(self, other: "DataFrame", on: Any = None, how: str = "inner") -> "DataFrame":
        assert how == "inner", "fake join models inner joins only"
        keys = [on] if isinstance(on, str) else list(on)
        left, right = pa.concat_tables(self._eager()), pa.concat_tables(other._eager())
        lk = [tuple(r) for r in zip(*[left.column(k).to_pylist() for k in keys])]
        rk = [tuple(r) for r in zip(*[right.column(k).to_pylist() for k in keys])]
        index: Dict[Any, List[int]] = {}
        for j, k in enumerate(rk):
            index.setdefault(k, []).append(j)
        li, ri = [], []
        for i, k in enumerate(lk):
            for j in index.get(k, []):
                li.append(i)
                ri.append(j)
        lt = left.take(pa.array(li, pa.int64()))
        rt = right.drop(keys).take(pa.array(ri, pa.int64()))
        out = pa.Table.from_arrays(lt.columns + rt.columns, schema=pa.schema(list(lt.schema) + list(rt.schema)))
        return self._new(_split(out, max(1, len(self._eager()))))

    def mapInArrow(self, f: Callable, schema: Any, barrier: bool = False) -> "DataFrame":
        base = self._materialized()
        return DataFrame(self.sparkSession, base._parts, mapper=f, parent=base, out_schema=schema, barrier=barrier)

    def mapInPandas(self, f: Callable, schema: Any) -> "DataFrame":
        raise AssertionError("the library must use mapInArrow (zero-copy Arrow batches), not mapInPandas")

    def cache(self) -> "DataFrame":
        return self._materialized()

    persist = cache

    def unpersist(self, blocking: bool = False) -> "DataFrame":
        return self

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


def _empty(schema: Any) -> pa.Table:
    if isinstance(schema, StructType):
        return pa.schema([pa.field(f.name, to_arrow_type(f.dataType)) for f in schema.fields]).empty_table()
    return pa.table({"result": pa.array([], pa.binary())})


def _run_barrier(df: DataFrame) -> List[pa.Table]:
    """One spawned process per partition (BarrierTaskContext); each returns its output batches."""
    from spark_rapids_ml_nai_amd.parallel.testing import run_fake_barrier_stage

    session = df.sparkSession
    mx = int(session.conf.get("spark.sql.execution.arrow.maxRecordsPerBatch", "10000"))
    mapper, schema = df._mapper, df._out_schema

    def task(ctx: Any, batches: Any) -> Any:
        from pyspark import taskcontext as tcm

        tcm._install(ctx)
        rbs = list(mapper(batches))
        t = pa.Table.from_batches(rbs) if rbs else _empty(schema)
        yield _ipc([t])

    parts = [t.to_batches(max_chunksize=mx) for t in df._parts]
    blobs = run_fake_barrier_stage(task, parts)
    return [pa.ipc.open_stream(b).read_all() for b in blobs]


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

    def _tables(self) -> List[pa.Table]:
        if not self._barrier:
            return self._df._eager()
        d = self._df
        return _run_barrier(DataFrame(d.sparkSession, d._parts, d._mapper, d._parent, d._out_schema, True))

    def collect(self) -> List[Dict[str, Any]]:
        return [r for t in self._tables() for r in t.to_pylist()]
