"""A partitioned, columnar (Apache Arrow) DataFrame: the Spark-free data plane.

The reference consumes Spark DataFrames inside barrier ``mapInPandas`` tasks and converts
every Arrow batch with a per-row Python loop (``np.array(list(pdf[col]))``,
``core.py:724-748``). Here a DataFrame is a list of ``pyarrow.Table`` partitions (one per
future device worker), and feature ingest is zero-copy: an ``array<float>`` column whose
rows all have the same length is the Arrow values buffer reshaped to ``(rows, n)``; a
VectorUDT-shaped column (struct ``type/size/indices/values`` exactly like Spark's
``VectorUDT.sqlType``) yields either that dense view or a CSR matrix assembled from the
child offset buffers (no Python per-row loop).

The DataFrame surface mirrors the subset of ``pyspark.sql.DataFrame`` that the ML API and
its tests use: ``columns``, ``schema``, ``select``, ``withColumn``, ``drop``, ``repartition``,
``union``, ``collect``, ``first``, ``toPandas``, ``count``, ``randomSplit``, ``filter``...
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.compute as pc

from .linalg import DenseVector, SparseVector, Vectors

VECTOR_META_KEY = b"srml.udt"
VECTOR_META_VAL = b"vector"

VECTOR_STRUCT = pa.struct(
    [
        pa.field("type", pa.int8()),
        pa.field("size", pa.int32()),
        pa.field("indices", pa.list_(pa.int32())),
        pa.field("values", pa.list_(pa.float64())),
    ]
)


class Row(tuple):
    """pyspark.sql.Row look-alike: tuple with attribute access and ``asDict``."""

    def __new__(cls, *args: Any, **kwargs: Any) -> "Row":
        if kwargs:
            row = tuple.__new__(cls, list(kwargs.values()))
            row.__fields__ = list(kwargs.keys())
            return row
        row = tuple.__new__(cls, args)
        row.__fields__ = None
        return row

    def asDict(self, recursive: bool = False) -> Dict[str, Any]:
        if self.__fields__ is None:
            raise TypeError("Cannot convert a Row class into dict")
        return dict(zip(self.__fields__, self))

    def __getattr__(self, item: str) -> Any:
        if item.startswith("__"):
            raise AttributeError(item)
        try:
            return self[self.__fields__.index(item)]
        except (ValueError, AttributeError, TypeError):
            raise AttributeError(item)

    def __getitem__(self, item: Any) -> Any:
        if isinstance(item, str):
            return super().__getitem__(self.__fields__.index(item))
        return super().__getitem__(item)

    def __repr__(self) -> str:
        if self.__fields__:
            return "Row(%s)" % ", ".join("%s=%r" % (k, v) for k, v in zip(self.__fields__, self))
        return "<Row(%s)>" % ", ".join(repr(v) for v in self)


# --------------------------------------------------------------------------------------
# Arrow helpers
# --------------------------------------------------------------------------------------
def is_vector_field(field: pa.Field) -> bool:
    md = field.metadata or {}
    return md.get(VECTOR_META_KEY) == VECTOR_META_VAL or (
        pa.types.is_struct(field.type)
        and [f.name for f in field.type] == ["type", "size", "indices", "values"]
    )


def vector_field(name: str) -> pa.Field:
    return pa.field(name, VECTOR_STRUCT, metadata={VECTOR_META_KEY: VECTOR_META_VAL})


def is_array_field(field: pa.Field) -> bool:
    return pa.types.is_list(field.type) or pa.types.is_large_list(field.type) or pa.types.is_fixed_size_list(
        field.type
    )


def dense_to_list_array(X: np.ndarray) -> pa.Array:
    """(rows, n) ndarray -> list<float> Arrow array sharing X's buffer (no per-row objects)."""
    X = np.ascontiguousarray(X)
    m, n = X.shape
    offsets = pa.array(np.arange(0, (m + 1) * n, n, dtype=np.int32) if m * n < 2**31 else
                       np.arange(0, (m + 1) * n, n, dtype=np.int64))
    values = pa.array(X.reshape(-1))
    if offsets.type == pa.int64():
        return pa.LargeListArray.from_arrays(offsets, values)
    return pa.ListArray.from_arrays(offsets, values)


def dense_to_vector_array(X: np.ndarray) -> pa.Array:
    X = np.ascontiguousarray(X, dtype=np.float64)
    m, n = X.shape
    types = pa.array(np.ones(m, dtype=np.int8))
    sizes = pa.array(np.full(m, n, dtype=np.int32))
    empty = pa.ListArray.from_arrays(pa.array(np.zeros(m + 1, dtype=np.int32)), pa.array([], pa.int32()))
    vals = pa.ListArray.from_arrays(pa.array(np.arange(0, (m + 1) * n, n, dtype=np.int32)), pa.array(X.reshape(-1)))
    return pa.StructArray.from_arrays([types, sizes, empty, vals], fields=list(VECTOR_STRUCT))


def vectors_to_arrow(values: Sequence[Any]) -> pa.Array:
    """Python Dense/SparseVector objects -> VectorUDT-shaped struct array."""
    types, sizes, idx_off, idx, val_off, vals = [], [], [0], [], [0], []
    for v in values:
        if isinstance(v, SparseVector) or (hasattr(v, "indices") and hasattr(v, "size") and not isinstance(v, DenseVector)):
            types.append(0)
            sizes.append(int(v.size))
            idx.extend(np.asarray(v.indices, dtype=np.int32).tolist())
            vals.extend(np.asarray(v.values, dtype=np.float64).tolist())
        else:
            arr = np.asarray(v.toArray() if hasattr(v, "toArray") else v, dtype=np.float64)
            types.append(1)
            sizes.append(arr.shape[0])
            vals.extend(arr.tolist())
        idx_off.append(len(idx))
        val_off.append(len(vals))
    return pa.StructArray.from_arrays(
        [
            pa.array(types, pa.int8()),
            pa.array(sizes, pa.int32()),
            pa.ListArray.from_arrays(pa.array(idx_off, pa.int32()), pa.array(idx, pa.int32())),
            pa.ListArray.from_arrays(pa.array(val_off, pa.int32()), pa.array(vals, pa.float64())),
        ],
        fields=list(VECTOR_STRUCT),
    )


def _combine(col: Union[pa.ChunkedArray, pa.Array]) -> pa.Array:
    if isinstance(col, pa.ChunkedArray):
        if col.num_chunks == 1:
            return col.chunk(0)
        return col.combine_chunks() if col.num_chunks else pa.array([], col.type)
    return col


def _list_offsets_values(arr: pa.Array) -> Tuple[np.ndarray, pa.Array]:
    if pa.types.is_fixed_size_list(arr.type):
        n = arr.type.list_size
        offs = np.arange(arr.offset, arr.offset + len(arr) + 1, dtype=np.int64) * n
        return offs, arr.values
    offs = np.asarray(arr.offsets.to_numpy(zero_copy_only=False), dtype=np.int64)
    return offs, arr.values


def array_column_to_dense(col: Union[pa.ChunkedArray, pa.Array], dtype: Optional[np.dtype] = None) -> np.ndarray:
    """list<float> column -> (rows, n) ndarray; zero-copy when rows are uniform and dtype matches.
    A multi-chunk column is converted chunk by chunk and concatenated in numpy: Arrow's
    ``combine_chunks`` overflows ``list<float>``'s int32 offsets past 2^31 values (a 1M x 3000
    partition delivered as record batches)."""
    if isinstance(col, pa.ChunkedArray) and col.num_chunks > 1:
        parts = [array_column_to_dense(c, dtype) for c in col.chunks if len(c) > 0]
        if not parts:
            return np.zeros((0, 0), dtype=dtype or np.float32)
        return np.concatenate(parts, 0)
    arr = _combine(col)
    m = len(arr)
    if m == 0:
        return np.zeros((0, 0), dtype=dtype or np.float32)
    offs, values = _list_offsets_values(arr)
    lens = np.diff(offs)
    n = int(lens[0])
    if not np.all(lens == n):
        raise ValueError("array column has rows of different lengths")
    flat = values.to_numpy(zero_copy_only=False)
    flat = flat[offs[0]: offs[0] + m * n]
    X = flat.reshape(m, n)
    if dtype is not None and X.dtype != dtype:
        X = X.astype(dtype)
    return X


class ChunkedRows:
    """Row blocks of one host partition, each a zero-copy (rows_i, n) view of one Arrow batch's
    values buffer (Spark delivers ``maxRecordsPerBatch``-row batches in separate buffers).
    ``ops.ingest.parts_to_device`` streams them to the device without first concatenating the
    partition on the host (a full extra copy of the data)."""

    ndim = 2

    def __init__(self, parts: List[np.ndarray]) -> None:
        self.parts = [p for p in parts if p.shape[0] > 0] or parts[:1]
        n = int(self.parts[0].shape[1]) if self.parts else 0
        if any(int(p.shape[1]) != n for p in self.parts):
            raise ValueError("array column has rows of different lengths")
        self.shape = (int(sum(p.shape[0] for p in self.parts)), n)
        self.dtype = self.parts[0].dtype if self.parts else np.dtype(np.float32)

    def __len__(self) -> int:
        return self.shape[0]

    def to_numpy(self) -> np.ndarray:
        return np.concatenate(self.parts, 0) if len(self.parts) > 1 else self.parts[0]

    def __array__(self, dtype: Any = None, copy: Any = None) -> np.ndarray:
        a = self.to_numpy()
        return a if dtype is None else a.astype(dtype, copy=False)


def array_column_chunks(col: Union[pa.ChunkedArray, pa.Array], dtype: Optional[np.dtype] = None) -> ChunkedRows:
    """list<float> column -> ``ChunkedRows``: one zero-copy 2-D view per Arrow chunk (a per-chunk
    cast only when the element type differs from ``dtype``)."""
    chunks = col.chunks if isinstance(col, pa.ChunkedArray) else [col]
    parts = [array_column_to_dense(c, dtype) for c in chunks if len(c) > 0]
    if not parts:
        parts = [np.zeros((0, 0), dtype=dtype or np.float32)]
    return ChunkedRows(parts)


def vector_column_is_sparse(col: Union[pa.ChunkedArray, pa.Array]) -> bool:
    arr = _combine(col)
    if len(arr) == 0:
        return False
    return int(arr.field("type")[0].as_py()) == 0


def vector_column_to_dense(col: Union[pa.ChunkedArray, pa.Array], dtype: Optional[np.dtype] = None) -> np.ndarray:
    arr = _combine(col)
    m = len(arr)
    if m == 0:
        return np.zeros((0, 0), dtype=dtype or np.float64)
    types = arr.field("type").to_numpy(zero_copy_only=False)
    if np.all(types == 1):
        X = array_column_to_dense(arr.field("values"))
        return X.astype(dtype) if dtype is not None and X.dtype != dtype else X
    csr = vector_column_to_csr(arr, dtype or np.float64)
    return csr.toarray()


def vector_column_to_csr(col: Union[pa.ChunkedArray, pa.Array], dtype: np.dtype = np.float64) -> Any:
    """VectorUDT struct column -> scipy CSR, built from Arrow offset buffers (dense rows expanded)."""
    import scipy.sparse as sp

    arr = _combine(col)
    m = len(arr)
    types = arr.field("type").to_numpy(zero_copy_only=False).astype(np.int8)
    sizes = arr.field("size").to_numpy(zero_copy_only=False)
    n = int(sizes.max()) if m else 0
    ioffs, ivals = _list_offsets_values(arr.field("indices"))
    voffs, vvals = _list_offsets_values(arr.field("values"))
    ind = ivals.to_numpy(zero_copy_only=False)
    val = vvals.to_numpy(zero_copy_only=False)
    vlen = np.diff(voffs)
    if np.all(types == 0):
        indptr = (ioffs - ioffs[0]).astype(np.int64)
        indices = ind[ioffs[0]: ioffs[-1]].astype(np.int32)
        data = val[voffs[0]: voffs[-1]].astype(dtype)
        return sp.csr_matrix((data, indices, indptr), shape=(m, n))
    # mixed dense/sparse rows: per-row index arrays synthesised vectorially
    row_nnz = np.where(types == 1, vlen, np.diff(ioffs))
    indptr = np.concatenate([[0], np.cumsum(row_nnz)]).astype(np.int64)
    indices = np.empty(indptr[-1], dtype=np.int32)
    data = np.empty(indptr[-1], dtype=dtype)
    dense_rows = np.nonzero(types == 1)[0]
    sparse_rows = np.nonzero(types == 0)[0]
    for r in dense_rows:
        s = indptr[r]
        L = vlen[r]
        indices[s: s + L] = np.arange(L, dtype=np.int32)
        data[s: s + L] = val[voffs[r]: voffs[r] + L]
    for r in sparse_rows:
        s, e = indptr[r], indptr[r + 1]
        indices[s:e] = ind[ioffs[r]: ioffs[r + 1]]
        data[s:e] = val[voffs[r]: voffs[r + 1]]
    return sp.csr_matrix((data, indices, indptr), shape=(m, n))


def _pandas_col_to_arrow(s: pd.Series) -> Tuple[pa.Array, bool]:
    """Returns (arrow array, is_vector)."""
    if s.dtype == object and len(s) > 0:
        first = next((v for v in s if v is not None), None)
        if isinstance(first, (DenseVector, SparseVector)) or (
            first is not None and hasattr(first, "toArray") and hasattr(first, "size")
        ):
            return vectors_to_arrow(list(s)), True
        if isinstance(first, (list, tuple, np.ndarray)):
            lens = {len(v) for v in s}
            if len(lens) == 1:
                X = np.stack([np.asarray(v) for v in s])
                if X.dtype == np.float64 or X.dtype == np.float32 or np.issubdtype(X.dtype, np.integer):
                    return dense_to_list_array(X), False
            return pa.array([list(v) for v in s]), False
    return pa.array(s), False


def _to_arrow_array(values: Any, n_rows: int) -> Tuple[pa.Array, bool]:
    if isinstance(values, (pa.Array, pa.ChunkedArray)):
        return _combine(values), False
    if isinstance(values, pd.Series):
        return _pandas_col_to_arrow(values.reset_index(drop=True))
    if isinstance(values, np.ndarray):
        if values.ndim == 2:
            return dense_to_list_array(values), False
        return pa.array(values), False
    if np.isscalar(values):
        return pa.array([values] * n_rows), False
    return _pandas_col_to_arrow(pd.Series(list(values)))


# --------------------------------------------------------------------------------------
# DataFrame
# --------------------------------------------------------------------------------------
class DataFrame:
    """List of Arrow tables (partitions) sharing one schema."""

    def __init__(self, partitions: List[pa.Table]) -> None:
        if not partitions:
            raise ValueError("DataFrame needs at least one partition")
        schema = partitions[0].schema
        self._parts = [p if p.schema.equals(schema) else p.cast(schema) for p in partitions]

    # ---- construction -------------------------------------------------------------
    @classmethod
    def from_arrow(cls, table: pa.Table, num_partitions: int = 1) -> "DataFrame":
        return cls([table]).repartition(num_partitions) if num_partitions > 1 else cls([table])

    @classmethod
    def from_pandas(cls, pdf: pd.DataFrame, num_partitions: int = 1) -> "DataFrame":
        arrays, fields = [], []
        for name in pdf.columns:
            arr, is_vec = _pandas_col_to_arrow(pdf[name].reset_index(drop=True))
            arrays.append(arr)
            fields.append(vector_field(name) if is_vec else pa.field(name, arr.type))
        table = pa.Table.from_arrays(arrays, schema=pa.schema(fields))
        return cls.from_arrow(table, num_partitions)

    @classmethod
    def from_numpy(
        cls,
        X: Any,
        y: Optional[np.ndarray] = None,
        features_col: str = "features",
        label_col: str = "label",
        num_partitions: int = 1,
        vector: bool = False,
        extra: Optional[Dict[str, Any]] = None,
    ) -> "DataFrame":
        """Build from a dense (rows, n) array, or a scipy sparse matrix (stored as VectorUDT)."""
        import scipy.sparse as sp

        arrays: List[pa.Array] = []
        fields: List[pa.Field] = []
        if sp.issparse(X):
            csr = sp.csr_matrix(X)
            m, n = csr.shape
            arr = pa.StructArray.from_arrays(
                [
                    pa.array(np.zeros(m, dtype=np.int8)),
                    pa.array(np.full(m, n, dtype=np.int32)),
                    pa.ListArray.from_arrays(pa.array(csr.indptr.astype(np.int32)), pa.array(csr.indices.astype(np.int32))),
                    pa.ListArray.from_arrays(pa.array(csr.indptr.astype(np.int32)), pa.array(csr.data.astype(np.float64))),
                ],
                fields=list(VECTOR_STRUCT),
            )
            arrays.append(arr)
            fields.append(vector_field(features_col))
        elif vector:
            arrays.append(dense_to_vector_array(np.asarray(X)))
            fields.append(vector_field(features_col))
        else:
            a = dense_to_list_array(np.asarray(X))
            arrays.append(a)
            fields.append(pa.field(features_col, a.type))
        if y is not None:
            ya = pa.array(np.asarray(y))
            arrays.append(ya)
            fields.append(pa.field(label_col, ya.type))
        for k, v in (extra or {}).items():
            a, is_vec = _to_arrow_array(v, len(arrays[0]))
            arrays.append(a)
            fields.append(vector_field(k) if is_vec else pa.field(k, a.type))
        table = pa.Table.from_arrays(arrays, schema=pa.schema(fields))
        return cls.from_arrow(table, num_partitions)

    @classmethod
    def createDataFrame(cls, data: Any, schema: Any = None, num_partitions: int = 1) -> "DataFrame":
        """Like ``SparkSession.createDataFrame`` for lists of tuples / Rows / dicts or pandas."""
        if isinstance(data, pd.DataFrame):
            return cls.from_pandas(data, num_partitions)
        rows = list(data)
        if isinstance(schema, str):
            names = [s.strip().split(" ")[0] for s in schema.split(",")]
        elif isinstance(schema, (list, tuple)):
            names = list(schema)
        elif rows and isinstance(rows[0], Row) and rows[0].__fields__:
            names = list(rows[0].__fields__)
        elif rows and isinstance(rows[0], dict):
            names = list(rows[0].keys())
            rows = [tuple(r[k] for k in names) for r in rows]
        else:
            names = ["_%d" % (i + 1) for i in range(len(rows[0]))]
        cols = {n: [r[i] for r in rows] for i, n in enumerate(names)}
        pdf = pd.DataFrame({n: pd.Series(v, dtype=object if _needs_object(v) else None) for n, v in cols.items()})
        return cls.from_pandas(pdf, num_partitions)

    @classmethod
    def read_parquet(cls, path: str, columns: Optional[List[str]] = None) -> "DataFrame":
        """One partition per Parquet file (a directory of part files, or a single file)."""
        import glob
        import os

        import pyarrow.parquet as pq

        files = sorted(glob.glob(os.path.join(path, "*.parquet"))) if os.path.isdir(path) else [path]
        if not files:
            raise FileNotFoundError("no parquet files under %s" % path)
        return cls([pq.read_table(f, columns=columns) for f in files])

    def write_parquet(self, path: str, overwrite: bool = False) -> None:
        import os
        import shutil

        import pyarrow.parquet as pq

        if os.path.exists(path):
            if not overwrite:
                raise FileExistsError(path)
            shutil.rmtree(path)
        os.makedirs(path)
        for i, p in enumerate(self._parts):
            pq.write_table(p, os.path.join(path, "part-%05d.parquet" % i))

    # ---- schema -------------------------------------------------------------------
    @property
    def schema(self) -> pa.Schema:
        return self._parts[0].schema

    @property
    def columns(self) -> List[str]:
        return list(self.schema.names)

    @property
    def dtypes(self) -> List[Tuple[str, str]]:
        out = []
        for f in self.schema:
            if is_vector_field(f):
                out.append((f.name, "vector"))
            elif is_array_field(f):
                out.append((f.name, "array<%s>" % _simple_type(f.type.value_type)))
            else:
                out.append((f.name, _simple_type(f.type)))
        return out

    @property
    def partitions(self) -> List[pa.Table]:
        return list(self._parts)

    def getNumPartitions(self) -> int:
        return len(self._parts)

    @property
    def rdd(self) -> "DataFrame":  # ``df.rdd.getNumPartitions()`` idiom
        return self

    def is_vector(self, name: str) -> bool:
        return is_vector_field(self.schema.field(name))

    def is_array(self, name: str) -> bool:
        return is_array_field(self.schema.field(name))

    # ---- transformations ----------------------------------------------------------
    def count(self) -> int:
        return sum(p.num_rows for p in self._parts)

    def select(self, *cols: Union[str, List[str]]) -> "DataFrame":
        names: List[str] = []
        for c in cols:
            names.extend(c if isinstance(c, (list, tuple)) else [c])
        if names == ["*"]:
            return self
        return DataFrame([p.select(names) for p in self._parts])

    def drop(self, *cols: str) -> "DataFrame":
        keep = [c for c in self.columns if c not in cols]
        return DataFrame([p.select(keep) for p in self._parts])

    def withColumnRenamed(self, existing: str, new: str) -> "DataFrame":
        names = [new if c == existing else c for c in self.columns]
        return DataFrame([_rename(p, names) for p in self._parts])

    def withColumn(self, name: str, values: Any, vector: Optional[bool] = None) -> "DataFrame":
        """Add/replace a column. ``values`` is a whole-frame array/list/Series, a scalar, or a
        function ``f(partition_table) -> array`` evaluated per partition."""
        parts = []
        if callable(values) and not isinstance(values, (np.ndarray, pd.Series, pa.Array)):
            per_part = [values(p) for p in self._parts]
        else:
            n_total = self.count()
            if isinstance(values, (pa.Array, pa.ChunkedArray)):
                arr_all, is_vec_all = _combine(values), False
            else:
                arr_all, is_vec_all = _to_arrow_array(values, n_total)
            per_part, off = [], 0
            for p in self._parts:
                per_part.append((arr_all.slice(off, p.num_rows), is_vec_all))
                off += p.num_rows
        for p, v in zip(self._parts, per_part):
            if isinstance(v, tuple):
                arr, is_vec = v
            else:
                arr, is_vec = _to_arrow_array(v, p.num_rows)
            if vector is not None:
                is_vec = vector
            fld = vector_field(name) if is_vec else pa.field(name, arr.type)
            if name in p.column_names:
                i = p.column_names.index(name)
                p = p.set_column(i, fld, arr)
            else:
                p = p.append_column(fld, arr)
            parts.append(p)
        return DataFrame(parts)

    def repartition(self, num_partitions: int, *cols: Any) -> "DataFrame":
        table = self._concat()
        m = table.num_rows
        num_partitions = max(1, int(num_partitions))
        bounds = np.linspace(0, m, num_partitions + 1).astype(np.int64)
        return DataFrame([table.slice(int(bounds[i]), int(bounds[i + 1] - bounds[i])) for i in range(num_partitions)])

    def coalesce(self, num_partitions: int) -> "DataFrame":
        return self.repartition(num_partitions) if num_partitions < len(self._parts) else self

    def union(self, other: "DataFrame") -> "DataFrame":
        other = other.select(*self.columns) if other.columns != self.columns else other
        o_parts = [p.cast(self.schema) for p in other._parts]
        return DataFrame(self._parts + o_parts)

    unionAll = union
    unionByName = union

    def filter(self, condition: Any) -> "DataFrame":
        """``condition``: boolean mask (whole frame), or f(partition_table)->mask, or pyarrow expression."""
        parts = []
        if callable(condition) and not isinstance(condition, (np.ndarray, pd.Series)):
            for p in self._parts:
                parts.append(p.filter(pa.array(np.asarray(condition(p), dtype=bool))))
        else:
            mask = np.asarray(condition, dtype=bool)
            off = 0
            for p in self._parts:
                parts.append(p.filter(pa.array(mask[off: off + p.num_rows])))
                off += p.num_rows
        return DataFrame(parts)

    where = filter

    def sort(self, col: str, ascending: bool = True) -> "DataFrame":
        table = self._concat()
        idx = pc.sort_indices(table, sort_keys=[(col, "ascending" if ascending else "descending")])
        return DataFrame([table.take(idx)]).repartition(len(self._parts))

    orderBy = sort

    def randomSplit(self, weights: Sequence[float], seed: Optional[int] = None) -> List["DataFrame"]:
        w = np.asarray(weights, dtype=np.float64)
        w = w / w.sum()
        rng = np.random.default_rng(seed)
        outs: List[List[pa.Table]] = [[] for _ in w]
        edges = np.concatenate([[0.0], np.cumsum(w)])
        for p in self._parts:
            u = rng.random(p.num_rows)
            for i in range(len(w)):
                outs[i].append(p.filter(pa.array((u >= edges[i]) & (u < edges[i + 1]))))
        return [DataFrame(o) for o in outs]

    def sample(self, fraction: float, seed: Optional[int] = None, withReplacement: bool = False) -> "DataFrame":
        rng = np.random.default_rng(seed)
        return DataFrame([p.filter(pa.array(rng.random(p.num_rows) < fraction)) for p in self._parts])

    def limit(self, n: int) -> "DataFrame":
        return DataFrame([self._concat().slice(0, n)])

    def with_row_id(self, name: str, start: int = 0) -> "DataFrame":
        """monotonically increasing int64 id (partition-major, like Spark's id generator) from
        ``start`` (an SPMD rank's global row offset)."""
        parts, off = [], int(start)
        for p in self._parts:
            ids = pa.array(np.arange(off, off + p.num_rows, dtype=np.int64))
            parts.append(p.append_column(pa.field(name, pa.int64()), ids))
            off += p.num_rows
        return DataFrame(parts)

    def cache(self) -> "DataFrame":
        return self

    persist = cache

    def unpersist(self, blocking: bool = False) -> "DataFrame":
        return self

    # ---- actions ------------------------------------------------------------------
    def _concat(self) -> pa.Table:
        if len(self._parts) == 1:
            return self._parts[0]
        return pa.concat_tables(self._parts)

    def column(self, name: str) -> pa.ChunkedArray:
        return self._concat().column(name)

    def to_numpy(self, name: str, dtype: Optional[np.dtype] = None) -> np.ndarray:
        """Dense numpy view of one column over the whole frame (arrays -> (rows, n))."""
        f = self.schema.field(name)
        col = self.column(name)
        if is_vector_field(f):
            return vector_column_to_dense(col, dtype)
        if is_array_field(f):
            return array_column_to_dense(col, dtype)
        out = col.to_numpy()
        return out.astype(dtype) if dtype is not None else out

    def toPandas(self) -> pd.DataFrame:
        table = self._concat()
        data = {}
        for f in table.schema:
            col = table.column(f.name)
            if is_vector_field(f):
                data[f.name] = pd.Series(_vectors_from_arrow(col), dtype=object)
            elif is_array_field(f):
                try:
                    X = array_column_to_dense(col)
                    data[f.name] = pd.Series(list(X), dtype=object)
                except ValueError:
                    data[f.name] = pd.Series([np.asarray(v) for v in col.to_pylist()], dtype=object)
            else:
                data[f.name] = col.to_pandas()
        return pd.DataFrame(data)

    def collect(self) -> List[Row]:
        pdf = self.toPandas()
        cols = list(pdf.columns)
        out = []
        for vals in zip(*[pdf[c].tolist() for c in cols]) if cols else []:
            out.append(Row(**dict(zip(cols, [_py(v) for v in vals]))))
        return out

    def first(self) -> Optional[Row]:
        rows = self.limit(1).collect()
        return rows[0] if rows else None

    def head(self, n: int = 1) -> List[Row]:
        return self.limit(n).collect()

    take = head

    def show(self, n: int = 20, truncate: bool = True) -> None:
        print(self.limit(n).toPandas())

    def __repr__(self) -> str:
        return "DataFrame[%s] (%d partitions)" % (
            ", ".join("%s: %s" % (n, t) for n, t in self.dtypes),
            len(self._parts),
        )


def _needs_object(v: List[Any]) -> bool:
    return any(isinstance(x, (list, tuple, np.ndarray)) or hasattr(x, "toArray") for x in v[:5])


def _py(v: Any) -> Any:
    if isinstance(v, np.ndarray):
        return v.tolist()
    if isinstance(v, np.generic):
        return v.item()
    return v


def _rename(p: pa.Table, names: List[str]) -> pa.Table:
    fields = [f.with_name(n) for f, n in zip(p.schema, names)]
    return pa.Table.from_arrays(p.columns, schema=pa.schema(fields))


def _simple_type(t: pa.DataType) -> str:
    m = {
        pa.float32(): "float", pa.float64(): "double", pa.int32(): "int", pa.int64(): "bigint",
        pa.int16(): "smallint", pa.int8(): "tinyint", pa.string(): "string", pa.bool_(): "boolean",
    }
    return m.get(t, str(t))


def _vectors_from_arrow(col: Union[pa.ChunkedArray, pa.Array]) -> List[Any]:
    arr = _combine(col)
    out: List[Any] = []
    for d in arr.to_pylist():
        if d is None:
            out.append(None)
        elif d["type"] == 1:
            out.append(Vectors.dense(d["values"]))
        else:
            out.append(Vectors.sparse(d["size"], d["indices"], d["values"]))
    return out


def as_dataframe(dataset: Any, num_partitions: Optional[int] = None) -> Tuple[DataFrame, str]:
    """Normalise user input -> (DataFrame, kind) where kind in {'srml', 'pandas'}."""
    if isinstance(dataset, DataFrame):
        return dataset, "srml"
    if isinstance(dataset, pd.DataFrame):
        return DataFrame.from_pandas(dataset, num_partitions or 1), "pandas"
    if isinstance(dataset, pa.Table):
        return DataFrame.from_arrow(dataset, num_partitions or 1), "arrow"
    raise TypeError("Unsupported dataset type %s" % type(dataset))


def restore_kind(df: DataFrame, kind: str) -> Any:
    if kind == "pandas":
        return df.toPandas()
    if kind == "arrow":
        return df._concat()
    return df
