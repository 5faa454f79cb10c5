"""Column expressions of the fake DataFrame: the slice of ``pyspark.sql.functions`` the library's
Spark paths use, evaluated per partition on Arrow tables (``Column.eval(table, pid)``)."""
from typing import Any, Callable, List, Optional

import numpy as np
import pyarrow as pa
import pyarrow.compute as pc


class Column:
    def __init__(self, name: Optional[str], op: Optional[str] = None, fn: Optional[Callable] = None,
                 explode: bool = False):
        self.name, self.op, self._fn, self.explode = name, op, fn, explode

    # evaluation ----------------------------------------------------------------------
    def eval(self, t: pa.Table, pid: int = 0) -> Any:
        if self._fn is not None:
            return self._fn(t, pid)
        if self.name in t.schema.names:
            return t.column(self.name).combine_chunks()
        if self.name and "." in self.name:  # struct field access "a.b"
            base, field = self.name.split(".", 1)
            arr = t.column(base).combine_chunks()
            return pc.struct_field(arr, field)
        raise KeyError("column %r not in %s" % (self.name, t.schema.names))

    def alias(self, name: str) -> "Column":
        return Column(name, self.op, self._fn or (lambda t, pid, c=self: c.eval(t, pid)), self.explode)

    def __getitem__(self, field: str) -> "Column":
        return Column("%s.%s" % (self.name, field), fn=lambda t, pid: pc.struct_field(self.eval(t, pid), field))

    # operators -----------------------------------------------------------------------
    def _bin(self, other: Any, f: Callable) -> "Column":
        def run(t, pid):
            a = self.eval(t, pid)
            b = other.eval(t, pid) if isinstance(other, Column) else other
            return f(a, b)

        return Column(self.name, fn=run)

    def __ge__(self, o): return self._bin(o, pc.greater_equal)  # noqa: E704
    def __gt__(self, o): return self._bin(o, pc.greater)  # noqa: E704
    def __le__(self, o): return self._bin(o, pc.less_equal)  # noqa: E704
    def __lt__(self, o): return self._bin(o, pc.less)  # noqa: E704
    def __eq__(self, o): return self._bin(o, pc.equal)  # type: ignore[override]  # noqa: E704
    def __ne__(self, o): return self._bin(o, pc.not_equal)  # type: ignore[override]  # noqa: E704
    def __and__(self, o): return self._bin(o, pc.and_)  # noqa: E704
    def __or__(self, o): return self._bin(o, pc.or_)  # noqa: E704

    def __invert__(self) -> "Column":
        return Column(self.name, fn=lambda t, pid: pc.invert(self.eval(t, pid)))

    def __hash__(self) -> int:
        return id(self)


def _c(x: Any) -> Column:
    return x if isinstance(x, Column) else Column(x)


def col(name: str) -> Column:
    return Column(name)


def lit(v: Any) -> Column:
    return Column("lit", fn=lambda t, pid: pa.array([v] * t.num_rows))


def unwrap_udt(c: Any) -> Column:
    return Column(_c(c).name, "unwrap_udt")


def monotonically_increasing_id() -> Column:
    # Spark: partition id in the upper 31 bits, record number within the partition in the lower 33
    return Column("monotonically_increasing_id()",
                  fn=lambda t, pid: pa.array((np.int64(pid) << 33) + np.arange(t.num_rows, dtype=np.int64)))


def rand(seed: Optional[int] = None) -> Column:
    def run(t, pid):
        return pa.array(np.random.default_rng((0 if seed is None else seed) * 7919 + pid).random(t.num_rows))

    return Column("rand", fn=run)


def struct(*cols: Any) -> Column:
    if len(cols) == 1 and isinstance(cols[0], (list, tuple)):
        cols = tuple(cols[0])
    cs = [_c(c) for c in cols]

    def run(t, pid):
        return pa.StructArray.from_arrays([c.eval(t, pid) for c in cs], names=[c.name for c in cs])

    return Column("struct", fn=run)


def arrays_zip(*cols: Any) -> Column:
    cs = [_c(c) for c in cols]

    def run(t, pid):
        arrs = [c.eval(t, pid) for c in cs]
        offsets = arrs[0].offsets
        flat = [pc.list_flatten(a) for a in arrs]
        return pa.ListArray.from_arrays(offsets, pa.StructArray.from_arrays(flat, names=[c.name for c in cs]))

    return Column("arrays_zip", fn=run)


def explode(c: Any) -> Column:
    cc = _c(c)
    return Column("col", fn=lambda t, pid: cc.eval(t, pid), explode=True)


def __getattr__(name: str) -> Any:  # anything else is outside the modelled slice
    raise AttributeError("fake pyspark.sql.functions has no %r" % name)


__all__: List[str] = ["Column", "col", "lit", "unwrap_udt", "monotonically_increasing_id", "rand", "struct",
                      "arrays_zip", "explode"]


def pandas_udf(f=None, returnType=None, functionType=None):
    """Scalar-iterator pandas UDF over one struct column (the only shape the library uses)."""
    def make(*cols):
        arg = _c(cols[0])

        def run(t, pid):
            import pandas as pd

            from .types import to_arrow_type

            a = arg.eval(t, pid)
            pdf = pa.Table.from_arrays(a.flatten(), names=[fl.name for fl in a.type]).to_pandas()
            outs = list(f(iter([pdf])))
            out = pd.concat(outs) if outs else pd.DataFrame()
            arrays = [pa.array(list(out[fl.name]) if len(out) else [], type=to_arrow_type(fl.dataType))
                      for fl in returnType.fields]
            return pa.StructArray.from_arrays(arrays, names=returnType.names)

        return Column("pandas_udf", fn=run)

    return make
