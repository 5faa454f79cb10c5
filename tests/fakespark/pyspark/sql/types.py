import pyarrow as pa


class DataType:
    def __repr__(self):
        return type(self).__name__ + "()"

    def __eq__(self, other):
        return type(self) is type(other) and vars(self) == vars(other)

    def __hash__(self):
        return hash(type(self).__name__)


class DoubleType(DataType):
    pass


class FloatType(DataType):
    pass


class LongType(DataType):
    pass


class IntegerType(DataType):
    pass


class BinaryType(DataType):
    pass


class StringType(DataType):
    pass


class ArrayType(DataType):
    def __init__(self, elementType, containsNull=True):
        self.elementType = elementType

    def __repr__(self):
        return "ArrayType(%r)" % (self.elementType,)


class StructField:
    def __init__(self, name, dataType, nullable=True):
        self.name, self.dataType, self.nullable = name, dataType, nullable

    def __repr__(self):
        return "StructField(%r, %r)" % (self.name, self.dataType)


class StructType(DataType):
    def __init__(self, fields=None):
        self.fields = list(fields or [])

    @property
    def names(self):
        return [f.name for f in self.fields]

    def __getitem__(self, name):
        for f in self.fields:
            if f.name == name:
                return f
        raise KeyError(name)

    def add(self, name, dataType, nullable=True):
        self.fields.append(StructField(name, dataType, nullable))
        return self


def to_arrow_type(t):
    from ..ml.linalg import VectorUDT

    if isinstance(t, VectorUDT):
        from spark_rapids_ml_nai_amd.core.dataframe import VECTOR_STRUCT

        return VECTOR_STRUCT
    if isinstance(t, DoubleType):
        return pa.float64()
    if isinstance(t, FloatType):
        return pa.float32()
    if isinstance(t, LongType):
        return pa.int64()
    if isinstance(t, IntegerType):
        return pa.int32()
    if isinstance(t, BinaryType):
        return pa.binary()
    if isinstance(t, StringType):
        return pa.string()
    if isinstance(t, ArrayType):
        return pa.list_(to_arrow_type(t.elementType))
    if isinstance(t, StructType):
        return pa.struct([pa.field(f.name, to_arrow_type(f.dataType)) for f in t.fields])
    raise TypeError("no Arrow type for %r" % (t,))
