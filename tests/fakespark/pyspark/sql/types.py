class DataType:
    def __repr__(self):
        return type(self).__name__ + "()"


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


class ArrayType(DataType):
    def __init__(self, elementType, containsNull=True):
        self.elementType = elementType


class StructField:
    def __init__(self, name, dataType, nullable=True):
        self.name, self.dataType, self.nullable = name, dataType, nullable


class StructType(DataType):
    def __init__(self, fields=None):
        self.fields = list(fields or [])

    @property
    def names(self):
        return [f.name for f in self.fields]
