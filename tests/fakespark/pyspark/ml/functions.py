"""``pyspark.ml.functions.array_to_vector`` / ``vector_to_array`` over the fake Column model."""
import numpy as np
import pyarrow as pa

from ..sql.functions import Column, _c


def array_to_vector(c):
    cc = _c(c)

    def run(t, pid):
        from spark_rapids_ml_nai_amd.core.dataframe import dense_to_vector_array

        a = cc.eval(t, pid)
        m = len(a)
        flat = np.asarray(pa.compute.list_flatten(a).to_numpy(zero_copy_only=False), dtype=np.float64)
        return dense_to_vector_array(flat.reshape(m, -1) if m else np.zeros((0, 0)))

    out = Column(cc.name, fn=run)
    out._field = lambda name: __import__("spark_rapids_ml_nai_amd.core.dataframe",
                                         fromlist=["vector_field"]).vector_field(name)
    return out


def vector_to_array(c, dtype="float64"):
    cc = _c(c)

    def run(t, pid):
        a = cc.eval(t, pid)
        vals = pa.compute.struct_field(a, "values")
        return vals.cast(pa.list_(pa.float32() if dtype == "float32" else pa.float64()))

    return Column(cc.name, fn=run)
