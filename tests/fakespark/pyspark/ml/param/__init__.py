from spark_rapids_ml_nai_amd.core._params_builtin import Param, Params, TypeConverters  # noqa: F401
