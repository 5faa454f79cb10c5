from .dataframe import DataFrame, SparkSession  # noqa: F401
