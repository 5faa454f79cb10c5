"""A few pyspark shared-param mixins (with Spark's defaults) so the library's shared-mixin switch
is exercised; names absent here fall back to the library's own mixins."""
from spark_rapids_ml_nai_amd.core._params_builtin import Param, Params, TypeConverters


class HasFeaturesCol(Params):
    featuresCol = Param(Params._dummy(), "featuresCol", "features column name.", typeConverter=TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(featuresCol="features")

    def getFeaturesCol(self):
        return self.getOrDefault(self.featuresCol)


class HasLabelCol(Params):
    labelCol = Param(Params._dummy(), "labelCol", "label column name.", typeConverter=TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(labelCol="label")

    def getLabelCol(self):
        return self.getOrDefault(self.labelCol)


class HasPredictionCol(Params):
    predictionCol = Param(Params._dummy(), "predictionCol", "prediction column name.",
                          typeConverter=TypeConverters.toString)

    def __init__(self):
        super().__init__()
        self._setDefault(predictionCol="prediction")

    def getPredictionCol(self):
        return self.getOrDefault(self.predictionCol)
