from spark_rapids_ml_nai_amd.core._params_builtin import Params


class Estimator(Params):
    def fit(self, dataset, params=None):
        if params is None:
            return self._fit(dataset)
        return self.copy(params)._fit(dataset)

    def _fit(self, dataset):
        raise NotImplementedError


class Transformer(Params):
    def transform(self, dataset, params=None):
        return (self.copy(params) if params else self)._transform(dataset)

    def _transform(self, dataset):
        raise NotImplementedError


class Model(Transformer):
    pass


class Pipeline(Estimator):
    """stages fitted in order (isinstance checks as pyspark.ml.Pipeline does)."""

    def __init__(self, stages):
        super().__init__()
        self.stages = list(stages)

    def _fit(self, dataset):
        fitted = []
        for st in self.stages:
            if isinstance(st, Estimator):
                m = st.fit(dataset)
                fitted.append(m)
                dataset = m.transform(dataset)
            elif isinstance(st, Transformer):
                fitted.append(st)
                dataset = st.transform(dataset)
            else:
                raise TypeError("Cannot recognize a pipeline stage of type %s." % type(st))
        return PipelineModel(fitted)


class PipelineModel(Model):
    def __init__(self, stages):
        super().__init__()
        self.stages = stages

    def _transform(self, dataset):
        for st in self.stages:
            dataset = st.transform(dataset)
        return dataset
