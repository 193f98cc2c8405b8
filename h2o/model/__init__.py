"""``h2o.model`` (reference: h2o-py/h2o/model): the model base class and the metrics / confusion-matrix
types the client returns (every metrics family is the engine's ModelMetrics)."""
from llama_github_io_amd.metrics import ConfusionMatrix, ModelMetrics

from ..estimators.estimator_base import H2OEstimator as ModelBase

MetricsBase = ModelMetrics
H2OBinomialModelMetrics = H2OMultinomialModelMetrics = H2ORegressionModelMetrics = ModelMetrics
H2OClusteringModelMetrics = H2OOrdinalModelMetrics = H2OAnomalyDetectionModelMetrics = ModelMetrics
H2ODimReductionModelMetrics = H2OCoxPHModelMetrics = H2OBinomialUpliftModelMetrics = ModelMetrics

__all__ = ["ModelBase", "MetricsBase", "ConfusionMatrix", "H2OBinomialModelMetrics", "H2OMultinomialModelMetrics",
           "H2ORegressionModelMetrics", "H2OClusteringModelMetrics", "H2OOrdinalModelMetrics",
           "H2OAnomalyDetectionModelMetrics", "H2ODimReductionModelMetrics", "H2OCoxPHModelMetrics",
           "H2OBinomialUpliftModelMetrics"]
