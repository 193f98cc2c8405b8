"""Estimator classes with the h2o-py names (reference: ``h2o-py/h2o/estimators/*.py``)."""
from .estimator_base import H2OEstimator, make_estimator

H2OGradientBoostingEstimator = make_estimator("H2OGradientBoostingEstimator", "gbm")
H2ORandomForestEstimator = make_estimator("H2ORandomForestEstimator", "drf")
H2OXGBoostEstimator = make_estimator("H2OXGBoostEstimator", "xgboost")
H2OIsolationForestEstimator = make_estimator("H2OIsolationForestEstimator", "isolationforest", supervised=False)
H2OExtendedIsolationForestEstimator = make_estimator("H2OExtendedIsolationForestEstimator", "extendedisolationforest",
                                                     supervised=False)
H2OGeneralizedLinearEstimator = make_estimator("H2OGeneralizedLinearEstimator", "glm", aliases={"Lambda": "lambda_",
                                                                                               "lambda": "lambda_"})
H2OKMeansEstimator = make_estimator("H2OKMeansEstimator", "kmeans", supervised=False)
H2ODeepLearningEstimator = make_estimator("H2ODeepLearningEstimator", "deeplearning")


class H2OAutoEncoderEstimator(H2ODeepLearningEstimator):
    supervised_learning = False

    def __init__(self, model_id=None, **kw):
        kw["autoencoder"] = True
        super().__init__(model_id, **kw)


def _extra():
    g = globals()
    for cls_name, algo, sup in (
            ("H2OPrincipalComponentAnalysisEstimator", "pca", False),
            ("H2OSingularValueDecompositionEstimator", "svd", False),
            ("H2OGeneralizedLowRankEstimator", "glrm", False),
            ("H2ONaiveBayesEstimator", "naivebayes", True),
            ("H2OWord2vecEstimator", "word2vec", False),
            ("H2OCoxProportionalHazardsEstimator", "coxph", True),
            ("H2OIsotonicRegressionEstimator", "isotonicregression", True),
            ("H2OAggregatorEstimator", "aggregator", False),
            ("H2OSupportVectorMachineEstimator", "psvm", True),
            ("H2ORuleFitEstimator", "rulefit", True),
            ("H2OStackedEnsembleEstimator", "stackedensemble", True),
            ("H2OTargetEncoderEstimator", "targetencoder", True),
            ("H2OGenericEstimator", "generic", False),
            ("H2OGeneralizedAdditiveEstimator", "gam", True),
            ("H2OANOVAGLMEstimator", "anovaglm", True),
            ("H2OModelSelectionEstimator", "modelselection", True),
            ("H2OUpliftRandomForestEstimator", "upliftdrf", True),
            ("H2ODecisionTreeEstimator", "dt", True),
            ("H2OInfogram", "infogram", True),
            ("H2OGrepEstimator", "grep", False)):
        if cls_name not in g:
            g[cls_name] = make_estimator(cls_name, algo, sup)


_extra()

__all__ = [n for n in list(globals()) if n.startswith("H2O")]
