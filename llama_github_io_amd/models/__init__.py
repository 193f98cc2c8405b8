"""Algorithm registry: every estimator of the reference (``h2o-algos``, extensions) maps to a trainer
here (``builder.REGISTRY``). Import cost is kept low: trainers are imported on first registration."""
from __future__ import annotations

from . import builder as _b


def _register_all():
    from .gbm import GBM_DEFAULTS, GBMTrainer
    from .drf import DRFTrainer
    from .xgboost import XGBoostTrainer
    from .isoforest import ExtendedIsolationForestTrainer, IsolationForestTrainer
    from .glm import GLMTrainer
    from .kmeans import KMeansTrainer
    from .deeplearning import DeepLearningTrainer
    _b.register("gbm", GBMTrainer)
    _b.register("drf", DRFTrainer)
    _b.register("xgboost", XGBoostTrainer)
    _b.register("isolationforest", IsolationForestTrainer, supervised=False, needs_response_optional=True)
    _b.register("extendedisolationforest", ExtendedIsolationForestTrainer, supervised=False)
    _b.register("glm", GLMTrainer)
    _b.register("kmeans", KMeansTrainer, supervised=False)
    _b.register("deeplearning", DeepLearningTrainer, needs_response_optional=True)
    try:
        from . import extra  # noqa: F401  (remaining algorithms register themselves)
    except ImportError:
        pass


_register_all()
REGISTRY = _b.REGISTRY
