"""Registration of the remaining algorithms (each lives in its own module)."""
from __future__ import annotations

import importlib

from . import builder as _b

_ALGOS = [
    # name, module, trainer class, supervised, extra kwargs
    ("stackedensemble", "stackedensemble", "StackedEnsembleTrainer", True, {}),
    ("pca", "pca", "PCATrainer", False, {}),
    ("svd", "pca", "SVDTrainer", False, {}),
    ("glrm", "glrm", "GLRMTrainer", False, {}),
    ("naivebayes", "naivebayes", "NaiveBayesTrainer", True, dict(classification_only=True)),
    ("word2vec", "word2vec", "Word2VecTrainer", False, {}),
    ("coxph", "coxph", "CoxPHTrainer", True, {}),
    ("isotonicregression", "isotonic", "IsotonicTrainer", True, {}),
    ("aggregator", "aggregator", "AggregatorTrainer", False, {}),
    ("psvm", "psvm", "PSVMTrainer", True, dict(classification_only=True)),
    ("rulefit", "rulefit", "RuleFitTrainer", True, {}),
    ("targetencoder", "targetencoder", "TargetEncoderTrainer", True, {}),
    ("generic", "generic", "GenericTrainer", False, {}),
    ("gam", "gam", "GAMTrainer", True, {}),
    ("anovaglm", "anovaglm", "ANOVAGLMTrainer", True, {}),
    ("modelselection", "modelselection", "ModelSelectionTrainer", True, {}),
    ("upliftdrf", "uplift", "UpliftDRFTrainer", True, dict(classification_only=True)),
    ("dt", "dt", "DTTrainer", True, dict(classification_only=True)),
    ("infogram", "infogram", "InfogramTrainer", True, {}),
    ("quantile", "quantile", "QuantileTrainer", False, {}),
    ("grep", "grep", "GrepTrainer", False, {}),
]

for name, mod, cls, sup, kw in _ALGOS:
    try:
        m = importlib.import_module(f".{mod}", __package__)
    except ModuleNotFoundError as e:
        if e.name and e.name.endswith(mod):
            continue
        raise
    _b.register(name, getattr(m, cls), supervised=sup, **kw)
