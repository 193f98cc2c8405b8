"""scikit-learn compatible wrappers of every H2O estimator (reference ``h2o-py/h2o/sklearn``).

For each estimator class ``H2OXxxEstimator`` of :mod:`h2o.estimators` (and :mod:`h2o.automl`) this module exposes
``H2OXxxEstimator`` (generic), ``H2OXxxClassifier`` and ``H2OXxxRegressor`` (supervised algorithms), and for the
munging transforms of :mod:`h2o.transforms` a transformer class. They follow the sklearn protocol —
``fit`` / ``predict`` / ``predict_proba`` / ``predict_log_proba`` / ``score`` / ``transform`` /
``fit_transform``, ``get_params`` / ``set_params`` over every parameter of the algorithm — and accept lists, numpy
arrays, pandas DataFrames or H2OFrames, returning numpy for numpy / pandas / list inputs and H2OFrames for
H2OFrame inputs, so they compose with ``sklearn.pipeline.Pipeline``, ``clone`` and the model-selection tools.
The engine runs in-process (no connection to manage); ``h2o_connection`` is kept as a no-op context manager.
"""
from __future__ import annotations

import contextlib
import inspect
import sys

import numpy as np
from sklearn.base import BaseEstimator, ClassifierMixin, RegressorMixin, TransformerMixin

from .. import automl as _automl
from .. import estimators as _estimators
from .. import transforms as _transforms

_module = sys.modules[__name__]

# estimators whose `predict` returns every column (transform-like), as the reference's `predictions_col='all'`
_ALL_COLUMNS = {"H2OAutoEncoderEstimator", "H2OGeneralizedLowRankEstimator", "H2OPrincipalComponentAnalysisEstimator",
                "H2OSingularValueDecompositionEstimator", "H2OTargetEncoderEstimator"}
_NO_PROBA = {"H2OAutoEncoderEstimator", "H2OExtendedIsolationForestEstimator", "H2OGeneralizedLowRankEstimator",
             "H2OIsolationForestEstimator", "H2OKMeansEstimator", "H2OPrincipalComponentAnalysisEstimator",
             "H2OSingularValueDecompositionEstimator", "H2OTargetEncoderEstimator", "H2OWord2vecEstimator",
             "H2OAggregatorEstimator", "H2OGenericEstimator", "H2OCoxProportionalHazardsEstimator"}
_TRANSFORMS = {"H2OAutoEncoderEstimator", "H2OGeneralizedLowRankEstimator", "H2OPrincipalComponentAnalysisEstimator",
               "H2OSingularValueDecompositionEstimator", "H2OTargetEncoderEstimator", "H2OAggregatorEstimator"}
_EXCLUDED = {"H2OEstimator", "H2OTransformer", "H2OInfogram", "H2OANOVAGLMEstimator", "H2OModelSelectionEstimator",
             "H2OIsotonicRegressionEstimator"}
_GENERIC_ONLY = {"H2OAggregatorEstimator", "H2OAutoEncoderEstimator", "H2OExtendedIsolationForestEstimator",
                 "H2OGeneralizedLowRankEstimator", "H2OGenericEstimator", "H2OIsolationForestEstimator",
                 "H2OKMeansEstimator", "H2OPrincipalComponentAnalysisEstimator",
                 "H2OSingularValueDecompositionEstimator", "H2OTargetEncoderEstimator", "H2OWord2vecEstimator"}
_CLASSIFIER_ONLY = {"H2ONaiveBayesEstimator", "H2OSupportVectorMachineEstimator"}
_REGRESSOR_ONLY = {"H2OCoxProportionalHazardsEstimator"}


def _frame_of(X, names=None):
    """(H2OFrame, input kind) of lists / numpy / pandas / H2OFrame input."""
    from .. import H2OFrame
    if isinstance(X, H2OFrame):
        return X, "h2o"
    try:
        import pandas as pd
        if isinstance(X, pd.DataFrame):
            return H2OFrame(X), "pandas"
        if isinstance(X, pd.Series):
            return H2OFrame(X.to_frame()), "pandas"
    except ImportError:                      # pragma: no cover - pandas is installed with the image
        pass
    a = np.asarray(X)
    if a.ndim == 1:
        a = a[:, None]
    cols = names or [f"C{i + 1}" for i in range(a.shape[1])]
    import pandas as pd
    return H2OFrame(pd.DataFrame(a, columns=cols)), "numpy"


def _as_class(v, classes):
    """A predicted factor level (a string) -> the matching original class value."""
    for c in classes:
        if str(c) == str(v):
            return c
        try:
            if float(c) == float(v):
                return c
        except (TypeError, ValueError):
            pass
    return v


def _out(fr, kind):
    if kind == "h2o":
        return fr
    arr = fr.as_data_frame().to_numpy()
    return arr[:, 0] if arr.shape[1] == 1 else arr


class _Base(BaseEstimator):
    """Common machinery of the generated wrappers; ``_cls`` is the wrapped H2O estimator class."""

    _cls = None
    _kind = "estimator"

    def __init__(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
        self._set = dict(params)

    # every parameter of the algorithm is a sklearn parameter (defaults from the algorithm's schema)
    @classmethod
    def _param_names(cls):
        from ..estimators._schema import PARAMS
        algo = getattr(cls._cls, "algo", None)
        names = list((PARAMS.get(algo) or {}).keys()) if algo else []
        return [n for n in names if n not in ("training_frame", "validation_frame", "response_column",
                                               "ignored_columns", "model_id")]

    def get_params(self, deep=True):
        from ..estimators._schema import PARAMS
        algo = getattr(self._cls, "algo", None)
        defaults = PARAMS.get(algo) or {}
        out = {}
        for n in self._param_names():
            d = defaults.get(n)
            out[n] = getattr(self, n, d.get("default") if isinstance(d, dict) else d)
        out.update({k: getattr(self, k) for k in getattr(self, "_set", {})})
        return out

    def set_params(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
            self._set[k] = v
        return self

    def _estimator(self):
        kw = {k: v for k, v in getattr(self, "_set", {}).items()}
        return self._cls(**kw)

    def fit(self, X, y=None, **fit_params):
        fr, _ = _frame_of(X)
        self.feature_names_in_ = list(fr.names)
        self.n_features_in_ = len(fr.names)
        est = self._estimator()
        resp = None
        if y is not None:
            yf, _ = _frame_of(y, ["target"]) if not hasattr(y, "names") else (y, "h2o")
            resp = yf.names[0]
            if resp in fr.names:
                resp = resp + "_target"
                yf.set_names([resp])
            if self._kind == "classifier":
                yv = np.asarray(y) if not hasattr(y, "names") else np.asarray(yf.as_data_frame().iloc[:, 0])
                self.classes_ = np.unique(yv.reshape(-1))
                yf = yf.asfactor()
            fr = fr.cbind(yf)
        if y is None or self._cls.__name__ in _TRANSFORMS and not getattr(self._cls, "supervised_learning", True):
            est.train(x=self.feature_names_in_, training_frame=fr)
        else:
            est.train(x=self.feature_names_in_, y=resp, training_frame=fr)
        self.estimator_ = est
        return self

    def _predict_frame(self, X):
        fr, kind = _frame_of(X, getattr(self, "feature_names_in_", None))
        return self.estimator_.predict(fr), kind

    def predict(self, X):
        p, kind = self._predict_frame(X)
        if self._cls.__name__ in _ALL_COLUMNS:
            return _out(p, kind)
        col = p[:, 0] if p.ncols > 1 else p
        out = _out(col, kind)
        if kind != "h2o" and self._kind == "classifier" and hasattr(self, "classes_"):
            out = np.asarray([_as_class(v, self.classes_) for v in out])
        return out


class _Proba:
    def predict_proba(self, X):
        p, kind = self._predict_frame(X)
        if p.ncols < 2:
            raise AttributeError("predict_proba is only available for classification models")
        return _out(p[:, 1:], kind)

    def predict_log_proba(self, X):
        return np.log(self.predict_proba(X))


class _Transform:
    def transform(self, X):
        p, kind = self._predict_frame(X)
        return _out(p, kind)

    def fit_transform(self, X, y=None, **fit_params):
        return self.fit(X, y, **fit_params).transform(X)


def _make(cls, suffix, kind):
    base = cls.__name__.replace("Estimator", "")
    name = base + suffix
    mixins = []
    if kind in ("estimator", "classifier") and cls.__name__ not in _NO_PROBA:
        mixins.append(_Proba)
    if kind in ("estimator", "transformer") and cls.__name__ in _TRANSFORMS:
        mixins.append(_Transform)
    if kind == "classifier":
        mixins.append(ClassifierMixin)
    elif kind == "regressor":
        mixins.append(RegressorMixin)
    if kind == "estimator" and cls.__name__ in _CLASSIFIER_ONLY:
        kind = "classifier"
    return type(name, tuple(mixins) + (_Base,), dict(_cls=cls, _kind=kind, __module__=__name__,
                                                     __doc__=f"sklearn wrapper of :class:`{cls.__name__}`."))


class _TransformerWrapper(TransformerMixin, BaseEstimator):
    """sklearn wrapper of an h2o.transforms transformer (fit / transform on H2OFrames or array-likes)."""

    _cls = None

    def __init__(self, **params):
        for k, v in params.items():
            setattr(self, k, v)
        self._set = dict(params)

    def get_params(self, deep=True):
        return dict(self._set)

    def set_params(self, **params):
        self._set.update(params)
        for k, v in params.items():
            setattr(self, k, v)
        return self

    def fit(self, X, y=None, **fit_params):
        fr, _ = _frame_of(X)
        self.transformer_ = self._cls(**self._set).fit(fr)
        return self

    def transform(self, X):
        fr, kind = _frame_of(X)
        return _out(self.transformer_.transform(fr), kind)


_generated = []
for _mod in (_automl, _estimators):
    for _n, _c in inspect.getmembers(_mod, inspect.isclass):
        if not _n.startswith("H2O") or _n in _EXCLUDED or not hasattr(_c, "train"):
            continue
        _generated.append(_make(_c, "Estimator", "estimator"))
        if _n not in _GENERIC_ONLY and getattr(_c, "supervised_learning", True):
            if _n not in _REGRESSOR_ONLY:
                _generated.append(_make(_c, "Classifier", "classifier"))
            if _n not in _CLASSIFIER_ONLY:
                _generated.append(_make(_c, "Regressor", "regressor"))
for _n, _c in inspect.getmembers(_transforms, inspect.isclass):
    if _n in _EXCLUDED or not _n.startswith("H2O"):
        continue
    _generated.append(type(_n, (_TransformerWrapper,), dict(_cls=_c, __module__=__name__)))

for _g in _generated:
    setattr(_module, _g.__name__, _g)


@contextlib.contextmanager
def h2o_connection(**init_args):
    """The reference opens / closes a backend connection around sklearn calls; the engine here is in-process."""
    yield


__all__ = sorted(["h2o_connection"] + [g.__name__ for g in _generated])
