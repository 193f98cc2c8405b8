"""``H2OEstimator`` (reference: ``h2o-py/h2o/estimators/estimator_base.py``): holds parameters,
``train()`` runs the ModelBuilder (as a Job), and after training delegates every model accessor
(``predict``, ``model_performance``, ``auc``, ``varimp``, ``coef``, ``download_mojo``...) to the
trained model object."""
from __future__ import annotations

from llama_github_io_amd.core.job import Job
from llama_github_io_amd.models import builder

from ..model_api import ModelBaseAPI

_OWN = {"algo", "_parms", "_model", "model_id", "_job", "supervised_learning"}


class H2OEstimator(ModelBaseAPI):
    algo: str = ""
    supervised_learning = True
    _param_aliases: dict = {}

    def __init__(self, model_id=None, **kwargs):
        object.__setattr__(self, "_parms", {})
        object.__setattr__(self, "_model", None)
        object.__setattr__(self, "_job", None)
        object.__setattr__(self, "model_id", model_id)
        from ._schema import PARAMS
        known = PARAMS.get(self.algo)
        for k, v in kwargs.items():
            kk = self._param_aliases.get(k, k)
            if known is not None and k not in known and kk not in known and not k.startswith("_") and \
                    k not in ("segment_columns", "segment_models_id"):
                # the reference estimators have explicit signatures: an unknown keyword is a TypeError
                from llama_github_io_amd.models import builder as _b
                if self.algo not in _b.REGISTRY or kk not in _b.extension_params(self.algo):
                    raise TypeError(f"{type(self).__name__}.__init__() got an unexpected keyword argument '{k}'")
            self._parms[kk] = v

    # ---- parameter access like h2o-py properties
    def __setattr__(self, k, v):
        if k in _OWN or k.startswith("_"):
            object.__setattr__(self, k, v)
        else:
            self._parms[self._param_aliases.get(k, k)] = v

    def __getattr__(self, k):
        if k.startswith("__"):
            raise AttributeError(k)
        m = object.__getattribute__(self, "_model")
        if m is not None and hasattr(m, k):
            return getattr(m, k)
        parms = object.__getattribute__(self, "_parms")
        if k in parms:
            return parms[k]
        spec = builder.REGISTRY.get(object.__getattribute__(self, "algo"))
        if spec is not None and k in spec.defaults:
            return spec.defaults[k]
        raise AttributeError(k)

    def set_params(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)
        return self

    def get_params(self, deep=True):
        return dict(self._parms)

    @property
    def params(self):
        if self._model is None:
            return {}
        return {k: {"default": None, "actual": v} for k, v in self._model.params.items()}

    @property
    def actual_params(self):
        return dict(self._model.params) if self._model is not None else {}

    # ---- training
    def train(self, x=None, y=None, training_frame=None, offset_column=None, fold_column=None, weights_column=None,
              validation_frame=None, max_runtime_secs=None, ignored_columns=None, model_id=None, verbose=False):
        p = dict(self._parms)
        for k, v in (("offset_column", offset_column), ("fold_column", fold_column), ("weights_column", weights_column),
                     ("max_runtime_secs", max_runtime_secs), ("ignored_columns", ignored_columns)):
            if v is not None:
                p[k] = v
        if y is None and "response_column" in p:
            y = p.pop("response_column")
        if not self.supervised_learning and y is not None and self.algo not in ("isolationforest", "deeplearning"):
            y = None
        mid = model_id or self.model_id or p.pop("model_id", None)
        job = Job(f"{self.algo} training", dest=mid)
        self._job = job
        m = job.run_sync(builder.train, self.algo, p, x, y, training_frame, validation_frame, job, mid)
        self._model = m
        self.model_id = m.key
        return self

    def train_segments(self, x=None, y=None, training_frame=None, offset_column=None, weights_column=None,
                       validation_frame=None, max_runtime_secs=None, segments=None, segment_models_id=None,
                       parallelism=1, verbose=False):
        """One model per segment (``hex/segments/SegmentModelsBuilder.java``); the segment columns come from
        the ``segment_columns`` parameter. Returns an ``H2OSegmentModels``-like object (``as_frame()``)."""
        from llama_github_io_amd.segments import train_segments
        p = dict(self._parms)
        seg_cols = p.pop("segment_columns", None)
        if not seg_cols:
            raise ValueError("set segment_columns on the estimator before train_segments()")
        for k, v in (("offset_column", offset_column), ("weights_column", weights_column),
                     ("max_runtime_secs", max_runtime_secs)):
            if v is not None:
                p[k] = v
        return train_segments(self.algo, p, x, y, training_frame, seg_cols, segments, validation_frame, parallelism,
                              segment_models_id)

    def start(self, x=None, y=None, training_frame=None, offset_column=None, fold_column=None, weights_column=None,
              validation_frame=None, **params):
        """Non-blocking train in h2o-py; here training is synchronous and ``join()`` returns at once."""
        for k, v in params.items():
            setattr(self, k, v)
        return self.train(x=x, y=y, training_frame=training_frame, offset_column=offset_column, fold_column=fold_column,
                          weights_column=weights_column, validation_frame=validation_frame)

    def weights(self, matrix_id=0):
        m = self._m()
        if not hasattr(m, "weights"):
            raise ValueError(f"{self.algo} models have no weight matrices")
        W = m.weights(matrix_id)
        if not hasattr(W, "nrows"):            # h2o-py returns the matrix as a frame [units, inputs]
            import torch
            from llama_github_io_amd.frame import H2OFrame
            W = torch.as_tensor(W, dtype=torch.float64)
            W = H2OFrame.from_tensor(W, [f"C{i + 1}" for i in range(W.shape[1])])
        return W

    def fit(self, X, y=None, **kw):  # scikit-learn style
        return self.train(x=None, y=y, training_frame=X, **kw)

    # ---- explicit delegation for the common API (clear errors before training)
    def _m(self):
        if self._model is None:
            raise ValueError("model not trained yet: call train() first")
        return self._model

    def predict(self, test_data, **kw):
        return self._m().predict(test_data, **kw) if kw else self._m().predict(test_data)

    def model_performance(self, test_data=None, train=False, valid=False, xval=False):
        return self._m().model_performance(test_data, train, valid, xval)

    def download_mojo(self, path=".", get_genmodel_jar=False, genmodel_name="", filename=None):
        from llama_github_io_amd.mojo import writer
        return writer.download_mojo(self._m(), path, filename)

    save_mojo = download_mojo

    def download_pojo(self, path="", get_genmodel_jar=False, genmodel_name=""):
        from llama_github_io_amd.mojo import pojo
        return pojo.download_pojo(self._m(), path, get_genmodel_jar, genmodel_name)

    def download_model(self, path=""):
        from llama_github_io_amd import persist
        return persist.save_model(self._m(), path)

    def cross_validation_models(self):
        from llama_github_io_amd.core import dkv
        keys = self._m().output.get("cross_validation_models") or []
        return [dkv.get(k) for k in keys]

    def cross_validation_holdout_predictions(self):
        from llama_github_io_amd.core import dkv
        return dkv.get(self._m().output.get("cross_validation_holdout_predictions_frame_id"))

    def cross_validation_metrics_summary(self):
        return self._m().output.get("cross_validation_metrics_summary")

    @property
    def key(self):
        return self.model_id

    def __repr__(self):
        if self._model is None:
            return f"<{type(self).__name__} (untrained) {self._parms}>"
        return f"<{type(self).__name__} model_id={self.model_id}>"


def make_estimator(name: str, algo: str, supervised: bool = True, aliases: dict | None = None, doc: str = ""):
    cls = type(name, (H2OEstimator,), dict(algo=algo, supervised_learning=supervised, _param_aliases=dict(aliases or {}),
                                           __doc__=doc or f"H2O {algo} estimator (MI355X-native engine)."))
    return cls
