"""``H2OGridSearch`` (reference: ``h2o-py/h2o/grid/grid_search.py``)."""
from __future__ import annotations

from llama_github_io_amd import grid as _grid
from llama_github_io_amd.core.job import Job


class H2OGridSearch:
    def __init__(self, model, hyper_params, grid_id=None, search_criteria=None, export_checkpoints_dir=None,
                 recovery_dir=None, parallelism=1):
        self.model = model() if isinstance(model, type) else model
        self.hyper_params = dict(hyper_params)
        self.grid_id = grid_id
        self.search_criteria = search_criteria
        self.parallelism = parallelism
        self.recovery_dir = recovery_dir
        self._grid = None

    def _job_args(self, x, y, training_frame, offset_column, fold_column, weights_column, validation_frame, params):
        base = dict(self.model._parms)
        base.update({k: v for k, v in params.items() if v is not None})
        for k, v in (("offset_column", offset_column), ("fold_column", fold_column), ("weights_column", weights_column)):
            if v is not None:
                base[k] = v
        job = Job(f"grid {self.model.algo}", dest=self.grid_id)
        return job, (_grid.grid_search, self.model.algo, self.hyper_params, base, x, y, training_frame, validation_frame,
                     self.grid_id, self.search_criteria, self.parallelism, job, self.recovery_dir)

    def train(self, x=None, y=None, training_frame=None, offset_column=None, fold_column=None, weights_column=None,
              validation_frame=None, **params):
        job, args = self._job_args(x, y, training_frame, offset_column, fold_column, weights_column, validation_frame,
                                   params)
        self._grid = job.run_sync(*args)
        self.grid_id = self._grid.grid_id
        return self

    # ---- asynchronous build (grid_search.py start / join / cancel / detach)
    def start(self, x, y=None, training_frame=None, offset_column=None, fold_column=None, weights_column=None,
              validation_frame=None, **params):
        self._job, args = self._job_args(x, y, training_frame, offset_column, fold_column, weights_column,
                                         validation_frame, params)
        self._job.run_async(*args)
        return self

    def join(self):
        job = getattr(self, "_job", None)
        if job is not None:
            job.join()
            self._grid = job.result if getattr(job, "result", None) is not None else self._grid
            if self._grid is not None:
                self.grid_id = self._grid.grid_id
        return self

    def cancel(self):
        job = getattr(self, "_job", None)
        if job is not None:
            job.cancel()

    def detach(self):
        self._job = None

    def resume(self, recovery_dir=None, **kwargs):
        """Continue a grid from its recovery directory (``recovery_dir`` of the original search)."""
        d = recovery_dir or self.recovery_dir
        if d is None:
            raise ValueError("resume needs the grid's recovery_dir")
        self._grid = _grid.resume(d)
        self.grid_id = self._grid.grid_id
        return self

    def build_model(self, algo_params):
        """grid_search.py build_model: ``algo_params`` carries x / y / training_frame / validation_frame and extra
        model parameters; runs the grid over the hyper-parameters with them."""
        ap = dict(algo_params)
        if ap.get("training_frame") is None:
            raise ValueError("Missing training_frame")
        x, y = ap.pop("x"), ap.pop("y", None)
        tf, vf = ap.pop("training_frame"), ap.pop("validation_frame", None)
        return self.train(x=x, y=y, training_frame=tf, validation_frame=vf, **ap)

    @property
    def key(self):
        return self.grid_id

    @property
    def model_ids(self):
        ms = getattr(self, "_grid_models_sorted", None) or self._grid.models
        return [m.key for m in ms]

    @property
    def hyper_names(self):
        return list(self.hyper_params)

    @property
    def failure_details(self):
        return [f.get("error") for f in self._grid.failures]

    @property
    def failure_stack_traces(self):
        return [f.get("error") for f in self._grid.failures]

    @property
    def failed_raw_params(self):
        return [list(f["params"].values()) for f in self._grid.failures]

    def __iter__(self):
        return iter(self.models)

    # ---- per-model accessors: {model_id: value} as in grid_search.py
    def _each(self, fn):
        return {m.model_id: fn(m) for m in self._wrap(getattr(self, "_grid_models_sorted", None) or self._grid.models)}

    def predict(self, test_data):
        return self._each(lambda m: m.predict(test_data))

    def model_performance(self, test_data=None, train=False, valid=False, xval=False):
        return self._each(lambda m: m.model_performance(test_data, train=train, valid=valid, xval=xval)
                          if test_data is None else m.model_performance(test_data))

    def is_cross_validated(self):
        return self._each(lambda m: m._m().params.get("nfolds", 0) not in (0, 1, None))

    def xval_keys(self):
        return self._each(lambda m: [x.model_id for x in (m.cross_validation_models() or [])])

    def get_xval_models(self, key=None):
        out = self._each(lambda m: m.cross_validation_models())
        return out[key] if key is not None else out

    @property
    def xvals(self):
        return self.get_xval_models()

    def scoring_history(self):
        return self._each(lambda m: m.scoring_history())

    def varimp(self, use_pandas=False):
        return self._each(lambda m: m.varimp(use_pandas=use_pandas))

    def coef(self):
        return self._each(lambda m: m.coef())

    def coef_norm(self):
        return self._each(lambda m: m.coef_norm())

    def pprint_coef(self):
        for k, v in self.coef().items():
            print(f"Model {k}: {v}")

    def deepfeatures(self, test_data, layer):
        return self._each(lambda m: m.deepfeatures(test_data, layer))

    def weights(self, matrix_id=0):
        return self._each(lambda m: m.weights(matrix_id))

    def biases(self, vector_id=0):
        return self._each(lambda m: m.biases(vector_id))

    def normmul(self):
        return self._each(lambda m: m.normmul())

    def normsub(self):
        return self._each(lambda m: m.normsub())

    def respmul(self):
        return self._each(lambda m: m.respmul())

    def respsub(self):
        return self._each(lambda m: m.respsub())

    def catoffsets(self):
        return self._each(lambda m: m.catoffsets())

    def get_summary(self):
        return self._each(lambda m: m.summary())

    def show_summary(self):
        for k, v in self.get_summary().items():
            print(f"Model {k}:\n{v}")

    def show(self, verbosity=None, fmt=None):
        print(f"Grid {self.grid_id}: {len(self)} models, {len(self._grid.failures)} failed")
        print(self.sorted_metric_table)

    def sort_by(self, metric, increasing=True):
        """Deprecated in the reference in favour of get_grid(sort_by, decreasing)."""
        return self.get_grid(metric, not increasing).sorted_metric_table

    def pareto_front(self, test_frame=None, x_metric=None, y_metric=None, optimum="top left", title=None,
                     color_col="algo"):
        """The grid's models not dominated in (x_metric, y_metric): metrics on ``test_frame`` when given, else
        the validation (or training) metrics of every model."""
        import pandas as pd
        from .explanation import pareto_front as _pf
        rows = []
        for m in self._wrap(getattr(self, "_grid_models_sorted", None) or self._grid.models):
            perf = m.model_performance(test_frame) if test_frame is not None else None
            mm = perf._metric_json if perf is not None and hasattr(perf, "_metric_json") else None
            if mm is None:
                out = m._m().output
                mm = out.get("validation_metrics") or out.get("training_metrics") or {}
            rows.append(dict(model_id=m.model_id, algo=m.algo,
                             **{k: v for k, v in dict(mm).items() if isinstance(v, (int, float))}))
        return _pf(pd.DataFrame(rows), x_metric=x_metric, y_metric=y_metric, optimum=optimum, title=title,
                   color_col=color_col)

    @property
    def models(self):
        return self._wrap(self._grid.models)

    def _wrap(self, ms):
        from .estimators.estimator_base import H2OEstimator
        out = []
        for m in ms:
            e = type(self.model)()
            e._model = m
            e.model_id = m.key
            out.append(e)
        return out

    def get_grid(self, sort_by=None, decreasing=None):
        g = H2OGridSearch(type(self.model), self.hyper_params, self.grid_id, self.search_criteria)
        g._grid = self._grid
        rows, _ = self._grid.sorted_models(sort_by, decreasing)
        g._sorted = rows
        g._sort = (sort_by, decreasing)
        g._grid_models_sorted = [r[0] for r in rows]
        return g

    @property
    def sorted_metric_table(self):
        import pandas as pd
        rows, key = self._grid.sorted_models(*getattr(self, "_sort", (None, None)))
        names = list(self.hyper_params)
        return pd.DataFrame([dict(zip(names, h), model_ids=m.key, **{key: v}) for m, h, v in rows])

    def summary(self):
        return self.sorted_metric_table

    def __getitem__(self, i):
        ms = getattr(self, "_grid_models_sorted", None) or self._grid.models
        return self._wrap([ms[i]])[0]

    def __len__(self):
        return len(self._grid.models)

    @property
    def failed_params(self):
        return [f["params"] for f in self._grid.failures]

    def get_hyperparams(self, id, display=True):
        return self._grid.hyper_values[id]

    def get_hyperparams_dict(self, id, display=True):
        return dict(zip(self.hyper_params, self._grid.hyper_values[id]))

    def r2(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.r2(train=train, valid=valid, xval=xval))

    def mse(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.mse(train=train, valid=valid, xval=xval))

    def rmse(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.rmse(train=train, valid=valid, xval=xval))

    def mae(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.mae(train=train, valid=valid, xval=xval))

    def rmsle(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.rmsle(train=train, valid=valid, xval=xval))

    def logloss(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.logloss(train=train, valid=valid, xval=xval))

    def mean_residual_deviance(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.mean_residual_deviance(train=train, valid=valid, xval=xval))

    def auc(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.auc(train=train, valid=valid, xval=xval))

    def aic(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.aic(train=train, valid=valid, xval=xval))

    def gini(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.gini(train=train, valid=valid, xval=xval))

    def aucpr(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.aucpr(train=train, valid=valid, xval=xval))

    def residual_deviance(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.residual_deviance(train=train, valid=valid, xval=xval))

    def residual_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.residual_degrees_of_freedom(train=train, valid=valid, xval=xval))

    def null_deviance(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.null_deviance(train=train, valid=valid, xval=xval))

    def null_degrees_of_freedom(self, train=False, valid=False, xval=False):
        return self._each(lambda m: m.null_degrees_of_freedom(train=train, valid=valid, xval=xval))

    def pr_auc(self, train=False, valid=False, xval=False):
        return self.aucpr(train=train, valid=valid, xval=xval)
