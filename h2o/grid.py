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

    def train(self, x=None, y=None, training_frame=None, offset_column=None, fold_column=None, weights_column=None,
              validation_frame=None, **params):
        base = dict(self.model._parms)
        base.update({k: v for k, v in params.items() if v is not None})
        for k, v in (("offset_column", offset_column), ("fold_column", fold_column), ("weights_column", weights_column)):
            if v is not None:
                base[k] = v
        job = Job(f"grid {self.model.algo}", dest=self.grid_id)
        self._grid = job.run_sync(_grid.grid_search, self.model.algo, self.hyper_params, base, x, y, training_frame,
                                  validation_frame, self.grid_id, self.search_criteria, self.parallelism, job,
                                  self.recovery_dir)
        self.grid_id = self._grid.grid_id
        return self

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
