"""``H2OAutoML`` (reference: ``h2o-py/h2o/automl/_estimator.py``)."""
from __future__ import annotations

from llama_github_io_amd import automl as _aml
from llama_github_io_amd.core import dkv
from llama_github_io_amd.core.job import Job


class H2OAutoML:
    def __init__(self, nfolds=5, balance_classes=False, class_sampling_factors=None, max_after_balance_size=5.0,
                 max_runtime_secs=None, max_runtime_secs_per_model=None, max_models=None, stopping_metric="AUTO",
                 stopping_tolerance=None, stopping_rounds=3, seed=None, project_name=None, exclude_algos=None,
                 include_algos=None, exploitation_ratio=-1, modeling_plan=None, preprocessing=None,
                 monotone_constraints=None, keep_cross_validation_predictions=False, keep_cross_validation_models=False,
                 keep_cross_validation_fold_assignment=False, sort_metric="AUTO", export_checkpoints_dir=None,
                 verbosity="warn"):
        self._aml = _aml.AutoML(
            project_name=project_name, max_models=max_models, max_runtime_secs=max_runtime_secs,
            max_runtime_secs_per_model=max_runtime_secs_per_model or 0, nfolds=nfolds, seed=seed,
            sort_metric=sort_metric, include_algos=include_algos, exclude_algos=exclude_algos,
            stopping_metric=stopping_metric, stopping_rounds=stopping_rounds, stopping_tolerance=stopping_tolerance,
            balance_classes=balance_classes, class_sampling_factors=class_sampling_factors,
            max_after_balance_size=max_after_balance_size,
            keep_cross_validation_predictions=keep_cross_validation_predictions,
            keep_cross_validation_models=keep_cross_validation_models,
            keep_cross_validation_fold_assignment=keep_cross_validation_fold_assignment, verbosity=verbosity,
            exploitation_ratio=exploitation_ratio, modeling_plan=modeling_plan, preprocessing=preprocessing,
            monotone_constraints=monotone_constraints, export_checkpoints_dir=export_checkpoints_dir)
        self.project_name = self._aml.project_name

    def train(self, x=None, y=None, training_frame=None, fold_column=None, weights_column=None, validation_frame=None,
              leaderboard_frame=None, blending_frame=None):
        job = Job("AutoML", dest=self.project_name)
        job.run_sync(self._aml.train, x, y, training_frame, validation_frame, leaderboard_frame, blending_frame,
                     fold_column, weights_column, job)
        return self

    @property
    def leader(self):
        from .estimators.estimator_base import H2OEstimator
        m = self._aml.leader
        if m is None:
            return None
        e = H2OEstimator()
        object.__setattr__(e, "algo", m.algo)
        e._model = m
        e.model_id = m.key
        return e

    @property
    def leaderboard(self):
        import pandas as pd
        from llama_github_io_amd.frame import H2OFrame
        rows, cols = self._aml.leaderboard_rows()
        return H2OFrame(pd.DataFrame(rows, columns=cols))

    @property
    def event_log(self):
        return self._aml.event_log

    def predict(self, test_data):
        return self.leader.predict(test_data)

    def get_best_model(self, algorithm=None, criterion=None):
        rows, _ = self._aml.leaderboard_rows()
        for r in rows:
            m = dkv.get(r["model_id"])
            if algorithm is None or m.algo == algorithm.lower():
                return m
        return None


def get_leaderboard(aml, extra_columns=None):
    return aml.leaderboard
