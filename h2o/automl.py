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

    # ---- h2o-py/h2o/automl/_base.py / _estimator.py surface
    @property
    def key(self):
        return self.project_name

    def detach(self):
        """Release the client-side job handle (the AutoML run and its models stay in the store)."""
        self._job = None

    @property
    def training_info(self):
        """event_log name / value pairs of the run: start / stop epochs and duration."""
        a = self._aml
        t0, t1 = getattr(a, "start_epoch", None), getattr(a, "stop_epoch", None)
        if t0 is None:
            return {}
        out = {"start_epoch": str(int(t0)), "creation_epoch": str(int(t0))}
        if t1 is not None:
            out.update(stop_epoch=str(int(t1)), duration_secs=str(int(round(t1 - t0))))
        return out

    @property
    def modeling_steps(self):
        """The executed plan, re-injectable as ``modeling_plan`` of a new run: [{name, steps: [{id, group, weight}]}]."""
        out, idx = [], {}
        for fam, sid, group, w in getattr(self._aml, "executed_steps", []):
            if fam not in idx:
                idx[fam] = len(out)
                out.append(dict(name=fam, steps=[]))
            out[idx[fam]]["steps"].append(dict(id=sid, group=int(group), weight=int(w)))
        return out

    def get_leaderboard(self, extra_columns=None):
        return get_leaderboard(self, extra_columns)

    def download_mojo(self, path=".", get_genmodel_jar=False, genmodel_name=""):
        return self.leader.download_mojo(path, get_genmodel_jar, genmodel_name)

    def download_pojo(self, path="", get_genmodel_jar=False, genmodel_name=""):
        from . import download_pojo
        return download_pojo(self.leader, path, get_jar=get_genmodel_jar, jar_name=genmodel_name)

    def pareto_front(self, test_frame=None, x_metric=None, y_metric=None, optimum="top left", title=None,
                     color_col="algo"):
        """Leaderboard models not dominated in (x_metric, y_metric); by default predict_time_per_row_ms vs the
        sort metric (h2o.explanation pareto_front over get_leaderboard('ALL'))."""
        from .explanation import pareto_front as _pf
        lb = get_leaderboard(self, "ALL").as_data_frame()
        if test_frame is not None:
            from llama_github_io_amd.automl import leaderboard_frame
            scored = leaderboard_frame([dkv.get(k) for k in lb["model_id"]], test_frame).as_data_frame()
            lb = lb.drop(columns=[c for c in lb.columns if c not in ("model_id", "algo", "training_time_ms",
                                                                        "predict_time_per_row_ms")])
            lb = lb.merge(scored, on="model_id")
        return _pf(lb, x_metric=x_metric, y_metric=y_metric, optimum=optimum, title=title, color_col=color_col)

    def get_best_model(self, algorithm=None, criterion=None):
        rows, _ = self._aml.leaderboard_rows()
        for r in rows:
            m = dkv.get(r["model_id"])
            if algorithm is None or m.algo == algorithm.lower():
                return m
        return None


def get_automl(project_name):
    """The AutoML run of ``project_name`` (reference: ``h2o-py/h2o/automl/autoh2o.py:13``): an object with the
    run's ``project_name``, ``leader``, ``leaderboard``, ``event_log`` and ``training_info``."""
    a = dkv.get(project_name)
    if not isinstance(a, _aml.AutoML):
        raise ValueError(f"no AutoML instance with project_name {project_name!r}")
    out = H2OAutoML.__new__(H2OAutoML)
    out._aml = a
    out.project_name = a.project_name
    return out


def get_leaderboard(aml, extra_columns=None):
    """autoh2o.get_leaderboard: the leaderboard plus the optional columns 'training_time_ms',
    'predict_time_per_row_ms' and 'algo' ('ALL': every one)."""
    import time as _time
    import pandas as pd
    from llama_github_io_amd.frame import H2OFrame
    rows, cols = aml._aml.leaderboard_rows()
    df = pd.DataFrame(rows, columns=cols)
    if extra_columns is None:
        return H2OFrame(df)
    ex = [extra_columns] if isinstance(extra_columns, str) else list(extra_columns)
    if any(str(e).upper() == "ALL" for e in ex):
        ex = ["training_time_ms", "predict_time_per_row_ms", "algo"]
    for c in ex:
        if c not in ("training_time_ms", "predict_time_per_row_ms", "algo"):
            raise ValueError(f"unknown leaderboard extension {c!r}")
    ms = [dkv.get(k) for k in df["model_id"]]
    if "training_time_ms" in ex:
        df["training_time_ms"] = [int(m.output.get("run_time_ms") or 0) for m in ms]
    if "predict_time_per_row_ms" in ex:
        fr = getattr(aml._aml, "leaderboard_frame", None) or getattr(aml._aml, "training_frame_ref", None)
        vals = []
        for m in ms:
            if fr is None:
                vals.append(float("nan"))
                continue
            t0 = _time.perf_counter()
            m.predict(fr)
            vals.append(1000.0 * (_time.perf_counter() - t0) / max(1, fr.nrows))
        df["predict_time_per_row_ms"] = vals
    if "algo" in ex:
        df["algo"] = [m.algo.replace("gbm", "GBM").replace("xgboost", "XGBoost").replace("glm", "GLM")
                      .replace("drf", "DRF").replace("deeplearning", "DeepLearning")
                      .replace("stackedensemble", "StackedEnsemble") for m in ms]
    return H2OFrame(df)
