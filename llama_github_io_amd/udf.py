"""User-defined functions: custom metrics and custom GBM distributions (reference:
``h2o-core/src/main/java/water/udf/CFuncRef.java``, ``CMetricFunc.java``, ``CDistributionFunc.java``,
``hex/CustomMetric.java``, ``hex/DistributionFactory.java:CustomDistribution``; client side
``h2o-py/h2o/h2o.py:upload_custom_metric`` / ``upload_custom_distribution``).

The reference ships the user's class to the cluster and runs it under Jython, row by row. Here the
user's class object runs in-process: it is first called with whole NumPy columns (most metric /
gradient code is plain arithmetic and vectorises as written); a function that only handles scalars
falls back to a per-row loop with the reference's row-wise semantics. References keep the reference
string format ``python:<key>=<module>.<Class>Wrapper``. A class given as a source string (the reference's
``func`` string form with ``class_name``) is compiled into its own module namespace in-process, where the
reference would compile it under Jython on the cluster.
"""
from __future__ import annotations

import inspect

import numpy as np

_REGISTRY: dict = {}


def _from_source(src: str, func_file: str, class_name: str | None):
    """h2o.py:upload_custom_metric string form: ``src`` defines ``class_name`` (required, as in the reference)."""
    import types
    if not class_name:
        raise ValueError("class_name is required when the custom function is given as a source string")
    mod = types.ModuleType(func_file[:-3] if func_file.endswith(".py") else func_file)
    exec(compile(src, func_file, "exec"), mod.__dict__)
    cls = mod.__dict__.get(class_name)
    if not inspect.isclass(cls):
        raise ValueError(f"the source does not define a class {class_name!r}")
    return cls


def _register(func, func_file, func_name, kind, methods, class_name=None):
    module = func_file[:-3] if func_file.endswith(".py") else func_file
    if isinstance(func, str):
        func = _from_source(func, func_file, class_name)
    if not inspect.isclass(func):
        raise TypeError("pass the custom function as a class or as class source code with class_name")
    for m in methods:
        if not callable(getattr(func, m, None)):
            raise TypeError(f"the {kind} class needs a `{m}` method")
    key = func_name or f"{kind}_{func.__name__}"
    _REGISTRY[key] = func()
    return f"python:{key}={module}.{func.__name__}Wrapper"


def upload_custom_metric(func, func_file="metrics.py", func_name=None, class_name=None, source_provider=None):
    return _register(func, func_file, func_name, "metrics", ("map", "reduce", "metric"), class_name)


def upload_custom_distribution(func, func_file="distributions.py", func_name=None, class_name=None,
                               source_provider=None):
    return _register(func, func_file, func_name, "distributions", ("link", "init", "gradient", "gamma"), class_name)


def resolve(ref: str):
    if not isinstance(ref, str) or not ref.startswith("python:"):
        raise ValueError(f"not a custom function reference: {ref!r}")
    key = ref[len("python:"):].split("=", 1)[0]
    if key not in _REGISTRY:
        raise KeyError(f"custom function {key} was not uploaded")
    return key, _REGISTRY[key]


def custom_metric_value(ref: str, preds: np.ndarray, actual: np.ndarray, w=None, offset=None, model=None):
    """CMetricFunc over all rows: map(pred_row, act_row, w, o, model) -> state, reduce, metric.
    ``preds`` [N, P] in the reference's prediction layout ([label, p0, p1, ...] or [value]),
    ``actual`` [N] (class index for classification)."""
    name, obj = resolve(ref)
    return name, custom_metric_finish(ref, [custom_metric_state(ref, preds, actual, w, offset, model)])


def custom_metric_finish(ref: str, states: list) -> float:
    """The reduce of per-shard map/reduce states (in shard order; empty shards give None) and the metric —
    MRTask's reduce across nodes (water/udf/CMetricFunc: the state is all that travels)."""
    _, obj = resolve(ref)
    state = None
    for s in states:
        if s is not None:
            state = s if state is None else obj.reduce(state, s)
    return float(obj.metric(state))


def custom_metric_state(ref: str, preds: np.ndarray, actual: np.ndarray, w=None, offset=None, model=None):
    """map + reduce over the rows of one shard: the shard's metric state (None for no rows)."""
    name, obj = resolve(ref)
    n = preds.shape[0]
    if n == 0:
        return None
    w = np.ones(n) if w is None else np.asarray(w, dtype=np.float64)
    o = np.zeros(n) if offset is None else np.asarray(offset, dtype=np.float64)
    try:                                    # vectorised: columns in, per-row state columns out, summed
        st = [np.broadcast_to(np.asarray(s, dtype=np.float64), (n,)).copy() for s in obj.map(preds.T, actual[None, :], w, o,
                                                                                                 model)]
        # the user's reduce itself, applied as a pairwise tree fold over the state columns (log2(N)
        # vectorised calls; MRTask reduces the same way, so reduce must be associative anyway)
        while st[0].shape[0] > 1:
            m = st[0].shape[0]
            h = m // 2
            left = [s[:2 * h:2] for s in st]
            right = [s[1:2 * h:2] for s in st]
            red = [np.broadcast_to(np.asarray(r, dtype=np.float64), (h,)) for r in obj.reduce(left, right)]
            if len(red) != len(st):
                raise ValueError("reduce changed the state arity")
            st = [np.concatenate([r, s[2 * h:]]) for r, s in zip(red, st)]
        state = [float(s[0]) for s in st]
        if not all(np.isfinite(v) for v in state):
            raise ValueError("non-finite vectorised state")
    except Exception:                       # noqa: BLE001 - scalar-only user code: row-wise path
        state = None
        for i in range(n):
            s = obj.map(list(preds[i]), [float(actual[i])], float(w[i]), float(o[i]), model)
            state = s if state is None else obj.reduce(state, s)
    return state


class CustomDistributionFns:
    """Vectorised adapter over a user CDistributionFunc (see module doc)."""

    def __init__(self, ref):
        self.ref = ref
        _, self.obj = resolve(ref)
        self.link = str(self.obj.link())

    def _call(self, fn, *arrays, n_out=1):
        shape = arrays[-1].shape
        try:
            r = fn(*arrays)
            if n_out == 1:
                return np.broadcast_to(np.asarray(r, dtype=np.float64), shape).copy()
            return [np.broadcast_to(np.asarray(v, dtype=np.float64), shape).copy() for v in r]
        except Exception:                   # noqa: BLE001 - scalar-only user code
            cols = [a.tolist() for a in arrays]
            rows = [fn(*[c[i] for c in cols]) for i in range(len(cols[0]))]
            if n_out == 1:
                return np.asarray(rows, dtype=np.float64)
            return [np.asarray([r[k] for r in rows], dtype=np.float64) for k in range(n_out)]

    def gradient(self, y, f):
        return self._call(self.obj.gradient, y, f)

    def init(self, w, o, y):
        return self._call(self.obj.init, w, o, y, n_out=2)

    def gamma(self, w, y, z, f):
        return self._call(self.obj.gamma, w, y, z, f, n_out=2)
