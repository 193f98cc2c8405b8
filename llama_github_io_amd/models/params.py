"""Parameter validation (reference: ``hex/ModelBuilder.java`` ``init(expensive)`` — every builder
checks its parameters and refuses bad or unsupported settings with an error message, and the REST /
h2o-py layer refuses unknown parameter names).

Every algorithm's public parameters come from the h2o-py estimator signatures
(``h2o/estimators/_schema.py``). Each one is either

* implemented by the trainer (the default),
* an **execution hint** of the Java cluster that has no meaning on this engine (thread counts,
  single-node mode, load balancing, DMatrix formats, ...): accepted and ignored, listed in ``HINTS``,
* or **not supported** yet (``UNSUPPORTED``): any non-default value raises ``ValueError`` instead of
  silently training a different model.

Names outside the schema (and outside the trainer's own extension defaults) raise too.
"""
from __future__ import annotations

import math

# execution hints of the Java backend: no effect on the model
HINTS = {
    "nthread", "gpu_id", "backend", "quiet_mode", "build_tree_one_node", "single_node_mode", "force_load_balance",
    "replicate_training_data", "col_major", "diagnostics", "fast_mode", "score_duty_cycle",
    "target_ratio_comm_to_comp", "parallelize_cross_validation", "nparallelism", "multinode_mode", "dmatrix_type",
    "save_matrix_directory", "check_constant_response", "reproducible", "pca_impl", "response_column",
    "auto_rebalance", "export_weights_and_biases", "verbose", "score_eval_metric_only",
    "max_confusion_matrix_size", "save_transformed_framekeys", "store_knot_locations", "generate_scoring_history",
    "score_iteration_interval", "score_validation_sampling", "u_name", "loading_name", "build_glm_model",
    "compute_metrics", "num_iteration_without_new_exemplar",
    "eval_metric", "export_checkpoints_dir", "gradient_epsilon", "svd_method",
    # DeepLearning ``sparse`` is a storage hint for sparse input.
    "sparse",
}

# parameters not implemented by this engine: a non-default value is refused
UNSUPPORTED: dict = {}
# (GLM ``rand_link`` is validated where the reference validates it: HGLM accepts identity / family_default per random
# column, hex/glm/GLMModel.java:534-548, see models/hglm.py)
# (Infogram ``max_iterations`` is a schema field with no InfogramParameters counterpart in the reference
# (hex/schemas/InfogramV3.java:82): accepted and, as there, without effect.)

# parameters the reference accepts but no longer honours: a non-default value warns like the reference
DEPRECATED = {
    "r2_stopping": "_r2_stopping is no longer supported - please use stopping_rounds, stopping_metric and "
                   "stopping_tolerance instead.",     # hex/tree/SharedTree.java:160
}

# values that count as "left at its default" whatever the schema says
_NEUTRAL = (None, "AUTO", "auto", "", [], {}, False)


def canon(v) -> str:
    """Spelling-independent form of an enum value: h2o-py ``uniform_adaptive``, Java
    ``UniformAdaptive`` and ``UNIFORM_ADAPTIVE`` all become ``uniformadaptive``."""
    return str(v).lower().replace("_", "").replace(" ", "")


def _is_default(v, default) -> bool:
    if v is None:
        return True
    if isinstance(v, str) and isinstance(default, str) and canon(v) == canon(default):
        return True
    if isinstance(v, float) and isinstance(default, (int, float)) and default is not None and not isinstance(default, bool):
        return math.isclose(v, float(default)) or (math.isinf(v) and math.isinf(float(default)))
    if v == default:
        return True
    return isinstance(v, (str, list, dict, bool)) and v in _NEUTRAL and default in _NEUTRAL


def schema(algo: str) -> dict | None:
    try:
        from h2o.estimators._schema import PARAMS
    except ImportError:    # pragma: no cover - the facade is part of the package tree
        return None
    return PARAMS.get(algo)


def validate(algo: str, params: dict, extra_allowed=()) -> None:
    """Raise ``ValueError`` on an unknown parameter name or on a non-default value of a parameter this
    engine does not implement (ModelBuilder.init's error messages)."""
    sch = schema(algo)
    if sch is None:
        return
    allowed = set(sch) | set(extra_allowed) | HINTS
    unknown = sorted(k for k in params if k not in allowed and not k.startswith("_"))
    if unknown:
        raise ValueError(f"{algo}: unknown parameter(s) {unknown}")
    for k, msg in DEPRECATED.items():
        if k in params and not _is_default(params[k], sch.get(k)) and params[k] != float("inf"):
            import warnings
            warnings.warn(msg, UserWarning, stacklevel=3)
    bad = sorted(k for k in UNSUPPORTED.get(algo, ()) if k in params and not _is_default(params[k], sch.get(k)))
    if bad:
        raise ValueError(f"{algo}: parameter(s) {bad} are not supported by this engine (leave them at their defaults)")
