"""MOJO writer (reference: ``h2o-genmodel/.../AbstractMojoWriter.java`` (model.ini [info]/[columns]/
[domains], ``domains/dNNN.txt``), ``GbmMojoWriter``/``DrfMojoWriter``/``IsolationForestMojoWriter``
(``trees/tCC_III.bin`` CompressedTree blobs), ``GLMMojoWriter``, ``KMeansMojoWriter``).

DeepLearning, PCA, Word2Vec, IsotonicRegression and StackedEnsemble (nested sub-MOJOs) use the
reference layouts of ``mojo/algos.py``. Models without a reference MOJO layout here are exported with
the same zip/ini container plus a ``model_state.json`` payload readable by this framework's reader
(``mojo_version`` suffix ``-amd``).
"""
from __future__ import annotations

import io
import json
import os
import time
import uuid
import zipfile

import numpy as np

from .treebytes import tree_to_bytes

MOJO_VERSIONS = {"gbm": "1.40", "drf": "1.40", "isolationforest": "1.40", "glm": "1.00", "kmeans": "1.00",
                 "deeplearning": "1.10", "pca": "1.00", "word2vec": "1.00", "isotonicregression": "1.00",
                 "stackedensemble": "1.01", "extendedisolationforest": "1.00", "coxph": "1.00", "targetencoder": "1.00",
                 "glrm": "1.10", "rulefit": "1.00"}
ALGO_FULL = {"gbm": "Gradient Boosting Machine", "drf": "Distributed Random Forest", "glm": "Generalized Linear Modeling",
             "kmeans": "K-means", "isolationforest": "Isolation Forest", "deeplearning": "Deep Learning",
             "pca": "Principal Components Analysis", "word2vec": "Word2Vec", "isotonicregression": "Isotonic Regression",
             "stackedensemble": "StackedEnsemble", "extendedisolationforest": "Extended Isolation Forest",
             "coxph": "Cox Proportional Hazards", "targetencoder": "TargetEncoder",
             "glrm": "Generalized Low Rank Modeling", "rulefit": "rulefit"}


def _escape(s: str) -> str:
    return s.replace("\\", "\\\\").replace("\n", "\\n")


def _arr(v):
    return "[" + ", ".join(repr(float(x)) if isinstance(x, float) else str(x) for x in v) + "]"


def _category(m):
    c = m.model_category
    return {"AnomalyDetection": "AnomalyDetection", "Clustering": "Clustering"}.get(c, c)


def _mojo_files(model, prefix: str = "") -> dict:
    """All entries of one model's MOJO (``model.ini``, domains, blobs), names under ``prefix``."""
    from . import algos as A
    from . import xgboost_mojo as XG
    info = model.info
    algo = model.algo
    cols = list(info.x) + ([info.response] if info.response else [])
    doms = list(info.domains) + ([info.response_domain] if info.response else [])
    if algo == "deeplearning":
        cols, doms = A.dl_columns(model)
    elif algo == "coxph" and getattr(model, "keep", None) is not None:
        cols, doms = A.coxph_columns(model)
    kv = {}
    kv["h2o_version"] = "3.46.0.amd0"
    kv["mojo_version"] = MOJO_VERSIONS.get(algo, "1.00-amd")
    kv["license"] = "Apache License Version 2.0"
    kv["algo"] = algo
    kv["algorithm"] = ALGO_FULL.get(algo, algo)
    kv["endianness"] = "LITTLE_ENDIAN"
    kv["category"] = _category(model)
    kv["uuid"] = str(uuid.uuid4().int >> 64)
    kv["supervised"] = "true" if info.response else "false"
    kv["n_features"] = info.F
    kv["n_classes"] = len(info.response_domain) if info.response_domain else 1
    kv["n_columns"] = len(cols)
    kv["n_domains"] = sum(1 for d in doms if d is not None)
    if info.offset:
        kv["offset_column"] = info.offset
    kv["balance_classes"] = "false"
    kv["default_threshold"] = model.default_threshold() if model.model_category == "Binomial" else 0.5
    kv["prior_class_distrib"] = "null"
    kv["model_class_distrib"] = "null"
    kv["timestamp"] = int(time.time() * 1000)
    kv["escape_domain_values"] = "true"
    blobs = {}
    if algo in ("gbm", "drf", "isolationforest"):
        _trees(model, kv, blobs)
    elif algo == "glm":
        _glm(model, kv)
    elif algo == "kmeans":
        _kmeans(model, kv)
    elif algo == "deeplearning":
        A.write_deeplearning(model, kv, blobs)
    elif algo == "pca":
        A.write_pca(model, kv, blobs)
    elif algo == "word2vec":
        A.write_word2vec(model, kv, blobs)
    elif algo == "isotonicregression":
        A.write_isotonic(model, kv, blobs)
    elif algo == "stackedensemble":
        _stacked(model, kv, blobs)
    elif algo == "extendedisolationforest":
        A.write_eif(model, kv, blobs)
    elif algo == "coxph" and getattr(model, "keep", None) is not None:
        A.write_coxph(model, kv, blobs)
    elif algo == "targetencoder":
        A.write_targetencoder(model, kv, blobs)
    elif algo == "glrm":
        A.write_glrm(model, kv, blobs)
    elif algo == "xgboost" and XG.supported(model):
        XG.write(model, kv, blobs)
    elif algo == "rulefit":
        A.write_rulefit(model, kv, blobs)
    elif algo == "gam":
        gcols, gdoms = A.write_gam(model, kv, blobs)
        cols = gcols + ([info.response] if info.response else [])
        doms = gdoms + [None] * (len(gcols) - len(gdoms)) + ([info.response_domain] if info.response else [])
        kv["n_features"] = len(cols) - (1 if info.response else 0)
        kv["n_columns"] = len(cols)
        kv["n_domains"] = sum(1 for d in doms if d is not None)
        kv["mojo_version"] = "1.00"
    else:
        _generic_state(model, kv, blobs)
    buf = io.StringIO()
    buf.write("[info]\n")
    for k, v in kv.items():
        buf.write(f"{k} = {v}\n")
    buf.write("\n[columns]\n")
    for c in cols:
        buf.write(c + "\n")
    buf.write("\n[domains]\n")
    di = 0
    files = {}
    for ci, d in enumerate(doms):
        if d is None:
            continue
        buf.write(f"{ci}: {len(d)} d{di:03d}.txt\n")
        files[prefix + f"domains/d{di:03d}.txt"] = "".join(_escape(str(s)) + "\n" for s in d)
        di += 1
    files[prefix + "model.ini"] = buf.getvalue()
    for n, b in blobs.items():
        files[n if n.startswith("models/") else prefix + n] = b
    return files


def write_mojo(model, path: str) -> str:
    if getattr(model, "preprocessors", None):
        # the reference refuses these too (ai/h2o/automl/preprocessing/TargetEncoding.java: "models obtained
        # with this feature can not yet be downloaded as MOJO")
        raise ValueError(f"model {model.key} has preprocessors (AutoML target encoding): no MOJO export")
    files = _mojo_files(model)
    os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
    with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as z:
        z.writestr("model.ini", files.pop("model.ini"))
        for n, b in files.items():
            z.writestr(n, b)
    return path


def _stacked(model, kv, blobs):
    """MultiModelMojoWriter layout: every base model and the metalearner as a nested MOJO."""
    subs = [(m.key, m) for m in model.base_models()] + [(model.meta.key, model.meta)]
    kv["submodel_count"] = len(subs)
    for i, (key, m) in enumerate(subs):
        d = f"models/{key}/"
        kv[f"submodel_key_{i}"] = key
        kv[f"submodel_dir_{i}"] = d
        blobs.update(_mojo_files(m, d))
    kv["base_models_num"] = len(subs) - 1
    kv["metalearner"] = model.meta.key
    kv["metalearner_transform"] = str(model.params.get("metalearner_transform", "NONE"))
    for i, (key, _) in enumerate(subs[:-1]):
        kv[f"base_model{i}"] = key


def _trees(model, kv, blobs):
    fr = model.forest
    algo = model.algo
    K = fr.K
    ntrees = len(fr.trees) // max(K, 1)
    kv["n_trees"] = ntrees
    kv["n_trees_per_class"] = K
    kv["_genmodel_encoding"] = "AUTO"
    vmap = lambda v: v  # noqa: E731
    if algo == "gbm":
        d = model.output["distribution"]
        kv["distribution"] = d
        kv["link_function"] = {"bernoulli": "logit", "quasibinomial": "logit", "modified_huber": "logit",
                               "multinomial": "log", "poisson": "log", "gamma": "log", "tweedie": "log"}.get(d, "identity")
        init = model.init_f if isinstance(model.init_f, (list, tuple)) else [model.init_f]
        kv["init_f"] = repr(float(init[0])) if K == 1 else "0.0"
    elif algo == "drf":
        kv["binomial_double_trees"] = "true" if model.output.get("double_trees") else "false"
        if model.model_category == "Binomial" and K == 1:
            vmap = lambda v: 1.0 - float(v)  # noqa: E731  H2O binomial DRF leaves hold P(class 0)
    else:
        kv["max_path_length"] = model.output["max_path_length"]
        kv["min_path_length"] = model.output["min_path_length"]
        kv["output_anomaly_flag"] = "true" if model.output.get("default_threshold") is not None else "false"
    for idx, (t, c) in enumerate(zip(fr.trees, fr.tree_class)):
        it = idx // max(K, 1)
        blobs[f"trees/t{c:02d}_{it:03d}.bin"] = tree_to_bytes(t, vmap)
    cm = getattr(model, "calibration_model", None)
    if cm is not None:                        # SharedTreeMojoWriter: calib_method + GLM beta / isotonic calibrator
        if cm.algo == "isotonicregression":
            from .algos import write_isotonic
            kv["calib_method"] = "isotonic"
            write_isotonic(cm, kv, blobs)
        else:
            co = cm.output["coefficients"]
            kv["calib_method"] = "platt"
            kv["calib_glm_beta"] = _arr([co["p"], co["Intercept"]])


def _glm(model, kv):
    ex = model.expander
    info = model.info
    kv["use_all_factor_levels"] = "true" if ex.use_all else "false"
    kv["cats"] = len(ex.cats)
    kv["cat_offsets"] = _arr(ex.cat_offsets + [ex.num_off])
    kv["nums"] = len(ex.nums)
    kv["mean_imputation"] = "true"
    kv["num_means"] = _arr(ex.num_mean.cpu().tolist())
    kv["cat_modes"] = _arr(ex.cat_modes)
    fam = model.output["family"]
    import torch
    betas = []
    for k in range(model.beta.shape[0]):
        braw, ic = ex.destandardize(model.beta[k, :-1], float(model.beta[k, -1]))
        betas += braw.cpu().tolist() + [ic]
    kv["beta"] = _arr(betas)
    kv["family"] = fam
    kv["link"] = model.output["link"]
    if fam == "tweedie":
        kv["tweedie_link_power"] = model.params.get("tweedie_link_power", 1.0)
    if fam == "ordinal":
        kv["ordinal_thresholds"] = _arr(model.output["ordinal_thresholds"])


def _kmeans(model, kv):
    ex = model.expander
    kv["standardize"] = "true" if ex.standardize else "false"
    if ex.standardize:
        kv["standardize_means"] = _arr(ex.num_mean.cpu().tolist())
        kv["standardize_mults"] = _arr((1.0 / ex.num_sd).cpu().tolist())
        kv["standardize_modes"] = _arr(ex.cat_modes)
    C = model.centers_std.cpu().double().numpy()
    kv["center_num"] = C.shape[0]
    for i in range(C.shape[0]):
        kv[f"center_{i}"] = _arr(C[i].tolist())


def _generic_state(model, kv, blobs):
    from ..persist import _default
    s = model.to_state()
    s["__class__"] = type(model).__module__ + ":" + type(model).__name__
    blobs["model_state.json"] = json.dumps(s, default=_default).encode()


def download_mojo(model, path=".", filename=None) -> str:
    name = filename or (model.key + ".zip")
    full = os.path.join(path, name) if (os.path.isdir(path) or not path.endswith(".zip")) else path
    if not os.path.isdir(path) and not path.endswith(".zip"):
        os.makedirs(path, exist_ok=True)
    return write_mojo(model, full)
