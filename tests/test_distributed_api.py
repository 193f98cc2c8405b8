"""Row-sharded training through the h2o API (gloo, world_size 2 and 4, CPU).

Every rank runs the same script (SPMD, as under torchrun): ``h2o.init()`` joins the process group,
``h2o.import_file`` parses its own byte range of the CSV (ParseDataset: domains unified over the
ranks), and each trainer reduces over the shards (all-reduce / reduce-scatter / exact order statistics /
an all-to-all range partition), never gathering rows in proportion to the frame. The sharded run must produce the model and training metrics of
the single-process run (reference: ``water/MRTask.java`` reduce semantics — the cluster size never
changes the answer).
"""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _write_csv(path, n=1200, seed=0):
    rng = np.random.default_rng(seed)
    x = rng.normal(size=(n, 4))
    # categorical levels that appear only in some row ranges -> every rank sees a different local domain
    cat = np.array(["a", "b", "c"])[rng.integers(0, 3, n)].astype(object)
    cat[-n // 5:] = np.where(rng.random(n // 5) < 0.5, "z_late", cat[-n // 5:])
    logit = 1.5 * x[:, 0] - x[:, 1] + 0.7 * x[:, 2] * x[:, 3] + (cat == "b") * 0.8 - (cat == "z_late") * 0.5
    yb = np.where(rng.random(n) < 1 / (1 + np.exp(-logit)), "yes", "no")
    yr = 2 * x[:, 0] + np.sin(3 * x[:, 1]) + 0.3 * rng.standard_t(3, n)
    y3 = np.array(["k0", "k1", "k2"])[np.clip((logit > -0.5).astype(int) + (logit > 1.0).astype(int), 0, 2)]
    with open(path, "w") as f:
        f.write("x0,x1,x2,x3,cat,yb,yr,y3,w,trt\n")
        wts = rng.integers(0, 4, n) * 0.5
        trt = np.where(rng.random(n) < 0.5, "treat", "ctrl")
        for i in range(n):
            xs = ",".join("" if (i % 97 == 5 and j == 2) else f"{x[i, j]:.6f}" for j in range(4))
            f.write(f"{xs},{cat[i]},{yb[i]},{yr[i]:.6f},{y3[i]},{wts[i]},{trt[i]}\n")


CASES = {
    "gbm_bernoulli": ("gbm", dict(ntrees=4, max_depth=3, seed=11, sample_rate=0.8, col_sample_rate=0.75), "yb"),
    "gbm_laplace": ("gbm", dict(ntrees=3, max_depth=3, seed=5, distribution="laplace"), "yr"),
    "gbm_quantile": ("gbm", dict(ntrees=3, max_depth=3, seed=5, distribution="quantile", quantile_alpha=0.8), "yr"),
    "gbm_huber": ("gbm", dict(ntrees=3, max_depth=3, seed=5, distribution="huber"), "yr"),
    "gbm_multinomial": ("gbm", dict(ntrees=3, max_depth=3, seed=3), "y3"),
    "drf": ("drf", dict(ntrees=4, max_depth=4, seed=7), "yb"),
    "xgboost": ("xgboost", dict(ntrees=4, max_depth=3, seed=2), "yb"),
    "glm_default_lambda": ("glm", dict(family="binomial"), "yb"),
    "glm_lambda_search": ("glm", dict(family="binomial", lambda_search=True, nlambdas=8), "yb"),
    "glm_gaussian_pvalues": ("glm", dict(family="gaussian", lambda_=0.0, compute_p_values=True), "yr"),
    "glm_multinomial": ("glm", dict(family="multinomial", lambda_=1e-3), "y3"),
    "kmeans": ("kmeans", dict(k=3, seed=3, init="Furthest"), None),
    "pca": ("pca", dict(k=2, transform="STANDARDIZE"), None),
    "naivebayes": ("naivebayes", dict(), "yb"),
    "gbm_cv": ("gbm", dict(ntrees=3, max_depth=2, seed=4, nfolds=3), "yb"),
    "deeplearning": ("deeplearning", dict(hidden=[8, 8], epochs=2, seed=1, mini_batch_size=64, score_interval=1e9), "yb"),
    "deeplearning_reg": ("deeplearning", dict(hidden=[6], epochs=1, seed=2, mini_batch_size=50, activation="Tanh",
                                              adaptive_rate=False, rate=0.01, momentum_start=0.5, score_interval=1e9), "yr"),
    "coxph": ("coxph", dict(stop_column="x3"), "yb"),
    "coxph_strata_breslow": ("coxph", dict(stop_column="x3", stratify_by=["cat"], ties="breslow", weights_column="w"),
                             "yb"),
    "aggregator": ("aggregator", dict(target_num_exemplars=60, rel_tol_num_exemplars=0.3, save_mapping_frame=True), None),
    "psvm": ("psvm", dict(gamma=0.3, hyper_param=0.5), "yb"),
    "infogram": ("infogram", dict(top_n_features=4, seed=3, algorithm_params=dict(ntrees=4, max_depth=3)), "yb"),
    "stackedensemble": ("stackedensemble", dict(), "yb"),
    "isotonic": ("isotonicregression", dict(), "yr"),
    "isotonic_weighted": ("isotonicregression", dict(weights_column="w", out_of_bounds="clip"), "yr"),
    "svd_gram": ("svd", dict(nv=3, transform="STANDARDIZE"), None),
    "svd_randomized": ("svd", dict(nv=2, svd_method="Randomized", transform="DEMEAN", seed=3), None),
    "pca_randomized": ("pca", dict(k=2, transform="STANDARDIZE", pca_method="Randomized", seed=3), None),
    "targetencoder": ("targetencoder", dict(blending=True, inflection_point=3, smoothing=2), "yb"),
    "targetencoder_multi": ("targetencoder", dict(), "y3"),
    "gam_cr": ("gam", dict(gam_columns=["x1"], num_knots=[6], family="binomial", seed=1), "yb"),
    "gam_tp_is": ("gam", dict(gam_columns=[["x1", "x2"], "x3"], bs=[1, 2], num_knots=[8, 5], seed=1), "yr"),
    "anovaglm": ("anovaglm", dict(family="gaussian", highest_interaction_term=2), "yr"),
    "modelselection_maxr": ("modelselection", dict(mode="maxr", max_predictor_number=2), "yr"),
    "modelselection_backward": ("modelselection", dict(mode="backward", min_predictor_number=2, family="gaussian"), "yr"),
    "upliftdrf": ("upliftdrf", dict(ntrees=3, max_depth=4, treatment_column="trt", seed=3, auuc_nbins=50), "yb"),
    "dt": ("dt", dict(max_depth=4, min_rows=20), "yb"),
    "glrm_svd": ("glrm", dict(k=2, init="SVD", transform="STANDARDIZE", max_iterations=30, seed=4, recover_svd=True), None),
    "glrm_pp": ("glrm", dict(k=3, init="PlusPlus", transform="STANDARDIZE", max_iterations=20, seed=4,
                             regularization_x="Quadratic", gamma_x=0.1), None),
    "hglm": ("glm", dict(family="gaussian", HGLM=True, random_columns=["cat"], seed=1), "yr"),
    "rulefit": ("rulefit", dict(min_rule_length=1, max_rule_length=2, rule_generation_ntrees=3, seed=2, lambda_=1e-3), "yb"),
    "quantile": ("quantile", dict(probs=[0.01, 0.1, 0.5, 0.77, 0.99]), None),
    "quantile_weighted_low": ("quantile", dict(probs=[0.25, 0.5, 0.9], combine_method="low"), None),
    "isolationforest": ("isolationforest", dict(ntrees=6, seed=5, contamination=0.05), None),
    "extendedisolationforest": ("extendedisolationforest", dict(ntrees=5, seed=5, extension_level=2), None),
    "gbm_quantile_weighted": ("gbm", dict(ntrees=3, max_depth=3, seed=5, distribution="quantile", quantile_alpha=0.3,
                                          weights_column="w"), "yr"),
    # custom metric (CMetricFunc map/reduce): per-shard states reduced across ranks, no row gather
    "gbm_custom_metric": ("gbm", dict(ntrees=3, max_depth=3, seed=5), "yr"),
}


class WeightedMAE:
    """A CMetricFunc (h2o-py custom metric protocol): state = [sum w|err|, sum w]."""

    def map(self, pred, act, w, o, model):
        return [w * abs(pred[0] - act[0]), w]

    def reduce(self, l, r):
        return [l[0] + r[0], l[1] + r[1]]

    def metric(self, l):
        return l[0] / l[1]

METRIC_KEYS = ("AUC", "logloss", "MSE", "RMSE", "mae", "mean_per_class_error", "tot_withinss", "r2", "AUUC", "qini",
               "concordance", "loglik", "custom_metric_value")


def _run_cases(csv, names, out_path):
    sys.path.insert(0, ROOT)
    import h2o
    from llama_github_io_amd.models import builder
    h2o.init(verbose=False)
    res = {"cloud_size": h2o.cluster().cloud_size}
    fr = h2o.import_file(csv)
    res["nrows"] = fr.nrows
    res["types"] = [fr.type(n) for n in fr.names]
    res["cat_levels"] = fr["cat"].levels()[0]
    res["mean_x0"] = fr["x0"].mean()
    res["sd_x1"] = fr["x1"].sd()[0]
    res["nacnt"] = fr.nacnt()
    for name in names:
        algo, params, y = CASES[name]
        x = ["x0", "x1", "x2", "x3", "cat"] if algo != "isotonicregression" else ["x0"]
        if algo in ("psvm", "aggregator", "kmeans", "pca", "svd", "quantile", "extendedisolationforest", "anovaglm", "modelselection", "glrm"):
            x = ["x0", "x1", "x2", "x3"]
        if algo == "dt":
            x = ["x0", "x1", "x3"]
        if algo == "upliftdrf":
            x = ["x0", "x1", "x2", "x3", "cat", "trt"]
        pp = dict(params)
        if name == "quantile_weighted_low":
            pp["weights_column"] = "w"
        if name == "gbm_custom_metric":
            pp["custom_metric_func"] = h2o.upload_custom_metric(WeightedMAE, func_name="dist_wmae")
        if algo == "stackedensemble":
            base = [builder.train(a, dict(nfolds=3, fold_assignment="Modulo", keep_cross_validation_predictions=True,
                                          seed=1, **kw), x=x, y=y, training_frame=fr, model_id=f"se_{a}")
                    for a, kw in (("gbm", dict(ntrees=3, max_depth=3)), ("glm", dict(family="binomial")))]
            pp["base_models"] = [b.key for b in base]
        import llama_github_io_amd.parallel.collectives as coll
        g0, c0 = coll.stats()["row_gathers"], coll.stats()["calls"]
        m = builder.train(algo, pp, x=x, y=y, training_frame=fr)
        res.setdefault("row_gathers", {})[name] = coll.stats()["row_gathers"] - g0
        res.setdefault("calls", {})[name] = coll.stats()["calls"] - c0
        if algo == "quantile":
            q = m.output["quantiles"]
            res[name] = dict(pred=[q[c] for c in sorted(q)], metrics={}, cv={})
            continue
        if algo == "infogram":
            res[name] = dict(pred=m.output["relevance"] + m.output["cmi_raw"], metrics={}, cv={})
            continue
        if algo == "aggregator":
            agg = m.aggregated_frame().as_data_frame()
            mp = h2o.get_frame(m.output["mapping_frame"]).as_data_frame()
            res.setdefault("shapes", {})[name] = [list(agg.shape), list(mp.shape)]
            res[name] = dict(pred=agg.select_dtypes(include=[np.number]).to_numpy(np.float64).ravel().tolist()
                             + mp.to_numpy(np.float64).ravel().tolist(), metrics={}, cv={})
            continue
        P = m.predict(fr).as_data_frame()
        num = P.select_dtypes(include=[np.number]).to_numpy(dtype=np.float64)
        tm = m.output.get("training_metrics") or {}
        cvm = m.output.get("cross_validation_metrics") or {}
        res[name] = dict(pred=num.tolist(), metrics={k: tm.get(k) for k in METRIC_KEYS if tm.get(k) is not None},
                         cv={k: cvm.get(k) for k in METRIC_KEYS if cvm.get(k) is not None})
    import llama_github_io_amd.parallel.collectives as coll
    if coll.rank() == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)


def _worker(rank, world, port, csv, names, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), H2O_AMD_DEVICE="cpu", OMP_NUM_THREADS="1",
                      H2O_AGG_CHUNK="250",   # aggregator chunks straddle the shard boundaries
                      H2O_DL_DP="sync")      # DeepLearning: per-step gradient sync (== single process);
    # the default model-averaging mode is pinned by tests/test_dl_model_averaging.py
    _run_cases(csv, names, out_path)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def _launch(world, csv, names, out_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_worker, args=(r, world, port, csv, names, out_path)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(600)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    with open(out_path) as f:
        return json.load(f)


def _compare(single, sharded, world):
    assert sharded["cloud_size"] == world and single["cloud_size"] == 1
    assert sharded["nrows"] == single["nrows"]
    assert sharded["types"] == single["types"]
    assert sharded["cat_levels"] == single["cat_levels"]
    assert sharded["nacnt"] == single["nacnt"]
    assert np.allclose(sharded["mean_x0"], single["mean_x0"], rtol=1e-12, atol=1e-14)
    assert np.allclose(sharded["sd_x1"], single["sd_x1"], rtol=1e-12, atol=1e-14)
    from llama_github_io_amd.models.builder import DISTRIBUTED
    # trainers that reduce over the shards never gather rows (no all-gather proportional to the frame)
    gathered = {n: c for n, c in sharded["row_gathers"].items() if CASES[n][0] in DISTRIBUTED and c}
    assert not gathered, gathered
    for name in CASES:
        if name not in single:
            continue
        a, b = np.asarray(single[name]["pred"]), np.asarray(sharded[name]["pred"])
        assert a.shape == b.shape, name
        tol = 1e-4 if name.startswith(("glm_multinomial", "glm_lambda", "glm_default", "deeplearning")) else 2e-5
        assert np.allclose(a, b, atol=tol, rtol=tol, equal_nan=True), (name, np.nanmax(np.abs(a - b)))
        for k, v in single[name]["metrics"].items():
            assert abs(v - sharded[name]["metrics"][k]) <= tol * max(1.0, abs(v)), (name, k, v, sharded[name]["metrics"][k])
        for k, v in single[name]["cv"].items():
            # fold models equal to the last float32 bit of a leaf value; those 1-ulp differences can
            # re-order tied holdout scores inside AUC, hence the looser bound
            assert abs(v - sharded[name]["cv"][k]) <= 1e-4 * max(1.0, abs(v)), (name, "cv", k)


@pytest.fixture(scope="module")
def csv_and_single(tmp_path_factory):
    d = tmp_path_factory.mktemp("dist")
    csv = str(d / "data.csv")
    _write_csv(csv)
    single = _launch(1, csv, list(CASES), str(d / "single.json"))
    return csv, single, d


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_api_equals_single(csv_and_single, world):
    csv, single, d = csv_and_single
    sharded = _launch(world, csv, list(CASES), str(d / f"w{world}.json"))
    _compare(single, sharded, world)


def _run_selection(csv, out_path):
    """Grid search and AutoML as SPMD programs (their budgets, model counts and orders agree over the ranks:
    ``coll.agree`` / ``broadcast_object``; every model trains row-sharded)."""
    sys.path.insert(0, ROOT)
    import h2o
    from h2o.automl import H2OAutoML
    from h2o.estimators import H2OGradientBoostingEstimator
    from h2o.grid import H2OGridSearch
    h2o.init(verbose=False)
    fr = h2o.import_file(csv)
    x = ["x0", "x1", "x2", "x3", "cat"]
    res = {"cloud_size": h2o.cluster().cloud_size}
    gs = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=3, seed=1),
                       hyper_params={"max_depth": [2, 3], "learn_rate": [0.1, 0.3]})
    gs.train(x=x, y="yb", training_frame=fr)
    g = gs.get_grid(sort_by="auc", decreasing=True)
    res["grid_n"] = len(g.model_ids)
    res["grid_auc"] = sorted(float(m.auc()) for m in g.models)
    gr = H2OGridSearch(H2OGradientBoostingEstimator(ntrees=2, seed=2), hyper_params={"max_depth": [1, 2, 3, 4]},
                       search_criteria={"strategy": "RandomDiscrete", "max_models": 2, "seed": 5})
    gr.train(x=x, y="yb", training_frame=fr)
    res["random_grid"] = sorted(int(m.actual_params["max_depth"]) for m in gr.models)
    # (AutoML's tree steps train up to 10^4 early-stopped trees: far too slow for the CPU reference builder; the SPMD
    # control flow — budgets, step plan, CV, leaderboard, the stacked ensemble — is what this pins)
    aml = H2OAutoML(max_models=3, seed=3, nfolds=2, include_algos=["GLM", "StackedEnsemble"])
    aml.train(x=x, y="yb", training_frame=fr)
    lb = aml.leaderboard.as_data_frame()
    res["aml_n"] = int(len(lb))
    res["aml_algos"] = sorted(str(m).split("_")[0] for m in lb["model_id"])
    res["aml_auc"] = sorted(float(v) for v in lb["auc"])
    import llama_github_io_amd.parallel.collectives as coll
    if coll.rank() == 0:
        with open(out_path, "w") as f:
            json.dump(res, f)


def _sel_worker(rank, world, port, csv, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), H2O_AMD_DEVICE="cpu", OMP_NUM_THREADS="1")
    _run_selection(csv, out_path)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


def _launch_sel(world, csv, out_path):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=_sel_worker, args=(r, world, port, csv, out_path)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(900)
        assert p.exitcode == 0, f"rank exited with {p.exitcode}"
    with open(out_path) as f:
        return json.load(f)


def test_sharded_grid_and_automl_equal_single(tmp_path):
    csv = str(tmp_path / "data.csv")
    _write_csv(csv)
    one = _launch_sel(1, csv, str(tmp_path / "sel1.json"))
    two = _launch_sel(2, csv, str(tmp_path / "sel2.json"))
    assert one["cloud_size"] == 1 and two["cloud_size"] == 2
    assert two["grid_n"] == one["grid_n"] == 4
    assert np.allclose(two["grid_auc"], one["grid_auc"], atol=1e-4)
    assert two["random_grid"] == one["random_grid"] and len(one["random_grid"]) == 2
    assert two["aml_n"] == one["aml_n"] >= 1 and two["aml_algos"] == one["aml_algos"]
    # CV AUCs of sharded runs merge fixed-lattice score histograms (equal to ~1e-4)
    assert np.allclose(two["aml_auc"], one["aml_auc"], atol=1e-4), (one["aml_auc"], two["aml_auc"])
