"""The rest of the reference REST surface (reference ``water/api/RegisterV3Api.java`` and the algo
extensions ``hex/api/RegisterAlgos.java``): explanation endpoints (PartialDependence,
FeatureInteraction, FriedmansPopescusH, SignificantRules, Tree), frame transforms (Interaction,
MissingInserter, DCTTransformer, Tabulate, ParseSVMLight), GLM helpers (GetGLMRegPath,
MakeGLMModel, ComputeGram, DataInfoFrame), Word2Vec helpers, model/grid/frame binary persistence
(Models.fetch.bin, Models.upload.bin, Grid.bin import/export, Frames save/load), the
NodePersistentStorage key-value store, metadata/typeahead/diagnostic endpoints and the
deletion variants. Every payload carries the V3 ``__meta`` schema the h2o clients dispatch on."""
from __future__ import annotations

import glob
import math
import json
import os
import tempfile
import time

import numpy as np
import torch

from ..core import dkv
from ..core.job import Job
from ..frame import H2OFrame
from ..models.base import Model
from . import v3

from fastapi import Request  # noqa: E402  (module level: FastAPI resolves the string annotations here)
from fastapi.responses import FileResponse, PlainTextResponse  # noqa: E402


def register(app, _params, _unquote, _model_json):

    def get_frame(fid):
        fid = _unquote(fid)
        if isinstance(fid, dict):
            fid = fid.get("name")
        fr = dkv.get(fid)
        if not isinstance(fr, H2OFrame):
            raise KeyError(f"Object '{fid}' not found for argument: key")
        return fr

    def get_model(mid):
        mid = _unquote(mid)
        if isinstance(mid, dict):
            mid = mid.get("name")
        m = dkv.get(mid)
        if not isinstance(m, Model):
            raise KeyError(f"Object '{mid}' not found for argument: key")
        return m

    def done_job(dest, desc, fn=None):
        """Run ``fn`` as a Job (the h2o clients poll /3/Jobs/{key} until DONE)."""
        job = Job(desc, dest=dest)
        if fn is None:
            job.run_async(lambda: None)
        else:
            job.run_async(fn)
        return job

    def as_list(v):
        if v is None:
            return []
        return [_unquote(x) for x in (v if isinstance(v, list) else [v])]

    # ------------------------------------------------------------------------- explanation
    @app.post("/3/PartialDependence/")
    @app.post("/3/PartialDependence")
    async def pdp_post(request: Request):
        """hex/PartialDependence.java: 1-D and 2-D partial dependence tables (job; the result is read
        back with GET /3/PartialDependence/{dest})."""
        from .. import explain
        p = await _params(request)
        m, fr = get_model(p.get("model_id")), get_frame(p.get("frame_id"))
        cols = as_list(p.get("cols"))
        pairs = p.get("col_pairs_2dpdp") or []
        pairs = [as_list(pr) for pr in pairs]
        targets = as_list(p.get("targets")) or None
        nbins = int(p.get("nbins") or 20)
        row_index = int(p.get("row_index", -1) if p.get("row_index") is not None else -1)
        wc = p.get("weight_column_index")
        wc = None if wc in (None, -1, "-1") else (_unquote(wc) if not isinstance(wc, int) else wc)
        splits = {}
        ucols = as_list(p.get("user_cols"))
        if ucols:
            nus = [int(v) for v in (p.get("num_user_splits") or [])]
            us = [float(v) for v in (p.get("user_splits") or [])]
            o = 0
            for c, k in zip(ucols, nus):
                splits[c] = us[o:o + k]
                o += k
        if not cols and not pairs:
            cols = list(m.info.x)
        dest = _unquote(p.get("destination_key")) or dkv.new_key("PDP")

        def run():
            res = explain.partial_plot(m, fr, cols, nbins, targets, bool(p.get("add_missing_na")), splits,
                                       weight_column=wc, row_index=row_index, col_pairs_2dpdp=pairs)
            tables = []
            for name, rows in res.items():
                parts = name.split("|")
                two = any("value2" in r for r in rows)
                cc = parts[:2] if two else parts[:1]
                tcols = []
                for c in cc:
                    tcols.append((c, "string" if fr.type(c) == "enum" else "double", "%s" if fr.type(c) == "enum" else "%5f"))
                tcols += [("mean_response", "double", "%5f"), ("stddev_response", "double", "%5f"),
                          ("std_error_mean_response", "double", "%5f")]
                data = [([r["value"], r["value2"]] if two else [r["value"]]) +
                        [r["mean_response"], r["stddev_response"], r["std_error_mean_response"]] for r in rows]
                title = ("2D-PartialDependence" if two else "PartialDependence")
                desc = f"Partial Dependence Plot of model {m.key} on column '{cc[0]}'" + (
                    f" and class {parts[-1]}" if targets else "")
                tables.append(v3.twodim(title, tcols, data, desc))
            dkv.put(dest, {"__pdp__": True, "model_id": m.key, "frame_id": fr.frame_id, "tables": tables,
                           "cols": cols, "nbins": nbins, "row_index": row_index, "targets": targets})
            return dest
        job = done_job(dest, "PartialDependencePlot", run)
        return {"__meta": v3.meta("JobV3", "Job"), "job": v3.job(job), **v3.job(job)}

    @app.get("/3/PartialDependence/{name}")
    def pdp_get(name: str):
        r = dkv.get(name)
        if not isinstance(r, dict) or not r.get("__pdp__"):
            raise KeyError(f"Object '{name}' not found for argument: key")
        return {"__meta": v3.meta("PartialDependenceV3", "PartialDependence"), "model_id": v3.model_key(r["model_id"]),
                "frame_id": v3.frame_key(r["frame_id"]), "row_index": r["row_index"], "cols": r["cols"],
                "nbins": r["nbins"], "targets": r["targets"], "destination_key": v3.key(name, "Key<PartialDependence>"),
                "partial_dependence_data": r["tables"]}

    @app.post("/3/FeatureInteraction")
    async def feature_interaction(request: Request):
        """hex/FeatureInteractions.java: xgbfi tables per depth, leaf statistics, split-value histograms."""
        from .. import explain
        p = await _params(request)
        m = get_model(p.get("model_id"))
        r = explain.feature_interaction(m, int(p.get("max_interaction_depth", 100)), int(p.get("max_tree_depth", 100)),
                                        int(p.get("max_deepening", -1)))
        cols = [("Interaction", "string", "%s"), ("Gain", "double", "%.5f"), ("FScore", "double", "%.5f"),
                ("wFScore", "double", "%.5f"), ("Average wFScore", "double", "%.5f"), ("Average Gain", "double", "%.5f"),
                ("Expected Gain", "double", "%.5f"), ("Gain Rank", "int", "%d"), ("FScore Rank", "int", "%d"),
                ("wFScore Rank", "int", "%d"), ("Avg wFScore Rank", "int", "%d"), ("Avg Gain Rank", "int", "%d"),
                ("Expected Gain Rank", "int", "%d"), ("Average Rank", "double", "%.5f"),
                ("Average Tree Index", "double", "%.5f"), ("Average Tree Depth", "double", "%.5f")]
        tables = [v3.twodim(f"Interaction Depth {d}", cols, [[row[c[0]] for c in cols] for row in rows])
                  for d, rows in enumerate(r["tables"])]
        lcols = [("Interaction", "string", "%s"), ("Sum Leaf Values Left", "double", "%.5f"),
                 ("Sum Leaf Values Right", "double", "%.5f"), ("Sum Leaf Covers Left", "double", "%.5f"),
                 ("Sum Leaf Covers Right", "double", "%.5f")]
        tables.append(v3.twodim("Leaf Statistics", lcols, [[row[c[0]] for c in lcols] for row in r["leaf_statistics"]]))
        for name, h in r["split_value_histograms"].items():
            tables.append(v3.twodim(f"{name} Split Value Histogram", [("Split Value", "double", "%.5f"), ("Count", "int", "%d")],
                                    [[k, v] for k, v in h.items()]))
        return {"__meta": v3.meta("FeatureInteractionV3", "FeatureInteraction"), "model_id": v3.model_key(m.key),
                "max_interaction_depth": int(p.get("max_interaction_depth", 100)),
                "max_tree_depth": int(p.get("max_tree_depth", 100)), "max_deepening": int(p.get("max_deepening", -1)),
                "feature_interaction": tables}

    @app.post("/3/FriedmansPopescusH")
    async def friedman_h(request: Request):
        from .. import explain
        p = await _params(request)
        m, fr = get_model(p.get("model_id")), get_frame(p.get("frame"))
        variables = as_list(p.get("variables"))
        return {"__meta": v3.meta("FriedmanPopescusHV3", "FriedmansPopescusH"), "model_id": v3.model_key(m.key),
                "frame": v3.frame_key(fr.frame_id), "variables": variables, "h": v3.num(explain.h(m, fr, variables))}

    @app.post("/3/SignificantRules")
    async def significant_rules(request: Request):
        p = await _params(request)
        m = get_model(p.get("model_id"))
        if m.algo != "rulefit":
            raise ValueError("SignificantRules is available for RuleFit models only")
        rows = m.rule_importance() or []
        keys = [k for k in ("variable", "coefficient", "support", "rule") if rows and k in rows[0]] or \
            (list(rows[0]) if rows else ["variable", "coefficient", "support", "rule"])
        cols = [(k, "double" if k in ("coefficient", "support") else "string", "%.5f" if k in ("coefficient", "support") else "%s")
                for k in keys]
        return {"__meta": v3.meta("SignificantRulesV3", "SignificantRules"), "model_id": v3.model_key(m.key),
                "significant_rules_table": v3.twodim("Rule Importance", cols, [[r.get(k) for k in keys] for r in rows])}

    @app.get("/3/Tree")
    def tree(model: str, tree_number: int, tree_class: str | None = None, plain_language_rules: str = "AUTO"):
        """hex/tree/TreeHandler.java: one tree as breadth-first node arrays."""
        return tree_json(get_model(model), tree_number, _unquote(tree_class), plain_language_rules)

    # ------------------------------------------------------------------------- frame transforms
    @app.post("/3/Interaction")
    async def interaction(request: Request):
        from ..frame_ops import interaction as inter
        p = await _params(request)
        fr = get_frame(p.get("source_frame"))
        dest = _unquote(p.get("dest")) or dkv.new_key("interaction")
        factors = as_list(p.get("factor_columns"))

        def run():
            out = inter(fr, factors, bool(p.get("pairwise")), int(p.get("max_factors") or 100),
                        int(p.get("min_occurrence") or 1))
            out.frame_id = dest
            dkv.put(dest, out)
            return dest
        job = done_job(dest, "Interactions", run)
        return {"__meta": v3.meta("JobV3", "Job"), "job": v3.job(job), **v3.job(job)}

    @app.post("/3/MissingInserter")
    async def missing_inserter(request: Request):
        """water/api/MissingInserterHandler: NAs inserted in place into ``dataset``."""
        from ..frame_ops import insert_missing_values
        p = await _params(request)
        fid = _unquote(p.get("dataset"))
        fr = get_frame(fid)

        def run():
            out = insert_missing_values(fr, float(p.get("fraction") or 0.1), p.get("seed"))
            for n in out.names:
                fr._cols[n] = out._col(n)
            return fid
        job = done_job(fid, "MissingInserter", run)
        return v3.job(job)

    @app.post("/99/DCTTransformer")
    async def dct_transformer(request: Request):
        from ..models.dct import dct
        p = await _params(request)
        fr = get_frame(p.get("dataset"))
        dest = _unquote(p.get("destination_frame")) or dkv.new_key("dct")
        dims = [int(v) for v in (p.get("dimensions") or [fr.ncols, 1, 1])]

        def run():
            out = dct(fr, dims, bool(p.get("inverse")))
            out.frame_id = dest
            dkv.put(dest, out)
            return dest
        job = done_job(dest, "DCTTransformer", run)
        return {"__meta": v3.meta("JobV3", "Job"), "job": v3.job(job), **v3.job(job)}

    @app.post("/99/Tabulate")
    async def tabulate(request: Request):
        """hex/Tabulate.java: co-occurrence counts and mean response of (predictor bin, response bin)."""
        p = await _params(request)
        fr = get_frame(p.get("dataset"))
        pc, rc = _unquote(p.get("predictor")), _unquote(p.get("response"))
        wc = _unquote(p.get("weight"))
        nbp, nbr = int(p.get("nbins_predictor") or 20), int(p.get("nbins_response") or 10)

        def bins(c, nb):
            col = fr._col(c)
            if col.type == "enum":
                codes = col.data.long().cpu().numpy()
                return codes, list(col.domain)
            v = col.as_float().double().cpu().numpy()
            lo, hi = np.nanmin(v), np.nanmax(v)
            edges = np.linspace(lo, hi, nb + 1)
            b = np.clip(np.searchsorted(edges, v, side="right") - 1, 0, nb - 1)
            b = np.where(np.isnan(v), -1, b)
            return b, [float(x) for x in edges[:-1]]
        bp, lp = bins(pc, nbp)
        br, lr = bins(rc, nbr)
        w = fr._col(wc).as_float().double().cpu().numpy() if wc else np.ones(len(bp))
        ok = (bp >= 0) & (br >= 0)
        cnt = np.zeros((len(lp), len(lr)))
        np.add.at(cnt, (bp[ok], br[ok]), w[ok])
        rv = fr._col(rc)
        yv = rv.data.double().cpu().numpy() if rv.type == "enum" else rv.as_float().double().cpu().numpy()
        resp = np.zeros(len(lp))
        sw = np.zeros(len(lp))
        np.add.at(resp, bp[ok], (w * yv)[ok])
        np.add.at(sw, bp[ok], w[ok])
        ctab = v3.twodim("(Weighted) co-occurrence counts", [(pc, "string", "%s"), (rc, "string", "%s"),
                                                              ("counts", "double", "%f")],
                         [[str(lp[i]), str(lr[j]), cnt[i, j]] for i in range(len(lp)) for j in range(len(lr))])
        rtab = v3.twodim("Mean value of response vs predictor", [(pc, "string", "%s"), ("mean " + rc, "double", "%f")],
                         [[str(lp[i]), resp[i] / sw[i] if sw[i] > 0 else float("nan")] for i in range(len(lp))])
        return {"__meta": v3.meta("TabulateV3", "Tabulate"), "dataset": v3.frame_key(fr.frame_id), "predictor": pc,
                "response": rc, "weight": wc, "nbins_predictor": nbp, "nbins_response": nbr,
                "count_table": ctab, "response_table": rtab}

    @app.post("/3/ParseSVMLight")
    async def parse_svmlight_ep(request: Request):
        from ..io.parse import parse_svmlight
        p = await _params(request)
        srcs = as_list(p.get("source_frames"))
        dest = _unquote(p.get("destination_frame")) or dkv.new_key("svmlight")

        def run():
            with open(srcs[0], "rb") as f:
                out = parse_svmlight(f.read())
            out.frame_id = dest
            dkv.put(dest, out)
            return dest
        job = done_job(dest, "Parse", run)
        return {"__meta": v3.meta("JobV3", "Job"), "job": v3.job(job), **v3.job(job)}

    # ------------------------------------------------------------------------- GLM / W2V helpers
    @app.get("/3/GetGLMRegPath")
    def glm_reg_path(model: str):
        m = get_model(model)
        rp = m.output.get("regularization_path") or {}
        names = list(rp.get("coefficient_names") or [])
        def rows(key):
            out = []
            for c in rp.get(key) or []:
                if isinstance(c, dict):
                    out.append([float(c.get(n, 0.0)) for n in names])
                elif c is None:
                    out.append([float("nan")] * len(names))
                else:
                    out.append([float(x) for x in np.asarray(c, dtype=np.float64).ravel()[:len(names)]])
            return out
        coefs = rows("coefficients")
        coefs_std = rows("coefficients_std") or None
        return {"__meta": v3.meta("GLMRegularizationPathV3", "RegularizationPath"), "model": v3.model_key(m.key),
                "lambdas": rp.get("lambdas") or [], "alphas": rp.get("alphas") or [],
                "explained_deviance_train": [v3.num(x) if x is not None else "NaN" for x in rp.get("explained_deviance_train") or []],
                "explained_deviance_valid": rp.get("explained_deviance_valid"), "coefficient_names": names,
                "coefficients": coefs, "coefficients_std": coefs_std, "z_values": None, "p_values": None, "std_errs": None}

    @app.post("/3/MakeGLMModel")
    async def make_glm(request: Request):
        from ..models.glm import make_glm_model
        p = await _params(request)
        m = get_model(p.get("model"))
        names = as_list(p.get("names"))
        beta = [float(v) for v in (p.get("beta") or [])]
        nm = make_glm_model(m, dict(zip(names, beta)))
        nm.key = _unquote(p.get("dest")) or dkv.new_key(f"{m.key}_modified")
        if p.get("threshold") is not None:
            nm.output["default_threshold"] = float(p.get("threshold"))
        dkv.put(nm.key, nm)
        return _model_json(nm)

    @app.get("/3/ComputeGram")
    def compute_gram(X: str, W: str | None = None, use_all_factor_levels: bool = False, standardize: bool = True,
                     skip_missing: bool = False):
        """hex/api/MakeGLMModelHandler.computeGram: weighted Gram of the expanded design (with intercept)."""
        from ..models.base import DataInfo
        from ..models.datainfo import Expander
        fr = get_frame(X)
        xs = [n for n in fr.names if n != W]
        info = DataInfo(xs, np.array([1 if fr.type(n) == "enum" else 0 for n in xs], np.int32),
                        [list(fr._col(n).domain) if fr.type(n) == "enum" else None for n in xs])
        Xm, _ = fr.model_matrix(info)
        ex = Expander(info, standardize=standardize, use_all_factor_levels=use_all_factor_levels).fit(Xm)
        Z = ex.transform(Xm).double()
        w = fr._col(W).as_float().double() if W else torch.ones(Z.shape[0], dtype=torch.float64, device=Z.device)
        if skip_missing:
            ok = ~torch.isnan(Z).any(1)
            Z, w = Z[ok], w[ok]
        Zi = torch.cat([Z, torch.ones(Z.shape[0], 1, dtype=Z.dtype, device=Z.device)], 1)
        G = (Zi * w[:, None]).T @ Zi
        names = ex.names + ["Intercept"]
        dest = dkv.new_key("gram")
        out = H2OFrame({n: G[:, i].cpu().tolist() for i, n in enumerate(names)})
        out.frame_id = dest
        dkv.put(dest, out)
        return {"__meta": v3.meta("GramV3", "Gram"), "X": v3.frame_key(fr.frame_id), "destination_frame": v3.frame_key(dest)}

    @app.post("/3/DataInfoFrame")
    async def data_info_frame(request: Request):
        """The expanded design matrix (one-hot / standardised) as a frame (hex/api/DataInfoFrameHandler)."""
        from ..models.base import DataInfo
        from ..models.datainfo import Expander
        p = await _params(request)
        fr = get_frame(p.get("frame"))
        xs = list(fr.names)
        info = DataInfo(xs, np.array([1 if fr.type(n) == "enum" else 0 for n in xs], np.int32),
                        [list(fr._col(n).domain) if fr.type(n) == "enum" else None for n in xs])
        Xm, _ = fr.model_matrix(info)
        ex = Expander(info, standardize=bool(p.get("standardize")), use_all_factor_levels=bool(p.get("use_all", True))).fit(Xm)
        Z = ex.transform(Xm).double()
        dest = dkv.new_key("datainfo")
        out = H2OFrame({n: Z[:, i].cpu().tolist() for i, n in enumerate(ex.names)})
        out.frame_id = dest
        dkv.put(dest, out)
        return {"__meta": v3.meta("DataInfoFrameV3", "DataInfoFrame"), "frame": v3.frame_key(fr.frame_id),
                "result": v3.frame_key(dest)}

    @app.get("/3/Word2VecSynonyms")
    def w2v_synonyms(model: str, word: str, count: int = 20):
        m = get_model(model)
        syn = m.find_synonyms(word, count)
        return {"__meta": v3.meta("Word2VecSynonymsV3", "Word2VecSynonyms"), "model": v3.model_key(m.key),
                "word": word, "count": count, "synonyms": list(syn), "scores": list(syn.values())}

    @app.get("/3/Word2VecTransform")
    def w2v_transform(model: str, words_frame: str, aggregate_method: str = "NONE"):
        m = get_model(model)
        out = m.transform(get_frame(words_frame), aggregate_method)
        dest = dkv.new_key("w2v_transform")
        out.frame_id = dest
        dkv.put(dest, out)
        return {"__meta": v3.meta("Word2VecTransformV3", "Word2VecTransform"), "model": v3.model_key(m.key),
                "words_frame": v3.frame_key(words_frame), "vectors_frame": v3.frame_key(dest)}

    @app.get("/3/TargetEncoderTransform")
    def te_transform(request: Request):
        """TargetEncoderHandler.transform (h2o-extensions/target-encoder .../TargetEncoderHandler.java:14-37):
        blending / inflection_point / smoothing / noise not given (or inflection_point, smoothing < 0, noise < -1)
        keep the model's values; returns the transformed frame's key."""
        q = {k: _unquote(v) for k, v in request.query_params.items()}
        m = get_model(q["model"])
        fr = get_frame(q["frame"])
        tb = lambda v: str(v).lower() in ("true", "1")     # noqa: E731
        kw = dict(as_training=tb(q.get("as_training", "false")))
        if "blending" in q:
            kw["blending"] = tb(q["blending"])
        for k in ("inflection_point", "smoothing"):
            if k in q and float(q[k]) >= 0:
                kw[k] = float(q[k])
        if "noise" in q and float(q["noise"]) >= -1:
            kw["noise"] = float(q["noise"])
        out = m.transform(fr, **kw)
        dest = dkv.new_key("te_transform")
        out.frame_id = dest
        dkv.put(dest, out)
        return v3.frame_key(dest)

    # ------------------------------------------------------------------------- persistence
    @app.get("/3/Models.fetch.bin/{mid}")
    def fetch_bin(mid: str):
        """Binary model download (h2o.download_model)."""
        from ..persist import save_model
        m = get_model(mid)
        d = tempfile.mkdtemp(prefix="h2o_fetch_")
        path = save_model(m, d, True)
        return FileResponse(path, filename=os.path.basename(path),
                            headers={"Content-Disposition": f'attachment; filename="{os.path.basename(path)}"'})

    @app.post("/99/Models.upload.bin/{mid}")
    @app.post("/99/Models.upload.bin/")
    async def upload_bin(request: Request, mid: str = ""):
        """h2o.upload_model: the file arrived through /3/PostFile.bin; ``dir`` is its server-side path."""
        from ..persist import load_model
        p = await _params(request)
        m = load_model(_unquote(p["dir"]))
        if mid:
            dkv.remove(m.key)
            m.key = mid
            dkv.put(mid, m)
        return {"__meta": v3.meta("ModelsV99", "Models", 99), "models": [_model_json(m)]}

    @app.post("/99/Models.bin/{mid}")
    async def save_bin_post(mid: str, request: Request):
        from ..persist import save_model
        p = await _params(request)
        return {"__meta": v3.meta("ModelExportV3", "ModelExport"), "model_id": v3.model_key(mid),
                "dir": save_model(get_model(mid), _unquote(p.get("dir")) or tempfile.gettempdir(), bool(p.get("force", True)))}

    @app.get("/99/Models.mojo/{mid}")
    def save_mojo_get(mid: str, dir: str = "", force: bool = True):
        from ..mojo.writer import write_mojo
        m = get_model(mid)
        path = dir if dir.endswith(".zip") else os.path.join(dir or tempfile.gettempdir(), f"{mid}.zip")
        if os.path.exists(path) and not force:
            raise ValueError(f"{path} exists (force=False)")
        write_mojo(m, path)
        return {"__meta": v3.meta("ModelExportV3", "ModelExport"), "model_id": v3.model_key(mid), "dir": path}

    @app.get("/99/Models/{mid}/json")
    def model_json_export(mid: str):
        return {"__meta": v3.meta("ModelsV99", "Models", 99), "models": [_model_json(get_model(mid))]}

    @app.post("/3/Grid.bin/{gid}/export")
    async def grid_export(gid: str, request: Request):
        from h2o._more import save_grid
        p = await _params(request)
        path = save_grid(_unquote(p.get("grid_directory")) or tempfile.gettempdir(), gid,
                         export_cross_validation_predictions=bool(p.get("export_cross_validation_predictions")))
        return {"__meta": v3.meta("GridExportV3", "GridExport"), "grid_id": v3.key(gid, "Key<Grid>"), "grid_directory": path}

    @app.post("/3/Grid.bin/import")
    async def grid_import(request: Request):
        from h2o._more import load_grid
        p = await _params(request)
        g = load_grid(_unquote(p.get("grid_path")), bool(p.get("load_params_references")))
        gid = getattr(g, "grid_id", None) or getattr(g, "key", None)
        return {"__meta": v3.meta("GridKeyV3", "Key<Grid>"), "name": gid, "type": "Key<Grid>"}

    @app.post("/3/Frames/{fid}/save")
    async def frame_save(fid: str, request: Request):
        from ..io.parse import save_frame
        p = await _params(request)
        d = _unquote(p.get("dir")) or tempfile.gettempdir()
        fr = get_frame(fid)
        job = done_job(fid, "Frame save", lambda: save_frame(fr, d, bool(p.get("force", True))))
        return {"__meta": v3.meta("FrameSaveV3", "FrameSave"), "frame_id": v3.frame_key(fid), "dir": d, "job": v3.job(job)}

    @app.post("/3/Frames/load")
    async def frame_load(request: Request):
        from ..io.parse import load_frame
        p = await _params(request)
        fid = _unquote(p.get("frame_id"))
        d = _unquote(p.get("dir"))

        def run():
            fr = load_frame(fid, d)
            dkv.put(fid, fr)
            return fid
        job = done_job(fid, "Frame load", run)
        return {"__meta": v3.meta("FrameLoadV3", "FrameLoad"), "frame_id": v3.frame_key(fid), "dir": d, "job": v3.job(job)}

    @app.get("/3/Frames/{fid}/export/{path:path}/overwrite/{force}")
    def frame_export_get(fid: str, path: str, force: str):
        from ..io.parse import export_file
        fr = get_frame(fid)
        export_file(fr, path, force=str(force).lower() == "true")
        job = done_job(fid, "Export")
        return {"__meta": v3.meta("FramesV3", "Frames"), "frame_id": v3.frame_key(fid), "path": path,
                "force": str(force).lower() == "true", "job": v3.job(job)}

    # ------------------------------------------------------------------------- node persistent storage
    nps_root = os.path.join(tempfile.gettempdir(), "h2o_nps")

    def nps_path(cat, name=None):
        d = os.path.join(nps_root, os.path.basename(cat))
        return d if name is None else os.path.join(d, os.path.basename(name))

    @app.get("/3/NodePersistentStorage/configured")
    def nps_configured():
        return {"__meta": v3.meta("NodePersistentStorageV3", "NodePersistentStorage"), "configured": True}

    @app.get("/3/NodePersistentStorage/categories/{cat}/exists")
    def nps_cat_exists(cat: str):
        return {"__meta": v3.meta("NodePersistentStorageV3", "NodePersistentStorage"), "category": cat,
                "exists": os.path.isdir(nps_path(cat))}

    @app.get("/3/NodePersistentStorage/categories/{cat}/names/{name}/exists")
    def nps_exists(cat: str, name: str):
        return {"__meta": v3.meta("NodePersistentStorageV3", "NodePersistentStorage"), "category": cat, "name": name,
                "exists": os.path.isfile(nps_path(cat, name))}

    @app.get("/3/NodePersistentStorage/{cat}")
    def nps_list(cat: str):
        d = nps_path(cat)
        entries = []
        for f in sorted(glob.glob(os.path.join(d, "*"))):
            st = os.stat(f)
            entries.append({"category": cat, "name": os.path.basename(f), "size": st.st_size,
                            "timestamp_millis": int(st.st_mtime * 1000)})
        return {"__meta": v3.meta("NodePersistentStorageV3", "NodePersistentStorage"), "category": cat, "entries": entries}

    @app.get("/3/NodePersistentStorage/{cat}/{name}")
    def nps_get(cat: str, name: str):
        with open(nps_path(cat, name)) as f:
            return {"__meta": v3.meta("NodePersistentStorageV3", "NodePersistentStorage"), "category": cat,
                    "name": name, "value": f.read()}

    @app.post("/3/NodePersistentStorage/{cat}")
    @app.post("/3/NodePersistentStorage/{cat}/{name}")
    async def nps_put(cat: str, request: Request, name: str | None = None):
        p = await _params(request)
        name = name or dkv.new_key("nps")
        os.makedirs(nps_path(cat), exist_ok=True)
        with open(nps_path(cat, name), "w") as f:
            v = p.get("value", "")      # JSON-looking values arrive parsed: store them as JSON text again
            f.write(v if isinstance(v, str) else json.dumps(v))
        return {"__meta": v3.meta("NodePersistentStorageV3", "NodePersistentStorage"), "category": cat, "name": name}

    @app.delete("/3/NodePersistentStorage/{cat}/{name}")
    def nps_del(cat: str, name: str):
        if os.path.isfile(nps_path(cat, name)):
            os.remove(nps_path(cat, name))
        return {"__meta": v3.meta("NodePersistentStorageV3", "NodePersistentStorage"), "category": cat, "name": name}

    # ------------------------------------------------------------------------- metadata / diagnostics
    @app.get("/3/Typeahead/files")
    def typeahead(src: str = "", limit: int = 1000):
        hits = sorted(glob.glob((src or ".") + "*"))[: max(int(limit), 0) or 1000]
        return {"__meta": v3.meta("TypeaheadV3", "Typeahead"), "src": src, "limit": limit, "matches": hits}

    @app.get("/3/Metadata/schemas")
    def schemas():
        return {"__meta": v3.meta("MetadataV3", "Metadata"),
                "schemas": [v3.schema_metadata(n)["schemas"][0] for n in sorted(v3.SCHEMA_FIELDS)]}

    @app.get("/3/Metadata/schemaclasses/{classname}")
    def schema_class(classname: str):
        return v3.schema_metadata(classname)

    @app.get("/3/Metadata/endpoints/{path:path}")
    def endpoint_meta(path: str):
        routes = [r for r in app.routes if getattr(r, "path", "").strip("/") == path.strip("/")
                  or str(getattr(r, "name", "")) == path]
        return {"__meta": v3.meta("MetadataV3", "Metadata"),
                "routes": [{"http_method": sorted(getattr(r, "methods", []) or ["GET"])[0], "url_pattern": r.path,
                            "summary": (getattr(r, "endpoint", None).__doc__ or "").strip().split("\n")[0]
                            if getattr(r, "endpoint", None) else ""} for r in routes]}

    @app.get("/99/Rapids/help")
    def rapids_help():
        from ..rapids import Session
        return {"__meta": v3.meta("RapidsHelpV3", "RapidsHelp"), "syntax": sorted(Session().prims)}

    @app.get("/99/Grids")
    def grids():
        from ..grid import Grid
        gs = [k for k, v in dkv.items() if isinstance(v, Grid)]
        return {"__meta": v3.meta("GridsV99", "Grids", 99), "grids": [{"grid_id": v3.key(g, "Key<Grid>")} for g in gs]}

    @app.get("/99/Leaderboards")
    def leaderboards(project_name: str | None = None):
        from ..automl import AutoML
        out = []
        for k, v in dkv.items():
            if isinstance(v, AutoML) and (project_name is None or k == project_name):
                rows, cols = v.leaderboard_rows()
                out.append({"project_name": k, "models": [v3.model_key(r["model_id"]) for r in rows]})
        return {"__meta": v3.meta("LeaderboardsV99", "Leaderboards", 99), "leaderboards": out}

    @app.post("/3/ModelBuilders/{algo}/model_id")
    def new_model_id(algo: str):
        from ..models import builder
        return {"__meta": v3.meta("ModelIdV3", "ModelId"), "model_id": builder.make_key(algo)}

    @app.post("/3/ModelMetrics/predictions_frame/{pf}/actuals_frame/{af}")
    async def metrics_from_predictions(pf: str, af: str, request: Request):
        """h2o.make_metrics: metrics straight from a predictions frame and an actuals frame."""
        from .. import metrics as mm
        p = await _params(request)
        pred, act = get_frame(pf), get_frame(af)
        dom = as_list(p.get("domain")) or None
        dist = str(_unquote(p.get("distribution")) or "gaussian")
        wts = get_frame(p["weights_frame"])._col(0).as_float().double() if p.get("weights_frame") else None
        cat = "Regression" if not dom else ("Binomial" if len(dom) == 2 else "Multinomial")
        ac = act._col(0)
        if ac.type == "enum" and dom:
            lut = {s: i for i, s in enumerate(dom)}
            y = torch.tensor([float(lut.get(ac.domain[int(c)], -1)) if c >= 0 else float("nan")
                              for c in ac.data.long().cpu().tolist()], dtype=torch.float64)
        else:
            y = ac.as_float().double().cpu()
        P = torch.stack([pred._col(n).as_float().double().cpu() for n in pred.names], 1)
        if cat == "Binomial":
            P = P[:, -1]
        elif cat == "Multinomial":
            P = P[:, -len(dom):]
        else:
            P = P[:, 0]
        res = mm.make_metrics(cat, y, P, None if wts is None else wts.cpu(), dom, dist)
        return {"__meta": v3.meta("ModelMetricsMakerSchemaV3", "ModelMetricsMaker"),
                "predictions_frame": pf, "actuals_frame": af, "model_metrics": v3.metrics(res, cat, None, af)}

    @app.delete("/3/ModelMetrics")
    @app.delete("/3/ModelMetrics/models/{mid}")
    @app.delete("/3/ModelMetrics/models/{mid}/frames/{fid}")
    @app.delete("/3/ModelMetrics/frames/{fid}")
    @app.delete("/3/ModelMetrics/frames/{fid}/models/{mid}")
    def metrics_delete(mid: str | None = None, fid: str | None = None):
        n = 0
        for k, v in dkv.items():
            if isinstance(v, Model) and (mid is None or k == mid):
                perf = getattr(v, "_perf_cache", None)
                if isinstance(perf, dict):
                    for key in [q for q in perf if fid is None or q == fid]:
                        perf.pop(key, None)
                        n += 1
        return {"__meta": v3.meta("ModelMetricsListSchemaV3", "ModelMetricsList"), "model_metrics": [], "deleted": n}

    @app.delete("/3/InitID")
    def end_session_id():
        return {"__meta": v3.meta("InitIDV3", "InitID"), "session_key": ""}

    @app.get("/3/Capabilities/API")
    @app.get("/3/Capabilities/Core")
    def capabilities_kind():
        return {"__meta": v3.meta("CapabilitiesV3", "Capabilities"),
                "capabilities": [{"name": n} for n in ("Algos", "AutoML", "Core", "MOJO", "REST", "Rapids", "HIP")]}

    @app.get("/3/NetworkTest")
    def network_test():
        """water/init/NetworkTest: collective latency/bandwidth of this cloud (one node here unless the
        process group is up)."""
        from ..parallel import collectives as coll
        sizes = [1, 1 << 10, 1 << 20]
        lat, bw = [], []
        for s in sizes:
            t = torch.zeros(max(s // 8, 1), dtype=torch.float64)
            t0 = time.perf_counter()
            if coll.world_active():
                coll.all_reduce_(t)
            dt = max(time.perf_counter() - t0, 1e-9)
            lat.append(dt * 1e6)
            bw.append(s / dt)
        table = v3.twodim("Network Test", [("msg_size", "long", "%d"), ("latency_us", "double", "%.3f"),
                                           ("bandwidth_Bps", "double", "%.1f")],
                          [[s, a, b] for s, a, b in zip(sizes, lat, bw)])
        return {"__meta": v3.meta("NetworkTestV3", "NetworkTest"), "msg_sizes": sizes, "microseconds_collective": lat,
                "bandwidths_collective": bw, "table": table, "nodes": ["127.0.0.1"]}

    @app.get("/3/JStack")
    def jstack():
        import sys
        import threading
        import traceback
        frames = sys._current_frames()
        traces = [{"thread": t.name, "stack": "".join(traceback.format_stack(frames.get(t.ident)))
                   if frames.get(t.ident) else ""} for t in threading.enumerate()]
        return {"__meta": v3.meta("JStackV3", "JStack"), "traces": [{"node": "127.0.0.1", "time": int(time.time() * 1000),
                                                                    "thread_traces": [t["thread"] + "\n" + t["stack"] for t in traces]}]}

    @app.get("/3/Find")
    def find(key: str, column: str | None = None, row: int = 0, match: str = ""):
        fr = get_frame(key)
        cols = [column] if column else fr.names
        for c in cols:
            vals = fr._col(c).to_numpy() if fr._col(c).type != "string" else fr._col(c).strings
            dom = fr._col(c).domain
            for i in range(int(row), len(vals)):
                v = vals[i]
                s = dom[int(v)] if dom is not None and v == v and v is not None and int(v) >= 0 else str(v)
                if s == match:
                    return {"__meta": v3.meta("FindV3", "Find"), "key": v3.frame_key(key), "column": c, "row": i,
                            "match": match, "prev": -1, "next": i}
        return {"__meta": v3.meta("FindV3", "Find"), "key": v3.frame_key(key), "column": column, "row": row,
                "match": match, "prev": -1, "next": -1}

    @app.get("/3/FrameChunks/{fid}")
    def frame_chunks(fid: str):
        fr = get_frame(fid)
        sh = getattr(fr, "_shard", None)
        n = fr._nlocal
        return {"__meta": v3.meta("FrameChunksV3", "FrameChunks"), "frame_id": v3.frame_key(fid),
                "chunks": [{"chunk_id": 0, "row_count": n, "node_idx": 0 if sh is None else sh.offset}]}

    @app.get("/3/WaterMeterCpuTicks/{nodeidx}")
    def cpu_ticks(nodeidx: int):
        t = os.times()
        return {"__meta": v3.meta("WaterMeterCpuTicksV3", "WaterMeterCpuTicks"), "nodeidx": nodeidx,
                "cpu_ticks": [[int(t.user * 100), int(t.system * 100), 0, int(t.elapsed * 100)]]}

    @app.get("/3/WaterMeterIo")
    @app.get("/3/WaterMeterIo/{nodeidx}")
    def io_meter(nodeidx: int = -1):
        return {"__meta": v3.meta("WaterMeterIoV3", "WaterMeterIo"), "nodeidx": nodeidx, "persist_stats": []}

    @app.get("/3/SteamMetrics")
    def steam_metrics():
        return {"__meta": v3.meta("SteamMetricsV3", "SteamMetrics"), "version": 0, "idle_millis": 0}

    @app.get("/99/Sample")
    def sample():
        return {"__meta": v3.meta("CloudV3", "Cloud"), "note": "sample endpoint"}

    @app.post("/3/CloudLock")
    async def cloud_lock(request: Request):
        p = await _params(request)
        return {"__meta": v3.meta("CloudLockV3", "CloudLock"), "reason": p.get("reason", "")}

    @app.post("/3/UnlockKeys")
    def unlock_keys():
        n = 0
        for k in list(getattr(dkv, "_locks", {}) or {}):
            try:
                dkv._locks.pop(k, None)
                n += 1
            except Exception:  # noqa: BLE001
                pass
        return {"__meta": v3.meta("UnlockKeysV3", "UnlockKeys"), "unlocked": n}

    @app.get("/3/KillMinus3")
    def kill_minus3():
        return PlainTextResponse("thread dump written to the server log")

    # endpoints of the Java cluster that have no meaning for this engine answer with an H2OError naming why
    @app.post("/3/DecryptionSetup")
    async def decryption_setup(request: Request):
        """DecryptionSetupHandler.setupDecryption: build the tool from the keystore (a raw file key), install it."""
        from ..io import decrypt as dec
        p = await _params(request)
        ks = p.get("keystore_id")
        ks = ks.get("name") if isinstance(ks, dict) else ks
        setup = dec.DecryptionSetup(keystore_id=_unquote(ks), keystore_type=p.get("keystore_type") or "JCEKS",
                                    key_alias=p.get("key_alias") or "", password=p.get("password") or "",
                                    cipher_spec=p.get("cipher_spec") or "",
                                    decrypt_tool_id=_unquote(p.get("decrypt_tool_id")) or None,
                                    decrypt_impl=p.get("decrypt_impl") or "water.parser.GenericDecryptionTool")
        tool = dec.make_tool(setup)
        return {"__meta": v3.meta("DecryptionSetupV3", "DecryptionSetup"),
                "decrypt_tool_id": {"__meta": v3.meta("DecryptionToolKeyV3", "Key<DecryptionTool>"),
                                    "name": tool.key_id, "type": "Key<DecryptionTool>", "URL": None},
                "decrypt_impl": setup.decrypt_impl, "keystore_id": v3.frame_key(str(setup.keystore_id)),
                "keystore_type": setup.keystore_type, "key_alias": setup.key_alias, "cipher_spec": setup.cipher_spec}

    for meth, path, why in (("POST", "/3/ImportHiveTable", "Hive is not available (single-node MI355X engine)"),
                            ("POST", "/3/SaveToHiveTable", "Hive is not available (single-node MI355X engine)"),
                            # the MOJO 2 pipeline export needs the external mojo2-runtime jar on the Java
                            # classpath in the reference too (h2o-py assembly.py:download_mojo)
                            ("GET", "/99/Assembly.fetch_mojo_pipeline/{aid}/{fname}",
                             "MOJO 2 munging pipelines need the mojo2-runtime library, which this engine does not "
                             "ship; export the assembly as a POJO (/99/Assembly.java)")):
        def make(why=why):
            def h():
                raise NotImplementedError(why)
            return h
        app.add_api_route(path, make(), methods=[meth])

    # ---- munging pipelines (water/api/AssemblyHandler.java, AssemblyV99)
    @app.post("/99/Assembly")
    async def assembly_fit(request: Request):
        from .. import assembly
        from ..core import dkv as _dkv
        p = await _params(request)
        steps = p.get("steps")
        if isinstance(steps, str):
            steps = [steps]
        fid = _unquote(p.get("frame"))
        fr = _dkv.get(fid)
        if fr is None:
            raise KeyError(f"frame {fid} not found")
        asm, out = assembly.fit_rest([_unquote(x) for x in steps or []], fr)
        return {"__meta": v3.meta("AssemblyV99", "Assembly"), "steps": steps, "frame": v3.frame_key(fid),
                "assembly": {"__meta": v3.meta("AssemblyKeyV3", "Key<Assembly>"), "name": asm.key,
                             "type": "Key<Assembly>", "URL": None},
                "result": v3.frame_key(out.frame_id)}

    @app.get("/99/Assembly.java/{aid}/{fname}")
    def assembly_java(aid: str, fname: str):
        from ..core import dkv as _dkv
        asm = _dkv.get(aid)
        if asm is None or not hasattr(asm, "to_java"):
            raise KeyError(f"assembly {aid} not found")
        return PlainTextResponse(asm.to_java(fname))

    @app.post("/99/ImportSQLTable")
    async def import_sql(request: Request):
        from h2o import _more
        p = await _params(request)
        fr = _more.import_sql_table(_unquote(p.get("connection_url")), _unquote(p.get("table")),
                                    _unquote(p.get("username")), _unquote(p.get("password")),
                                    columns=p.get("columns"))
        dest = fr.frame_id
        job = done_job(dest, "ImportSQLTable")
        return {"__meta": v3.meta("JobV3", "Job"), "job": v3.job(job), **v3.job(job)}


def tree_json(m, tree_number: int, tc=None, plain_language_rules: str = "AUTO") -> dict:
    """TreeV3 of one tree of a tree model (hex/tree/TreeHandler.java), breadth-first node arrays; shared by GET
    /3/Tree and the in-process ``h2o.tree.H2OTree``."""
    forest = getattr(m, "forest", None)
    if forest is None:
        raise ValueError(f"model {m.key} has no trees")
    dom = m.info.response_domain
    K = max(int(getattr(forest, "n_classes_out", 1) or 1), 1)
    cls = 0
    if tc not in (None, "", "null") and dom is not None and K > 1:
        if tc not in dom:
            raise ValueError(f"tree_class {tc!r} is not a response level")
        cls = dom.index(tc)
    idx = [i for i, c in enumerate(forest.tree_class) if c == cls]
    if tree_number < 0 or tree_number >= len(idx):
        raise ValueError(f"tree_number must be in [0, {len(idx)})")
    t = forest.trees[idx[tree_number]]
    order, pos = [0], {0: 0}
    i = 0
    while i < len(order):
        n = order[i]
        if t.feat[n] >= 0:
            for c in (int(t.left[n]), int(t.right[n])):
                pos[c] = len(order)
                order.append(c)
        i += 1
    names = m.info.x
    L, R, desc, thr, feats, levels, nas, preds = [], [], [], [], [], [None] * len(order), [], []
    for q, n in enumerate(order):
        if t.feat[n] < 0:
            L.append(-1)
            R.append(-1)
            thr.append("NaN")
            feats.append(None)
            nas.append(None)
            preds.append(float(t.value[n]))
            desc.append(f"Leaf node {n}: prediction {float(t.value[n]):.6g}")
            continue
        f = int(t.feat[n])
        ln, rn = int(t.left[n]), int(t.right[n])
        L.append(pos[ln] + 1000000)          # node ids (opaque to the client): BFS position + offset
        R.append(pos[rn] + 1000000)
        feats.append(names[f])
        nas.append("LEFT" if bool(t.na_left[n]) else "RIGHT")
        preds.append(float("nan"))
        if t.is_cat[n] and t.cat_bits[n] is not None:
            bits = np.asarray(t.cat_bits[n], dtype=np.uint32)
            nb = int(t.cat_nbits[n]) if t.cat_nbits[n] else len(m.info.domains[f] or [])
            left_lv = [lv for lv in range(nb) if (bits[lv >> 5] >> (lv & 31)) & 1]
            right_lv = [lv for lv in range(nb) if not (bits[lv >> 5] >> (lv & 31)) & 1]
            levels[pos[ln]] = left_lv
            levels[pos[rn]] = right_lv
            thr.append("NaN")
            desc.append(f"Node {n}: {names[f]} in left levels; NA {'left' if t.na_left[n] else 'right'}")
        else:
            thr.append(float(t.thr[n]))
            desc.append(f"Node {n}: {names[f]} < {float(t.thr[n]):.6g}; NA {'left' if t.na_left[n] else 'right'}")
    rules = None
    if str(plain_language_rules).upper() == "TRUE" or (str(plain_language_rules).upper() == "AUTO" and len(order) < 64):
        rules = tree_rules(L, R, feats, thr, nas, preds)
    return {"__meta": v3.meta("TreeV3", "Tree"), "model": v3.model_key(m.key), "tree_number": tree_number,
            "tree_class": tc if tc not in ("null",) else None, "left_children": L, "right_children": R,
            "root_node_id": 1000000, "thresholds": thr, "features": feats, "levels": levels, "nas": nas,
            "descriptions": desc, "predictions": [v3.num(v) for v in preds],
            "tree_decision_path": rules, "decision_paths": None if rules is None else [rules] * len(order),
            "plain_language_rules": plain_language_rules}


def tree_rules(L, R, feats, thr, nas, preds):
    lines = []

    def walk(i, conds):
        if L[i] == -1:
            lines.append(("If " + " and ".join(conds) if conds else "Always") + f" then {preds[i]:.6g}")
            return
        ln, rn = L[i] - 1000000, R[i] - 1000000
        t = thr[i]
        if t == "NaN":
            walk(ln, conds + [f"{feats[i]} in left levels"])
            walk(rn, conds + [f"{feats[i]} in right levels"])
        else:
            walk(ln, conds + [f"{feats[i]} < {t:.6g}" + (" or NA" if nas[i] == "LEFT" else "")])
            walk(rn, conds + [f"{feats[i]} >= {t:.6g}" + (" or NA" if nas[i] == "RIGHT" else "")])
    walk(0, [])
    return "\n".join(lines)
