"""RuleFit (reference: ``hex/rulefit/RuleFit.java``, ``RuleFitModel.java``, ``Rule.java``, ``Condition.java``).

1. Rule generation: tree ensembles (DRF by default, or GBM) with depths ``min_rule_length`` ..
   ``max_rule_length``, ``rule_generation_ntrees`` trees in total.
2. Every non-root node of every tree is a rule = conjunction of the conditions on its path; rule
   membership of all rows is computed on device level by level (parent mask & split test).
3. A Lasso GLM (``lambda`` or lambda search, ``alpha``=1) is fit on the 0/1 rule matrix (plus the
   standardized linear terms for ``model_type='rules_and_linear'``); non-zero coefficients form the
   ``rule_importance`` table (rule text, coefficient, support). Duplicate rules are removed.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key

RF_DEFAULTS = dict(algorithm="AUTO", min_rule_length=3, max_rule_length=3, max_num_rules=-1,
                   model_type="rules_and_linear", rule_generation_ntrees=50, remove_duplicates=True, lambda_=None,
                   distribution="AUTO", seed=-1)


def _node_masks(tree, X):
    """Row membership for every node: list (node id -> bool [N]) and condition text per node."""
    N = X.shape[1]
    masks = {0: torch.ones(N, dtype=torch.bool, device=X.device)}
    conds = {0: []}
    order = [0]
    for i in order:
        f = int(tree.feat[i])
        if f < 0:
            continue
        x = X[f]
        na = torch.isnan(x)
        if tree.is_cat[i]:
            words = torch.as_tensor(tree.cat_bits[i].astype(np.int64), device=X.device)
            code = torch.nan_to_num(x, nan=-1).long()
            inr = (code >= 0) & (code < int(tree.cat_nbits[i]))
            bit = (words[(code.clamp(min=0) >> 5).clamp(max=words.numel() - 1)] >> (code.clamp(min=0) & 31)) & 1
            go = torch.where(inr, bit.bool(), torch.full_like(na, bool(tree.na_left[i])))
            cl = ("in", f, tree.cat_bits[i], int(tree.cat_nbits[i]), bool(tree.na_left[i]))
        else:
            go = x < float(tree.thr[i])
            cl = ("<", f, float(tree.thr[i]), bool(tree.na_left[i]))
        go = torch.where(na, torch.full_like(go, bool(tree.na_left[i])), go)
        L, R = int(tree.left[i]), int(tree.right[i])
        masks[L] = masks[i] & go
        masks[R] = masks[i] & ~go
        conds[L] = conds[i] + [(cl, True)]
        conds[R] = conds[i] + [(cl, False)]
        order += [L, R]
    return masks, conds


def _cond_text(c, left, names, domains):
    kind = c[0]
    f = c[1]
    if kind == "<":
        op = "<" if left else ">="
        na = " or NA" if c[3] == left else ""
        return f"({names[f]} {op} {c[2]:.6g}{na})"
    words, nl = c[2], c[3]
    levels = [domains[f][lv] if domains[f] and lv < len(domains[f]) else str(lv)
              for lv in range(nl) if bool((int(words[lv >> 5]) >> (lv & 31)) & 1) == left]
    return f"({names[f]} in {{{', '.join(levels)}}})"


class RuleFitModel(Model):
    algo = "rulefit"

    def _rule_matrix(self, X):
        cols = []
        for ti, nodes in self.rule_nodes:
            masks, _ = _node_masks(self.trees[ti], X)
            for n in nodes:
                cols.append(masks[n].float())
        R = torch.stack(cols, 0) if cols else torch.zeros(0, X.shape[1], device=X.device)
        if self.params.get("model_type", "rules_and_linear") != "rules":
            R = torch.cat([R, X.float()], 0)
        return R

    def _predict_tensor(self, X, offset=None):
        return self.glm._predict_tensor(self._rule_matrix(X.to(self.device)), offset)

    def rule_importance(self):
        return self.output["rule_importance"]

    def predict_rules(self, frame, rule_ids):
        """0/1 column per requested rule: does the row satisfy the rule's conditions (RuleFitModel.predictRules)."""
        from ..frame import Column, H2OFrame
        X, _ = frame.model_matrix(self.info, device=self.device)
        where = {}
        for ti, nodes in self.rule_nodes:
            for n in nodes:
                where[f"M{ti}T{ti}N{n}"] = (ti, n)
        cols, cache = [], {}
        for rid in rule_ids:
            if rid not in where:
                raise ValueError(f"Rule {rid!r} is not part of the model")
            ti, n = where[rid]
            if ti not in cache:
                cache[ti] = _node_masks(self.trees[ti], X)[0]
            cols.append(Column(rid, "int", cache[ti][n].double()))
        return H2OFrame._from_columns(cols)


class RuleFitTrainer:
    def __init__(self, params):
        p = dict(RF_DEFAULTS)
        if "lambda" in params:
            params = dict(params)
            params["lambda_"] = params.pop("lambda")
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .drf import DRFTrainer
        from .gbm import GBMTrainer
        from .glm import GLMTrainer
        t0 = time.time()
        p = self.p
        algo = str(p["algorithm"]).upper()
        lo, hi = int(p["min_rule_length"]), int(p["max_rule_length"])
        depths = list(range(lo, hi + 1))
        per = max(1, int(p["rule_generation_ntrees"]) // len(depths))
        trees = []
        for d in depths:
            kw = dict(ntrees=per, max_depth=d, seed=p["seed"], min_rows=1)
            tr = GBMTrainer(dict(kw, learn_rate=0.1)) if algo == "GBM" else DRFTrainer(kw)
            m = tr.fit(X, y, w, offset, info)
            trees += list(m.forest.trees)
        rule_nodes, seen, rule_text, cols = [], set(), [], []
        for ti, t in enumerate(trees):
            masks, conds = _node_masks(t, X)
            keep = []
            for n in range(1, t.n_nodes):
                text = " & ".join(_cond_text(c, left, info.x, info.domains) for c, left in conds[n])
                if p["remove_duplicates"] and text in seen:
                    continue
                seen.add(text)
                keep.append(n)
                rule_text.append((f"M{ti}T{ti}N{n}", text))
                cols.append(masks[n].float())
            rule_nodes.append((ti, keep))
        R = torch.stack(cols, 0)
        names = [r[0] for r in rule_text]
        iscat = [0] * len(names)
        doms = [None] * len(names)
        Xg = R
        if p["model_type"] != "rules":
            Xg = torch.cat([R, X.float()], 0)
            names = names + [f"linear.{n}" for n in info.x]
            iscat += [0] * info.F
            doms += [None] * info.F
        ginfo = DataInfo(names, np.asarray(iscat, np.int32), doms, info.response, info.response_domain)
        gp = dict(alpha=1.0, standardize=True, seed=p["seed"])
        if p.get("lambda_") is not None:
            gp["lambda_"] = p["lambda_"]
        else:
            gp["lambda_search"] = True
            gp["nlambdas"] = 30
        if info.response_domain is not None and len(info.response_domain) > 2:
            gp["family"] = "multinomial"
            gp["alpha"] = 0.0
        glm = GLMTrainer(gp).fit(Xg, y, w, offset, ginfo, valid and (None if valid is None else None))
        model = RuleFitModel(model_key or make_key("rulefit"), p, info)
        model.device = X.device
        model.trees = trees
        model.rule_nodes = rule_nodes
        model.glm = glm
        coefs = glm.output["coefficients"]
        texts = dict(rule_text)
        support = {r[0]: float(c.mean()) for r, c in zip(rule_text, cols)}
        imp = [dict(variable=k, coefficient=v, rule=texts.get(k, k), support=support.get(k, 1.0))
               for k, v in coefs.items() if k != "Intercept" and v != 0]
        imp.sort(key=lambda r: -abs(r["coefficient"]))
        mx = int(p["max_num_rules"])
        model.output["rule_importance"] = imp[:mx] if mx > 0 else imp
        model.output["training_metrics"] = model.metrics_for(X, y, w, offset)
        if valid is not None:
            Xv, yv, wv, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
