"""RuleFit (reference: ``hex/rulefit/RuleFit.java``, ``RuleFitModel.java``, ``Rule.java``, ``Condition.java``,
``RuleEnsemble.java``, ``RuleFitUtils.java``; scoring as ``hex/genmodel/algos/rulefit/*``).

1. Rule generation: one tree ensemble per depth ``min_rule_length .. max_rule_length`` (DRF by default, or
   GBM), each with ``rule_generation_ntrees`` trees, trained on the device tree engine.
2. Every LEAF of every tree is a rule ``M<model>T<tree>N<node>`` (``_<class>`` per multinomial class tree):
   the conditions on its root path, one per (feature, operator) — the one closest to the leaf — sorted by
   feature name (``Rule.extractRulesFromTree`` / ``traversePath``).
3. The linear model's input has one CATEGORICAL column per tree (``M<i>T<j>``, or ``M<i>T<j>C<k>``) whose
   level is the last rule of that tree the row satisfies (``RuleEnsemble.createGLMTrainFrame`` + ``Decoder``),
   plus ``linear.<x>`` copies of the predictors for ``rules_and_linear`` / ``linear``.
4. A Lasso GLM (alpha 1; ``max_num_rules`` -> ``max_active_predictors``) on that frame; rules with non-zero
   coefficients form ``rule_importance`` (duplicate conditions merged when ``remove_duplicates``).

Rule membership is evaluated on the device for all rows at once (one boolean tensor per condition).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key

RF_DEFAULTS = dict(algorithm="AUTO", min_rule_length=3, max_rule_length=3, max_num_rules=-1,
                   model_type="rules_and_linear", rule_generation_ntrees=50, remove_duplicates=True, lambda_=None,
                   distribution="AUTO", seed=-1, max_categorical_levels=10)


class Condition:
    """One rule condition (``Condition.java``): numeric ``<`` / ``>=`` threshold or categorical ``in`` levels,
    with ``nas_included`` for missing values."""

    def __init__(self, feat, name, ctype, op, thr=-1.0, levels=None, level_names=None, nas=False):
        self.feat, self.name, self.ctype, self.op = int(feat), name, ctype, op
        self.thr = float(thr)
        self.levels = list(levels or [])
        self.level_names = list(level_names or [])
        self.nas = bool(nas)

    def text(self) -> str:
        """Condition.constructLanguageCondition."""
        s = f"({self.name}"
        if self.op == "<":
            s += f" < {_jfloat(self.thr)}"
        elif self.op == ">=":
            s += f" >= {_jfloat(self.thr)}"
        else:
            s += " in {" + ", ".join(self.level_names) + "}"
        if self.nas:
            s += f" or {self.name} is NA"
        return s + ")"

    def holds(self, X: torch.Tensor) -> torch.Tensor:
        """Condition.map over all rows (X [F, N])."""
        x = X[self.feat].double()
        na = torch.isnan(x)
        if self.ctype == "num":
            ok = (x < self.thr) if self.op == "<" else (x >= self.thr)
        else:
            lv = torch.as_tensor(self.levels, dtype=torch.float64, device=x.device)
            ok = (x[:, None] == lv[None, :]).any(1) if lv.numel() else torch.zeros_like(na)
        return torch.where(na, torch.full_like(na, self.nas), ok & ~na)

    def to_state(self):
        return [self.feat, self.name, self.ctype, self.op, self.thr, self.levels, self.level_names, self.nas]

    @staticmethod
    def from_state(s):
        return Condition(*s)


def _jfloat(v: float) -> str:
    """Java ``Double.toString`` (thresholds are float32 split values widened to double)."""
    v = float(v)
    if v != v or v in (float("inf"), float("-inf")):
        return {True: "NaN"}.get(v != v, "Infinity" if v > 0 else "-Infinity")
    if v == 0 or 1e-3 <= abs(v) < 1e7:
        r = repr(v)
        return r if "." in r else r + ".0"
    mant, exp = np.format_float_scientific(v, unique=True, trim="-").split("e")
    if "." not in mant:
        mant += ".0"
    return f"{mant}E{int(exp)}"


class Rule:
    def __init__(self, conds, pred, var, coef=0.0, support=float("nan")):
        self.conds, self.pred, self.var = conds, float(pred), var
        self.coef, self.support = float(coef), float(support)

    def text(self) -> str:
        """Rule.generateLanguageRule."""
        return " & ".join(c.text() for c in self.conds)

    def holds(self, X):
        m = torch.ones(X.shape[1], dtype=torch.bool, device=X.device)
        for c in self.conds:
            m &= c.holds(X)
        return m

    def to_state(self):
        return [[c.to_state() for c in self.conds], self.pred, self.var, self.coef, self.support]

    @staticmethod
    def from_state(s):
        return Rule([Condition.from_state(c) for c in s[0]], s[1], s[2], s[3], s[4])


def leaf_rules(tree, mid: int, tj: int, names, domains, cls_suffix: str = ""):
    """Rules of every leaf of one tree, in node order (Rule.extractRulesFromTree)."""
    n = tree.n_nodes
    parent = np.full(n, -1, np.int64)
    for i in range(n):
        if tree.feat[i] >= 0:
            parent[tree.left[i]] = i
            parent[tree.right[i]] = i
    rules = []
    for leaf in range(n):
        if tree.feat[leaf] >= 0:
            continue
        conds, seen = [], set()
        node = leaf
        while parent[node] >= 0:                # leaf -> root: the first condition per (feature, op) is kept
            p = parent[node]
            f = int(tree.feat[p])
            is_left = tree.left[p] == node
            nas = bool(tree.na_left[p]) == bool(is_left)
            if tree.is_cat[p]:
                dom = domains[f] or []
                bits, nb = tree.cat_bits[p], int(tree.cat_nbits[p])
                lv = [lvl for lvl in range(len(dom))
                      if ((lvl < nb and bool((int(bits[lvl >> 5]) >> (lvl & 31)) & 1)) or
                          (lvl >= nb and bool(tree.na_left[p]))) == bool(is_left)]
                c = Condition(f, names[f], "cat", "in", -1.0, lv, [dom[v] for v in lv], nas)
            else:
                c = Condition(f, names[f], "num", "<" if is_left else ">=", float(np.float32(tree.thr[p])), nas=nas)
            if (f, c.op) not in seen:
                seen.add((f, c.op))
                conds.append(c)
            node = p
        conds.sort(key=lambda c: c.name)
        rules.append(Rule(conds, float(tree.value[leaf]), f"M{mid}T{tj}N{leaf}{cls_suffix}"))
    return rules


class RuleFitModel(Model):
    algo = "rulefit"

    def _groups(self):
        """[(column name, [rules])] in the GLM frame's column order."""
        return self.rule_groups

    def _rule_codes(self, X):
        """One categorical code per tree column: index of the last satisfied rule, NaN when none (Decoder)."""
        rows = []
        for _, rules in self._groups():
            code = torch.full((X.shape[1],), float("nan"), dtype=torch.float32, device=X.device)
            for r_i, r in enumerate(rules):
                code = torch.where(r.holds(X), torch.full_like(code, float(r_i)), code)
            rows.append(code)
        return rows

    def _glm_matrix(self, X):
        rows = self._rule_codes(X) if self.params.get("model_type", "rules_and_linear") != "linear" else []
        if self.params.get("model_type", "rules_and_linear") != "rules":
            rows += [X[f].float() for f in range(X.shape[0])]
        return torch.stack(rows, 0)

    def _predict_tensor(self, X, offset=None):
        return self.glm._predict_tensor(self._glm_matrix(X.to(self.device)), offset)

    def rule_importance(self):
        return self.output["rule_importance"]

    def all_rules(self):
        return [r for _, rules in self._groups() for r in rules]

    def predict_rules(self, frame, rule_ids):
        """0/1 column per requested rule: does the row satisfy the rule's conditions (RuleFitModel.predictRules)."""
        from ..frame import Column, H2OFrame
        X, _ = frame.model_matrix(self.info, device=self.device)
        by = {r.var: r for r in self.all_rules()}
        cols = []
        for rid in rule_ids:
            if rid not in by:
                raise ValueError(f"Rule {rid!r} is not part of the model")
            cols.append(Column(rid, "int", by[rid].holds(X).double()))
        return H2OFrame._from_columns(cols)

    def to_state(self):
        s = super().to_state()
        s["rule_groups"] = [[n, [r.to_state() for r in rules]] for n, rules in self.rule_groups]
        s["depth"], s["ntrees"] = self.depth, self.ntrees
        s["glm"] = self.glm.to_state()
        s["glm_class"] = type(self.glm).__module__ + ":" + type(self.glm).__name__
        return s

    def _restore(self, s):
        from ..persist import _from_state
        super()._restore(s)
        self.rule_groups = [(n, [Rule.from_state(r) for r in rules]) for n, rules in s["rule_groups"]]
        self.depth, self.ntrees = s["depth"], s["ntrees"]
        gs = dict(s["glm"])
        gs["__class__"] = s["glm_class"]
        self.glm = _from_state(gs)


class RuleFitTrainer:
    def __init__(self, params):
        p = dict(RF_DEFAULTS)
        if "lambda" in params:
            params = dict(params)
            params["lambda_"] = params.pop("lambda")
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    @staticmethod
    def _enum_limited(X, info, maxl):
        """The rule trees see categoricals through EnumLimited (RuleFit.java:113-114): the ``maxl`` most frequent
        levels (global counts) keep their own code, the rest share one ``other`` level. Returns the tree design,
        its DataInfo and per feature the original level indices behind each limited code (None: unchanged)."""
        from ..parallel import collectives as coll
        Xt, doms, lmap = X, list(info.domains), [None] * info.F
        for j in range(info.F):
            dom = info.domains[j]
            if not info.iscat[j] or dom is None or len(dom) <= maxl:
                continue
            c = X[j]
            ok = ~torch.isnan(c)
            cnt = torch.bincount(c[ok].long(), minlength=len(dom)).double()
            if coll.is_dist():
                cnt = coll.all_reduce_(cnt.to(coll.comm_device())).to(c.device)
            keep = sorted(np.argsort(-cnt.cpu().numpy(), kind="stable")[:maxl].tolist())
            m = torch.full((len(dom),), float(len(keep)), dtype=X.dtype, device=X.device)
            for i, k in enumerate(keep):
                m[k] = float(i)
            if Xt is X:
                Xt = X.clone()
            Xt[j] = torch.where(ok, m[c.clamp(min=0).long()], c)
            doms[j] = [dom[k] for k in keep] + ["other"]
            lmap[j] = [[k] for k in keep] + [[k for k in range(len(dom)) if k not in set(keep)]]
        tinfo = DataInfo(info.x, info.iscat, doms, info.response, info.response_domain)
        return Xt, tinfo, lmap

    @staticmethod
    def _unlimit(rules, lmap):
        """Categorical conditions on limited codes -> the original levels they stand for (names stay those of the
        limited domain, 'other' included, as the reference's rule text shows them)."""
        for r in rules:
            for c in r.conds:
                if c.ctype == "cat" and lmap[c.feat] is not None:
                    c.levels = sorted(k for lv in c.levels for k in lmap[c.feat][lv])

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .drf import DRFTrainer
        from .gbm import GBMTrainer
        from .glm import GLMTrainer
        t0 = time.time()
        p = self.p
        algo = str(p["algorithm"]).upper()
        mtype = str(p["model_type"]).lower()
        lo, hi = int(p["min_rule_length"]), int(p["max_rule_length"])
        depths = list(range(lo, hi + 1))
        ntrees = int(p["rule_generation_ntrees"])
        dom = info.response_domain
        multi = dom is not None and len(dom) > 2
        groups = []
        Xt, tinfo, lmap = self._enum_limited(X, info, int(p.get("max_categorical_levels") or 10))
        if mtype != "linear":
            for mid, d in enumerate(depths):
                kw = dict(ntrees=ntrees, max_depth=d, seed=p["seed"])
                if str(p.get("distribution", "AUTO")).upper() != "AUTO":
                    kw["distribution"] = p["distribution"]
                tr = GBMTrainer(kw) if algo == "GBM" else DRFTrainer(kw)
                m = tr.fit(Xt, y, w, offset, tinfo)
                fr = m.forest
                K = max(1, fr.K)
                for t, (tree, c) in enumerate(zip(fr.trees, fr.tree_class)):
                    tj = t // K
                    suffix = f"_{dom[c]}" if multi else ""
                    name = f"M{mid}T{tj}C{c}" if multi else f"M{mid}T{tj}"
                    rules = leaf_rules(tree, mid, tj, info.x, tinfo.domains, suffix)
                    self._unlimit(rules, lmap)
                    groups.append((name, rules))
                # columns ordered (model, tree, class) as in createGLMTrainFrame
            groups.sort(key=lambda g: _group_key(g[0]))
        model = RuleFitModel(model_key or make_key("rulefit"), p, info)
        model.device = X.device
        model.rule_groups = groups
        model.depth, model.ntrees = len(depths), ntrees
        names, iscat, doms = [], [], []
        for n, rules in groups:
            names.append(n)
            iscat.append(1)
            doms.append([r.var for r in rules])
        if mtype != "rules":
            names += [f"linear.{n}" for n in info.x]
            iscat += list(np.asarray(info.iscat).tolist())
            doms += list(info.domains)
        ginfo = DataInfo(names, np.asarray(iscat, np.int32), doms, info.response, info.response_domain)
        Xg = model._glm_matrix(X)
        # support of every rule (RuleEnsemble.calculateSupport: weighted share of rows satisfying it)
        # (row-sharded: the tree and GLM trainers reduce over the shards themselves; the supports are
        # weighted rule counts summed over every rank's rows)
        from ..parallel import collectives as coll
        wv = torch.ones(Xg.shape[1], dtype=torch.float64, device=Xg.device) if w is None else w.double()
        cnt = []
        for gi, (_, rules) in enumerate(groups):
            code = Xg[gi]
            cnt += [((code == r_i).double() * wv).sum() for r_i in range(len(rules))]
        tot = torch.stack(cnt + [wv.sum()]) if cnt else wv.sum().reshape(1)
        if coll.is_dist():
            tot = coll.all_reduce_(tot.to(coll.comm_device())).to(Xg.device)
        tot = tot.cpu().tolist()
        i = 0
        for gi, (_, rules) in enumerate(groups):
            for r in rules:
                r.support = tot[i] / tot[-1]
                i += 1
        gp = dict(alpha=1.0, seed=p["seed"])
        if p.get("lambda_") is not None:
            gp["lambda_"] = p["lambda_"]
        else:
            gp["lambda_search"] = True
            gp["nlambdas"] = 30
        if int(p["max_num_rules"]) > 0:
            gp["max_active_predictors"] = int(p["max_num_rules"]) + 1
        fam = str(p.get("distribution", "AUTO")).lower()
        if multi:
            gp["family"] = "multinomial"
        elif fam in ("gaussian", "poisson", "gamma", "tweedie", "bernoulli", "quasibinomial"):
            gp["family"] = "binomial" if fam == "bernoulli" else fam
        gvalid = None
        if valid is not None:
            Xv, yv, wv2, ov = valid
            gvalid = (model._glm_matrix(Xv), yv, wv2, ov)
        glm = GLMTrainer(gp).fit(Xg, y, w, offset, ginfo, gvalid)
        model.glm = glm
        model.output["linear_names"] = names + [f"linear.{info.response}"]
        model.output["glm_model_key"] = glm.key
        coefs = glm.output["coefficients"]
        by = {r.var: r for _, rules in groups for r in rules}
        imp = []
        for k, v in coefs.items():
            if k.startswith("Intercept") or v == 0:
                continue
            base, suf = k, ""
            if multi:
                for c in dom:
                    if k.endswith("_" + c):
                        base, suf = k[: -len(c) - 1], "_" + c
                        break
            lvl = base.split(".", 1)[1] if "." in base and not base.startswith("linear.") else None
            r = by.get(lvl) if lvl is not None else None
            if r is not None:
                imp.append(dict(variable=r.var, coefficient=float(v), support=r.support, rule=r.text()))
            else:
                imp.append(dict(variable=base + suf, coefficient=float(v), support=float("nan"), rule=""))
        if p["remove_duplicates"]:
            merged = {}
            for row in imp:
                key = (row["rule"] or row["variable"], row["variable"].split("_")[-1] if multi else "")
                if key in merged and row["rule"]:
                    merged[key]["variable"] += ", " + row["variable"]
                    merged[key]["coefficient"] += row["coefficient"]
                else:
                    merged[key] = dict(row)
            imp = list(merged.values())
        imp.sort(key=lambda r: -abs(r["coefficient"]))
        for r in imp:
            if r["variable"] in by:
                by[r["variable"]].coef = r["coefficient"]
        model.output["rule_importance"] = imp
        model.output["intercept"] = [v for k, v in coefs.items() if k.startswith("Intercept")]
        model.output["training_metrics"] = model.metrics_for(X, y, w, offset)
        if valid is not None:
            Xv, yv, wv2, ov = valid
            model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv2, ov)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model


def _group_key(name: str):
    """(model, tree, class) order of a rule column name ``M<i>T<j>`` / ``M<i>T<j>C<k>``."""
    m, rest = name[1:].split("T", 1)
    t, _, c = rest.partition("C")
    return int(m), int(t), int(c or 0)
