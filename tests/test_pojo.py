"""POJO export: the generated Java is evaluated by a small translator of the emitted expression subset
(nested ternaries, NaN tests, float thresholds, GRPSPLIT bitsets, spilled sub-classes) and must
reproduce the model's own predictions. No JDK exists in this image, so javac is not exercised."""
import re
import shutil
import subprocess

import numpy as np
import pandas as pd
import pytest

import h2o
from h2o.estimators import (H2OGeneralizedLinearEstimator, H2OGradientBoostingEstimator, H2OKMeansEstimator,
                            H2ORandomForestEstimator)
from llama_github_io_amd.mojo import pojo as P

_TOK = re.compile(r"\s*(Double\.isNaN|GenModel\.bitSetContains|Double\.NaN|Float\.POSITIVE_INFINITY|"
                  r"Float\.NEGATIVE_INFINITY|[A-Za-z_][A-Za-z0-9_]*\.score0|[A-Za-z_][A-Za-z0-9_]*|"
                  r"-?\d+\.\d*(?:[eE][-+]?\d+)?f?|-?\d+(?:[eE][-+]?\d+)?f?|\|\||&&|>=|<=|[?:()\[\],<>!])")


class _Parser:
    """Java expression subset -> vectorised numpy expression over D[f] (one array per column)."""

    def __init__(self, s):
        self.t = [m for m in _TOK.findall(s) if m]
        self.i = 0

    def peek(self):
        return self.t[self.i] if self.i < len(self.t) else None

    def eat(self, x=None):
        tok = self.t[self.i]
        assert x is None or tok == x, (tok, x, self.t[max(0, self.i - 5):self.i + 5])
        self.i += 1
        return tok

    def expr(self):
        c = self.orx()
        if self.peek() == "?":
            self.eat("?")
            a = self.expr()
            self.eat(":")
            b = self.expr()
            return f"np.where({c}, {a}, {b})"
        return c

    def orx(self):
        a = self.andx()
        while self.peek() == "||":
            self.eat()
            a = f"({a}) | ({self.andx()})"
        return a

    def andx(self):
        a = self.unary()
        while self.peek() == "&&":
            self.eat()
            a = f"({a}) & ({self.unary()})"
        return a

    def unary(self):
        if self.peek() == "!":
            self.eat()
            return f"~({self.unary()})"
        a = self.prim()
        if self.peek() in ("<", ">=", "<=", ">"):
            op = self.eat()
            a = f"({a} {op} {self.prim()})"
        return a

    def prim(self):
        tok = self.eat()
        if tok == "(" and self.peek() == "float" and self.t[self.i + 1] == ")":
            self.eat("float"); self.eat(")")
            return f"np.float64(np.float32({self.prim()}))"
        if tok == "(":
            e = self.expr()
            self.eat(")")
            return f"({e})"
        if tok == "data":
            self.eat("[")
            k = self.eat()
            self.eat("]")
            return f"D[{k}]"
        if tok == "Double.isNaN":
            self.eat("(")
            e = self.expr()
            self.eat(")")
            return f"np.isnan({e})"
        if tok == "GenModel.bitSetContains":
            self.eat("(")
            g = self.eat(); self.eat(","); nb = self.eat(); self.eat(","); off = self.eat(); self.eat(",")
            e = self.expr()
            self.eat(")")
            return f"bsc({g}, {nb}, {off}, {e})"
        if tok.endswith(".score0"):
            self.eat("("); self.eat("data"); self.eat(")")
            return f"SUB['{tok[:-7]}'](D)"
        if tok in ("true", "false"):
            return "True" if tok == "true" else "False"
        if tok == "Double.NaN":
            return "np.nan"
        if tok.startswith("Float."):
            return "np.inf" if "POSITIVE" in tok else "-np.inf"
        if tok.endswith("f"):
            return f"np.float64(np.float32({tok[:-1]}))"
        return f"np.float64({tok})"


def _bsc(bits, nb, off, x):
    idx = np.nan_to_num(x, nan=0).astype(np.int64) - off
    ok = (idx >= 0) & (idx < nb)
    i = np.clip(idx, 0, nb - 1)
    return ok & ((bits[i >> 3].astype(np.int64) & (1 << (i & 7))) != 0)


def _tree_functions(src):
    """Every generated tree class -> python callable D -> per-row score."""
    classes = re.findall(r"class (\w+) \{\n  static final double score0\(double\[\] data\) \{\n    double pred = "
                         r"(.*?);\n    return pred;\n  \}\n((?:  [^\n]*\n)*)\}", src, re.S)
    sub = {}
    for name, body, grp in classes:
        env = dict(np=np, SUB=sub)
        for g, arr in re.findall(r"public static final byte\[\] (GRPSPLIT\d+) = new byte\[\] \{(.*?)\};", grp):
            env[g] = np.array([int(v) & 0xFF for v in arr.split(",")], dtype=np.uint8)
        code = _Parser(body).expr()
        env["bsc"] = _bsc
        sub[name] = eval(f"lambda D: {code}", env)   # noqa: S307 (our own generated source)
    return sub


@pytest.fixture(scope="module")
def df():
    h2o.init(verbose=False)
    rng = np.random.default_rng(5)
    n = 600
    a = rng.normal(size=n)
    a[rng.random(n) < 0.08] = np.nan
    d = pd.DataFrame({"a": a, "b": rng.normal(size=n), "c": rng.choice(list("pqrstu"), n)})
    d["y"] = np.where(np.nan_to_num(d.a) - d.b + d.c.isin(["p", "s"]) + rng.normal(size=n) * 0.3 > 0, "1", "0")
    d["r"] = np.nan_to_num(d.a) * 2 + d.b + rng.normal(size=n) * 0.1
    return h2o.H2OFrame(d, column_types={"c": "enum", "y": "enum"})


def _cols(df, m):
    pdf = df.as_data_frame()
    out = []
    for n, dom in zip(m.info.x, m.info.domains):
        v = pdf[n]
        out.append(v.map({s: i for i, s in enumerate(dom)}).astype(float).values if dom else v.astype(float).values)
    return out


@pytest.mark.parametrize("algo,y", [("gbm", "y"), ("gbm", "r"), ("drf", "y"), ("drf", "r")])
def test_tree_pojo_reproduces_model(df, tmp_path, algo, y):
    est = (H2OGradientBoostingEstimator(ntrees=6, max_depth=5, seed=1) if algo == "gbm"
           else H2ORandomForestEstimator(ntrees=4, max_depth=8, seed=1))
    est.train(x=["a", "b", "c"], y=y, training_frame=df)
    path = est.download_pojo(str(tmp_path))
    src = open(path).read()
    assert "extends GenModel" in src and "public final double[] score0(double[] data, double[] preds)" in src
    m = est._model
    fns = _tree_functions(src)
    D = _cols(df, m)
    import torch
    from llama_github_io_amd.frame import H2OFrame  # noqa: F401
    X = torch.tensor(np.stack(D), dtype=torch.float32)
    raw = m.forest.predict_raw(X).double().numpy()
    tot = np.zeros_like(raw)
    for idx, c in enumerate(m.forest.tree_class):
        it = idx // max(m.forest.K, 1)
        tot[:, c] += fns[f"{P.java_ident(m.key)}_Tree_{it}_class_{c}"](D)
    np.testing.assert_allclose(tot, raw, rtol=1e-5, atol=1e-5)


def test_tree_pojo_spills_large_trees(df, tmp_path, monkeypatch):
    monkeypatch.setattr(P, "MAX_NODES_PER_CLASS", 3)
    est = H2OGradientBoostingEstimator(ntrees=2, max_depth=6, seed=2, min_rows=2)
    est.train(x=["a", "b", "c"], y="r", training_frame=df)
    src = P.pojo_source(est._model)
    assert re.search(r"_Tree_0_class_0_\d+\.score0\(data\)", src)
    fns = _tree_functions(src)
    D = _cols(df, est._model)
    import torch
    raw = est._model.forest.predict_raw(torch.tensor(np.stack(D), dtype=torch.float32)).double().numpy()
    k = P.java_ident(est._model.key)
    np.testing.assert_allclose(fns[f"{k}_Tree_0_class_0"](D) + fns[f"{k}_Tree_1_class_0"](D), raw[:, 0], rtol=1e-5,
                               atol=1e-5)


def test_glm_and_kmeans_pojo_constants(df, tmp_path):
    g = H2OGeneralizedLinearEstimator(family="binomial", lambda_=0)
    g.train(x=["a", "b", "c"], y="y", training_frame=df)
    src = P.pojo_source(g._model)
    beta = [float(v) for v in re.search(r"BETA = new double\[\] \{(.*?)\};", src).group(1).split(",")]
    coef = g.coef()
    assert abs(beta[-1] - coef["Intercept"]) < 1e-9
    k = H2OKMeansEstimator(k=3, seed=1)
    k.train(x=["a", "b"], training_frame=df)
    ks = P.pojo_source(k._model)
    assert ks.count("{") == ks.count("}") and "CENTERS" in ks
    assert h2o.download_pojo(g, str(tmp_path)).endswith(".java")


@pytest.mark.skipif(shutil.which("javac") is None, reason="no JDK in this image")
def test_pojo_compiles(df, tmp_path):   # pragma: no cover - exercised only where a JDK exists
    est = H2OGradientBoostingEstimator(ntrees=2, seed=1)
    est.train(x=["a", "b", "c"], y="y", training_frame=df)
    path = est.download_pojo(str(tmp_path))
    subprocess.run(["javac", "-d", str(tmp_path), path], check=True)


def _arr(src, name):
    m = re.search(name + r" = new double\[\]\[\] \{(.*?)\};\n", src, re.S)
    if m:
        rows = re.findall(r"\{([^{}]*)\}", m.group(1))
        return np.array([[float(v) for v in r.split(",")] for r in rows])
    m = re.search(name + r" = new (?:double|int)\[\] \{(.*?)\};", src)
    body = m.group(1).strip()
    return np.array([float(v) for v in body.split(",")]) if body else np.zeros(0)


@pytest.mark.parametrize("y", ["y", "r"])
def test_deeplearning_pojo_reproduces_model(df, y):
    from h2o.estimators import H2ODeepLearningEstimator
    m = H2ODeepLearningEstimator(hidden=[6, 5], epochs=2, seed=1, activation="Tanh")
    m.train(x=["a", "b", "c"], y=y, training_frame=df)
    mod = m._model
    src = P.pojo_source(mod)
    assert src.count("{") == src.count("}") and "static double act(double v) { return Math.tanh(v); }" in src
    X, _ = df.model_matrix(mod.info)
    D = X.double().numpy()
    cats, offs, sizes, modes, nums = (_arr(src, n).astype(int) for n in ("CATS", "CAT_OFFS", "CAT_SIZES", "CAT_MODES", "NUMS"))
    fill, sub, mul = _arr(src, "NUM_FILL"), _arr(src, "NUM_SUB"), _arr(src, "NUM_MUL")
    start = 0 if mod.expander.use_all else 1
    N = D.shape[1]
    x = np.zeros((N, mod.expander.P))
    for i, j in enumerate(cats):
        v = np.where(np.isnan(D[j]), modes[i], D[j]).astype(int) - start
        ok = (v >= 0) & (v < sizes[i])
        x[np.nonzero(ok)[0], offs[i] + v[ok]] = 1
    for i, j in enumerate(nums):
        x[:, mod.expander.num_off + i] = (np.where(np.isnan(D[j]), fill[i], D[j]) - sub[i]) * mul[i]
    L = len(mod.net.hidden)
    for i in range(L):
        x = np.tanh(x @ _arr(src, f"W{i}").T + _arr(src, f"B{i}"))
    o = x @ _arr(src, f"W{L}").T + _arr(src, f"B{L}")
    P_ = mod.score_tensor(X).double().numpy()
    if y == "y":
        e = np.exp(o - o.max(1, keepdims=True))
        assert np.allclose(e / e.sum(1, keepdims=True), P_, atol=1e-4)
    else:
        assert np.allclose(o[:, 0] * mod.resp_sd + mod.resp_mu, P_.reshape(-1), atol=1e-3)


def test_naivebayes_pojo_constants_reproduce_model(df):
    from h2o.estimators import H2ONaiveBayesEstimator
    m = H2ONaiveBayesEstimator()
    m.train(x=["a", "b", "c"], y="y", training_frame=df)
    mod = m._model
    src = P.pojo_source(mod)
    assert src.count("{") == src.count("}")
    prior = _arr(src, "PRIOR")
    X, _ = df.model_matrix(mod.info)
    D = X.double().numpy()
    ll = np.log(prior)[None, :].repeat(D.shape[1], 0)
    p = mod.params
    for j in range(mod.info.F):
        c = _arr(src, f"COND{j}")
        na = np.isnan(D[j])
        if mod.info.iscat[j]:
            code = np.clip(np.nan_to_num(D[j]).astype(int), 0, c.shape[1] - 1)
            pr = c[:, code].T
            pr = np.where(pr <= p["eps_prob"], p["min_prob"], pr)
            ll += np.where(na[:, None], 0, np.log(pr))
        else:
            sd = np.where(c[1] <= p["eps_sdev"], p["min_sdev"], c[1])
            z = (D[j][:, None] - c[0][None, :]) / sd[None, :]
            ll += np.where(na[:, None], 0, -0.5 * z * z - np.log(sd)[None, :] - 0.5 * np.log(2 * np.pi))
    e = np.exp(ll - ll.max(1, keepdims=True))
    assert np.allclose(e / e.sum(1, keepdims=True), mod.score_tensor(X).double().numpy(), atol=1e-5)


def _const(src, name, kind="double"):
    m = re.search(rf"public static final {kind}\[\](?:\[\])? {name} = new {kind}\[\](?:\[\])? \{{(.*?)\}};", src, re.S)
    body = m.group(1)
    if "{" in body:
        return np.array([[float(v) for v in row.split(",") if v.strip()] for row in re.findall(r"\{(.*?)\}", body)])
    return np.array([float(v) for v in body.split(",") if v.strip()])


def _design_replay(src, D, P):
    """Python replay of the emitted z[] construction (_design_java)."""
    cats, offs = _const(src, "CATS", "int").astype(int), _const(src, "CAT_OFFS", "int").astype(int)
    levels, modes = _const(src, "CAT_LEVELS", "int").astype(int), _const(src, "CAT_MODES", "int").astype(int)
    nums = _const(src, "NUMS", "int").astype(int)
    fill, sub, mul = _const(src, "NUM_FILL"), _const(src, "NUM_SUB"), _const(src, "NUM_MUL")
    start = int(re.search(r"int col = c - (\d+);", src).group(1))
    noff = int(re.search(r"z\[(\d+) \+ i\] = \(v - NUM_SUB", src).group(1))
    n = len(D[0])
    Z = np.zeros((n, P))
    for i, j in enumerate(cats):
        v = D[j]
        c = np.where(np.isnan(v), modes[i], np.nan_to_num(v)).astype(int)
        ok = (c >= 0) & (c < levels[i]) & (c - start >= 0)
        Z[np.nonzero(ok)[0], offs[i] + (c - start)[ok]] = 1
    for i, j in enumerate(nums):
        v = np.where(np.isnan(D[j]), fill[i], D[j])
        Z[:, noff + i] = (v - sub[i]) * mul[i]
    return Z


@pytest.mark.parametrize("algo", ["pca", "svd"])
def test_pca_svd_pojo_reproduces_model(df, algo):
    from h2o.estimators import H2OPrincipalComponentAnalysisEstimator, H2OSingularValueDecompositionEstimator
    if algo == "pca":
        m = H2OPrincipalComponentAnalysisEstimator(k=2, transform="STANDARDIZE", use_all_factor_levels=True)
    else:
        m = H2OSingularValueDecompositionEstimator(nv=2, transform="DEMEAN")
    m.train(x=["a", "b", "c"], training_frame=df)
    src = P.pojo_source(m._model)
    assert "public final double[] score0(double[] data, double[] preds)" in src
    V = _const(src, "EIGVECS")
    Z = _design_replay(src, _cols(df, m._model), V.shape[0])
    got = Z @ V
    ref = m.predict(df).as_data_frame().to_numpy(dtype=float)
    assert np.allclose(got, ref, rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("y,booster", [("y", "gbtree"), ("r", "gbtree"), ("r", "gblinear")])
def test_xgboost_pojo_reproduces_model(df, y, booster):
    from h2o.estimators import H2OXGBoostEstimator
    m = H2OXGBoostEstimator(ntrees=5, max_depth=3, seed=1, booster=booster)
    m.train(x=["a", "b", "c"], y=y, training_frame=df)
    src = P.pojo_source(m._model)
    D = _cols(df, m._model)
    if booster == "gblinear":
        W, bias = _const(src, "W"), _const(src, "BIAS")
        f = _design_replay(src, D, W.shape[1]) @ W[0] + bias[0]
    else:
        sub = _tree_functions(src)
        init = float(re.search(r"double\[\] f = new double\[\] \{(.*?)\};", src).group(1))
        f = np.full(len(D[0]), init)
        for call in re.findall(r"f\[0\] \+= \(float\) (\w+)\.score0\(data\);", src):
            f = f + np.float32(sub[call](D))
    pred = m.predict(df).as_data_frame()
    if y == "y":
        assert np.allclose(1 / (1 + np.exp(-f)), pred["1"].to_numpy(), atol=1e-5)
    else:
        assert np.allclose(f, pred["predict"].to_numpy(), rtol=1e-5, atol=1e-4)
