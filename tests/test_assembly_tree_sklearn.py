"""In-process h2o.assembly (munging pipelines, reference water/rapids/Assembly.java + h2o-py/h2o/assembly.py),
h2o.tree.H2OTree (h2o-py/h2o/tree/tree.py over the TreeV3 arrays) and the h2o.sklearn wrappers
(h2o-py/h2o/sklearn)."""
import math

import numpy as np
import pytest


@pytest.fixture(scope="module")
def fr():
    import h2o
    h2o.init(verbose=False)
    rng = np.random.default_rng(5)
    n = 300
    return h2o.H2OFrame({"a": rng.normal(size=n).tolist(), "b": rng.uniform(1, 2, n).tolist(),
                         "s": rng.choice(["xs", "ss", "ab"], n).tolist()})


def test_assembly_fit_and_pojo(fr):
    from h2o.assembly import H2OAssembly
    from h2o.transforms.preprocessing import H2OBinaryOp, H2OCol, H2OColOp, H2OColSelect
    from llama_github_io_amd.frame import H2OFrame
    asm = H2OAssembly(steps=[("sel", H2OColSelect(["a", "b", "s"])),
                             ("cos_a", H2OColOp(op=H2OFrame.cos, col="a", inplace=True)),
                             ("cnt", H2OColOp(op=H2OFrame.countmatches, col="s", inplace=False, pattern="s")),
                             ("ratio", H2OBinaryOp(op=H2OAssembly.divide, col="a", inplace=False, right=H2OCol("b")))])
    out = asm.fit(fr)
    assert out.names == ["a", "b", "s", "s0", "a0"]
    a0 = np.asarray(fr.as_data_frame()["a"])
    got = out.as_data_frame()
    np.testing.assert_allclose(got["a"], np.cos(a0), rtol=1e-12)
    np.testing.assert_allclose(got["a0"], np.cos(a0) / got["b"], rtol=1e-12)
    np.testing.assert_array_equal(got["s0"], [v.count("s") for v in fr.as_data_frame()["s"]])
    assert asm.names == ("sel", "cos_a", "cnt")
    java = asm.to_pojo("P1", "")
    assert java.startswith("import hex.genmodel.GenMunger;") and "_steps = new Step[4];" in java
    assert 'GenMunger.divide((Double)row.get("a"), _params)' in java
    assert '_params.put("rightArg", new String[]{String.valueOf(row.get("b"))});' in java


def test_assembly_rest_wire_form(fr):
    """The step strings the reference client posts to /99/Assembly (name__Class__ast__inplace__names)."""
    from llama_github_io_amd import assembly
    steps = ["sel__H2OColSelect__(cols_py dummy ['a', 's'])__False__|",
             "up__H2OColOp__(toupper (cols_py dummy 's'))__False__S_UP",
             "p__H2OBinaryOp__(+ 2 (cols_py dummy 'a'))__True__|"]
    asm, out = assembly.fit_rest(steps, fr)
    assert out.names == ["a", "s", "S_UP"]
    d = out.as_data_frame()
    np.testing.assert_allclose(d["a"], np.asarray(fr.as_data_frame()["a"]) + 2)
    assert set(d["S_UP"]) <= {"XS", "SS", "AB"}
    assert asm.steps[2].left_is_col is False and asm.steps[2].params["leftArg"] == "2"
    with pytest.raises(ValueError):
        assembly.Assembly.from_rest(["bad_step"])


def test_h2otree_in_process(fr):
    from h2o.estimators import H2OGradientBoostingEstimator
    from h2o.tree import H2OLeafNode, H2OSplitNode, H2OTree
    import h2o
    f2 = fr.cbind(h2o.H2OFrame({"y": (np.asarray(fr.as_data_frame()["a"]) > 0).astype(int).astype(str).tolist()}))
    f2["y"] = f2["y"].asfactor()
    m = H2OGradientBoostingEstimator(ntrees=2, max_depth=3, seed=1)
    m.train(x=["a", "b", "s"], y="y", training_frame=f2)
    t = H2OTree(m, 1, "1")
    assert len(t) == len(t.left_children) == len(t.node_ids) > 2
    assert isinstance(t.root_node, H2OSplitNode) and t.root_node.split_feature == "a"
    leaves = [i for i in range(len(t)) if t.left_children[i] == -1]
    assert all(not math.isnan(t.predictions[i]) for i in leaves)

    def walk(n):
        if isinstance(n, H2OLeafNode):
            return 1
        return walk(n.left_child) + walk(n.right_child)
    assert walk(t.root_node) == len(leaves)
    assert "Tree related to model" in str(t)


def test_sklearn_wrappers():
    import h2o.sklearn as hs
    from sklearn.base import clone
    from sklearn.model_selection import cross_val_score
    from sklearn.pipeline import Pipeline
    rng = np.random.default_rng(0)
    X = rng.normal(size=(300, 3))
    y = np.where(X[:, 0] - X[:, 1] > 0, "pos", "neg")
    for name in ("H2OGradientBoostingClassifier", "H2OGradientBoostingRegressor", "H2OGradientBoostingEstimator",
                 "H2OKMeansEstimator", "H2OPrincipalComponentAnalysisEstimator", "H2OAutoMLClassifier"):
        assert name in hs.__all__, name
    c = hs.H2OGradientBoostingClassifier(ntrees=5, max_depth=3, seed=1)
    assert c.get_params()["ntrees"] == 5 and "learn_rate" in c.get_params()
    c2 = clone(c).fit(X, y)
    assert set(c2.predict(X)) <= {"pos", "neg"} and c2.score(X, y) > 0.9
    pr = c2.predict_proba(X)
    assert pr.shape == (300, 2) and np.allclose(pr.sum(1), 1)
    r = hs.H2OGeneralizedLinearRegressor(lambda_=0).fit(X, 2 * X[:, 0] + 1)
    assert r.score(X, 2 * X[:, 0] + 1) > 0.999
    pipe = Pipeline([("pca", hs.H2OPrincipalComponentAnalysisEstimator(k=2)),
                     ("glm", hs.H2OGeneralizedLinearClassifier(family="binomial"))]).fit(X, y)
    assert pipe.predict(X).shape == (300,)
    s = cross_val_score(hs.H2OGeneralizedLinearClassifier(family="binomial"), X, y, cv=3)
    assert s.mean() > 0.9
