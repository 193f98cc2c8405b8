"""RuleFit in the reference layout: leaf rules per tree, one categorical GLM column per tree, and the
RuleFitMojoWriter multi-model MOJO scored back through the RuleFitMojoModel semantics."""
import numpy as np
import pandas as pd
import pytest
import torch

import h2o
from h2o.estimators import H2ORuleFitEstimator


@pytest.fixture(scope="module")
def df():
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    n = 1200
    d = pd.DataFrame({"a": rng.normal(size=n), "b": rng.normal(size=n), "c": rng.choice(list("xyzw"), n)})
    d.loc[rng.choice(n, 40, replace=False), "a"] = np.nan
    d["y"] = np.where(d.a.fillna(0) - d.b + (d.c == "x") + rng.normal(size=n) * 0.3 > 0, "1", "0")
    d["r"] = np.sin(d.a.fillna(0)) * 2 + d.b + rng.normal(size=n) * 0.1
    return h2o.H2OFrame(d, column_types={"c": "enum", "y": "enum"})


@pytest.mark.parametrize("model_type,y", [("rules_and_linear", "y"), ("rules", "y"), ("rules_and_linear", "r")])
def test_rulefit_mojo_roundtrip(df, tmp_path, model_type, y):
    m = H2ORuleFitEstimator(min_rule_length=2, max_rule_length=3, rule_generation_ntrees=4, seed=1,
                            model_type=model_type)
    m.train(x=["a", "b", "c"], y=y, training_frame=df)
    mod = m._model
    # one categorical GLM column per (depth model, tree); its levels are that tree's leaf rules
    cols = [n for n, _ in mod.rule_groups]
    assert cols == [f"M{i}T{j}" for i in range(2) for j in range(4)]
    for _, rules in mod.rule_groups:
        assert all(r.var.startswith("M") and "N" in r.var for r in rules)
    imp = mod.output["rule_importance"]
    assert imp and all(set(r) >= {"variable", "coefficient", "support", "rule"} for r in imp)
    path = m.download_mojo(str(tmp_path))
    import zipfile
    with zipfile.ZipFile(path) as z:
        names = z.namelist()
        ini = z.read("model.ini").decode()
    assert any(n.startswith("models/") and n.endswith("model.ini") for n in names)
    assert "linear_model = " in ini and "num_rules_M0T0 = " in ini and "data_from_rules_codes_len" in ini
    g = h2o.import_mojo(path)
    p0 = m.predict(df).as_data_frame()
    p1 = g.predict(df).as_data_frame()
    col = "p1" if y == "y" else "predict"
    c1 = "1" if y == "y" else "predict"
    assert np.allclose(p0[c1].to_numpy(), p1[c1].to_numpy(), atol=1e-6)


def test_rulefit_leaf_rules_partition_rows(df):
    m = H2ORuleFitEstimator(min_rule_length=3, max_rule_length=3, rule_generation_ntrees=3, seed=2)
    m.train(x=["a", "b", "c"], y="y", training_frame=df)
    mod = m._model
    X, _ = df.model_matrix(mod.info)
    for _, rules in mod.rule_groups:
        hits = torch.stack([r.holds(X) for r in rules]).sum(0)
        # every row satisfies its leaf's rule; rows with NA or with a categorical level routed by an ancestor
        # can also match a second one (the reference keeps only the condition closest to the leaf per
        # (feature, operator)); the Decoder takes the last match
        assert bool((hits >= 1).all())
        assert float((hits == 1).double().mean()) > 0.9
