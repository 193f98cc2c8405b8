"""MOJO compatibility against MOJOs produced by the reference H2O (fixtures inside the reference
tree, read as data: zip/ini/bin files). Skipped when the reference checkout is not mounted.

* prostate GBM (``h2o-algos/src/jmh/resources/hex/tree/gbm/prostate``: 50 bernoulli trees with a
  categorical RACE split, CompressedTree v1.20 blobs) scored on ``prostate.csv`` through our reader:
  a correct decode of the byte format gives the training-set AUC of an overfit 50-tree GBM (≈1.0);
  any mis-decoded node would collapse it. Exact per-row parity with genmodel is unpinned (no Java).
* GLM regression MOJO (``h2o-genmodel/.../pipeline/glm_model.zip``): our scorer must reproduce
  ``beta · [one-hot(CLUSTER), nums] + intercept`` computed by hand from model.ini.
"""
import os
import zipfile

import numpy as np
import pytest

REF = "/root/reference"
PROSTATE_DIR = os.path.join(REF, "h2o-algos/src/jmh/resources/hex/tree/gbm/prostate")
PROSTATE_CSV = os.path.join(REF, "h2o-py/h2o/h2o_data/prostate.csv")
GLM_ZIP = os.path.join(REF, "h2o-genmodel/src/test/resources/hex/genmodel/algos/pipeline/glm_model.zip")

pytestmark = pytest.mark.skipif(not os.path.isdir(PROSTATE_DIR), reason="reference checkout not mounted")


def test_reference_gbm_mojo_scores_prostate(tmp_path):
    import h2o
    z = tmp_path / "prostate_gbm.zip"
    with zipfile.ZipFile(z, "w") as zf:
        for root, _, files in os.walk(PROSTATE_DIR):
            for f in files:
                full = os.path.join(root, f)
                zf.write(full, os.path.relpath(full, PROSTATE_DIR))
    fr = h2o.import_file(PROSTATE_CSV)
    fr["RACE"] = fr["RACE"].asfactor()
    fr["CAPSULE"] = fr["CAPSULE"].asfactor()
    m = h2o.import_mojo(str(z))
    assert m.output["original_algo"] == "gbm" and len(m.forest) == 50
    perf = m.model_performance(fr)
    assert perf["AUC"] > 0.97
    p = m.predict(fr).as_data_frame()
    assert ((p["1"] >= 0) & (p["1"] <= 1)).all()


def test_reference_glm_mojo_matches_hand_computation(tmp_path):
    import h2o
    import pandas as pd
    from llama_github_io_amd.mojo.reader import parse_mojo
    mj = parse_mojo(GLM_ZIP)
    beta = [float(v) for v in mj["info"]["beta"].strip("[]").split(",")]
    dom = mj["domains"][0]
    rng = np.random.default_rng(0)
    n = 50
    df = pd.DataFrame({"CLUSTER": rng.choice(dom, n), "DPROS": rng.integers(1, 5, n), "DCAPS": rng.integers(1, 3, n),
                       "PSA": rng.uniform(0, 50, n), "VOL": rng.uniform(0, 40, n), "GLEASON": rng.integers(4, 9, n)})
    fr = h2o.H2OFrame(df, column_types={"CLUSTER": "enum"})
    m = h2o.import_mojo(GLM_ZIP)
    got = m.predict(fr).as_data_frame()["predict"].values
    lut = {s: i for i, s in enumerate(dom)}
    X = np.zeros((n, len(dom) + 5))
    for i, s in enumerate(df["CLUSTER"]):
        X[i, lut[s]] = 1
    X[:, len(dom):] = df[["DPROS", "DCAPS", "PSA", "VOL", "GLEASON"]].values
    ref = X @ np.array(beta[:-1]) + beta[-1]
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-6)
