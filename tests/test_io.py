"""Parsers (native CSV tokenizer + type guessing, SVMLight, ARFF) and ParseSetup."""
import numpy as np

from llama_github_io_amd.io import parse as P


def test_csv_types_and_na(tmp_path):
    p = tmp_path / "t.csv"
    p.write_text('a,b,c,d,e\n1,2.5,x,2020-01-01,"q,1"\n2,NA,y,2020-01-02,z\n3,4.0,x,2020-02-03,\n')
    f = P.import_file(str(p))
    assert f.types == {"a": "int", "b": "real", "c": "enum", "d": "time", "e": "enum"}
    df = f.as_data_frame()
    assert np.isnan(df["b"][1]) and df["e"][0] == "q,1" and df["e"][2] is None
    s = P.parse_setup(str(p))
    assert s["separator"] == "," and s["column_names"] == ["a", "b", "c", "d", "e"]


def test_csv_guess_separator_no_header_and_coltypes(tmp_path):
    p = tmp_path / "t.tsv"
    p.write_text("1\t2\tfoo\n3\t4\tbar\n5\t6\tfoo\n")
    f = P.import_file(str(p), col_types={"C1": "enum"})
    assert f.names == ["C1", "C2", "C3"] and f.types["C1"] == "enum" and f.types["C3"] == "enum"
    assert f.nrows == 3


def test_svmlight_and_arff(tmp_path):
    p = tmp_path / "t.svm"
    p.write_text("1 1:0.5 3:2\n0 2:1.5\n")
    f = P.import_file(str(p))
    assert f.ncols == 4 and f.as_data_frame().values.tolist() == [[1, 0.5, 0, 2], [0, 0, 1.5, 0]]
    a = tmp_path / "t.arff"
    a.write_text("@relation r\n@attribute x numeric\n@attribute c {u,v}\n@data\n1.5,u\n2,v\n")
    f = P.import_file(str(a))
    assert f.names == ["x", "c"] and f.types["c"] == "enum" and f.nrows == 2


def test_multi_file_import(tmp_path):
    for i in range(3):
        (tmp_path / f"p{i}.csv").write_text(f"a,b\n{i},{i * 2}\n{i + 10},{i}\n")
    f = P.import_file(str(tmp_path))
    assert f.nrows == 6 and f.names == ["a", "b"]


def test_uuid_columns(tmp_path):
    """ParseSetup's UUID type (C16Chunk): a column of UUIDs parses to two int64 halves per row, prints
    back as the same strings, survives row filters and is NA for empty cells."""
    import uuid
    import h2o
    h2o.init(verbose=False)
    us = [str(uuid.uuid5(uuid.NAMESPACE_DNS, f"row{i}")) for i in range(20)]
    p = tmp_path / "u.csv"
    p.write_text("id,x\n" + "\n".join(f"{u},{i}" for i, u in enumerate(us)) + "\n,99\n")
    fr = h2o.import_file(str(p))
    assert fr.types["id"] == "uuid"
    vals = fr.as_data_frame()["id"].tolist()
    assert vals[:20] == us and vals[20] is None
    sub = fr[fr["x"] >= 18, :].as_data_frame()["id"].tolist()
    assert sub == us[18:] + [None]
    assert fr["id"].isna().as_data_frame().values.ravel().tolist()[-2:] == [0, 1]


def test_numeric_columns_compress_bit_exactly(tmp_path, monkeypatch):
    """Chunk compression (C1/C2/C4 and the scaled C1S/C2S/C4S encodings of water/fvec): integer and
    short-decimal numeric columns are stored as 8/16/32-bit codes at import and decode bit for bit; writes
    through ``data`` decode the column for good; models see the same values."""
    import numpy as np
    import pandas as pd
    import torch
    import h2o
    from h2o.estimators import H2OGradientBoostingEstimator
    h2o.init(verbose=False)
    rng = np.random.default_rng(3)
    n = 4000
    df = pd.DataFrame({"small": rng.integers(0, 100, n), "mid": rng.integers(-20000, 20000, n),
                       "dec": np.round(rng.normal(size=n) * 50, 2), "real": rng.normal(size=n)})
    df.loc[::11, "dec"] = np.nan
    df["y"] = (df["small"] + df["real"] * 10 > 50).astype(int)
    p = tmp_path / "c.csv"
    df.to_csv(p, index=False)
    fr = h2o.import_file(str(p))
    cols = fr._cols
    assert cols["small"].compressed and cols["small"].raw_data().dtype == torch.int8
    assert cols["mid"].compressed and cols["mid"].raw_data().dtype == torch.int16
    assert cols["dec"].compressed and not cols["real"].compressed
    for name in ("small", "mid", "dec", "real"):
        v = cols[name].values().cpu().numpy()
        ref = df[name].to_numpy(dtype=np.float64)
        assert np.array_equal(np.isnan(v), np.isnan(ref)) and np.array_equal(v[~np.isnan(v)], ref[~np.isnan(ref)])
    m1 = H2OGradientBoostingEstimator(ntrees=3, max_depth=3, seed=1)
    m1.train(x=["small", "mid", "dec", "real"], y="y", training_frame=fr)
    assert cols["small"].compressed                      # model matrices decode transiently
    monkeypatch.setenv("H2O_COMPRESS", "0")
    fr2 = h2o.import_file(str(p))
    assert not fr2._cols["small"].compressed
    m2 = H2OGradientBoostingEstimator(ntrees=3, max_depth=3, seed=1)
    m2.train(x=["small", "mid", "dec", "real"], y="y", training_frame=fr2)
    assert np.allclose(m1.predict(fr).as_data_frame().to_numpy(float), m2.predict(fr2).as_data_frame().to_numpy(float))
    c = cols["mid"]
    c.data[0] = 12345.5                                  # a write decodes the column for good
    assert not c.compressed and float(c.values()[0]) == 12345.5


def test_column_codec_keeps_negative_zero():
    """A column holding -0.0 is not integer-compressed (codes would decode it as +0.0)."""
    import torch
    from llama_github_io_amd.frame import _encode
    x = torch.zeros(4096)
    x[7] = 1.5
    assert _encode(x) is not None
    x[5] = -0.0
    assert _encode(x) is None
