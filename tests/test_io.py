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
