"""XLSX / XLS (BIFF8 in OLE2) / Avro ingest through h2o.import_file. The fixtures are written by the
minimal writers below (no spreadsheet or Avro library exists in this image, and the reference ships no
such files): parity with the reference parser is unpinned beyond the cell values asserted here."""
import io
import json
import struct
import zipfile
import zlib

import numpy as np
import pytest

import h2o


ROWS = [["x", "name", "flag"], [1.5, "alpha", 1.0], [2.0, "beta", 0.0], [-3.25, "alpha", None], [1e6, "gamma", 1.0]]


def _xlsx_bytes(rows):
    strings = sorted({v for r in rows for v in r if isinstance(v, str)})
    idx = {s: i for i, s in enumerate(strings)}
    ns = 'xmlns="http://schemas.openxmlformats.org/spreadsheetml/2006/main"'
    sst = f'<sst {ns} count="{len(strings)}">' + "".join(f"<si><t>{s}</t></si>" for s in strings) + "</sst>"
    body = []
    for i, r in enumerate(rows):
        cells = []
        for j, v in enumerate(r):
            ref = f"{chr(65 + j)}{i + 1}"
            if v is None:
                continue
            if isinstance(v, str):
                cells.append(f'<c r="{ref}" t="s"><v>{idx[v]}</v></c>')
            else:
                cells.append(f'<c r="{ref}"><v>{v!r}</v></c>')
        body.append(f'<row r="{i + 1}">' + "".join(cells) + "</row>")
    sheet = f"<worksheet {ns}><sheetData>" + "".join(body) + "</sheetData></worksheet>"
    b = io.BytesIO()
    with zipfile.ZipFile(b, "w") as z:
        z.writestr("xl/sharedStrings.xml", sst)
        z.writestr("xl/worksheets/sheet1.xml", sheet)
    return b.getvalue()


def _rec(typ, data=b""):
    return struct.pack("<HH", typ, len(data)) + data


def _xls_bytes(rows):
    strings = sorted({v for r in rows for v in r if isinstance(v, str)})
    idx = {s: i for i, s in enumerate(strings)}
    sst_body = b"".join(struct.pack("<HB", len(s), 0) + s.encode("latin-1") for s in strings)
    # split the SST into SST + CONTINUE in the middle of a string (exercises the resume-with-flags rule)
    head = struct.pack("<II", len(strings), len(strings))
    cut = 5
    s1, s2 = sst_body[:cut], sst_body[cut:]
    cont = bytes([0]) + s2 if s2 else b""
    glob = _rec(0x0809, struct.pack("<HHHH", 0x0600, 0x0005, 0, 0)) + _rec(0x00FC, head + s1)
    if cont:
        glob += _rec(0x003C, cont)
    sheet = _rec(0x0809, struct.pack("<HHHH", 0x0600, 0x0010, 0, 0))
    for i, r in enumerate(rows):
        for j, v in enumerate(r):
            if v is None:
                continue
            if isinstance(v, str):
                sheet += _rec(0x00FD, struct.pack("<HHHI", i, j, 15, idx[v]))
            elif float(v).is_integer() and abs(v) < 1 << 29:
                sheet += _rec(0x027E, struct.pack("<HHHI", i, j, 15, (int(v) << 2 | 2) & 0xFFFFFFFF))
            else:
                sheet += _rec(0x0203, struct.pack("<HHHd", i, j, 15, float(v)))
    sheet += _rec(0x000A)
    bound_len = len(_rec(0x0085, struct.pack("<IBB", 0, 0, 0) + b"\x06\x00Sheet1"))
    pad = _rec(0x00E1, b"\x00" * 64) * 70      # keeps the stream above the 4096-byte mini-stream cutoff
    off = len(glob) + bound_len + len(pad) + len(_rec(0x000A))
    wb = glob + _rec(0x0085, struct.pack("<IBB", off, 0, 0) + b"\x06\x00Sheet1") + pad + _rec(0x000A) + sheet
    # OLE2 container: header, 1 FAT sector, 1 directory sector, workbook sectors
    nsec = (len(wb) + 511) // 512
    wb += b"\x00" * (nsec * 512 - len(wb))
    fat = [0xFFFFFFFD, 0xFFFFFFFE] + [3 + k for k in range(nsec - 1)] + [0xFFFFFFFE]
    fat += [0xFFFFFFFF] * (128 - len(fat))
    hdr = bytearray(512)
    hdr[:8] = b"\xd0\xcf\x11\xe0\xa1\xb1\x1a\xe1"
    struct.pack_into("<HHHH", hdr, 24, 0x3E, 3, 0xFFFE, 9)
    struct.pack_into("<H", hdr, 32, 6)
    struct.pack_into("<II", hdr, 44, 1, 1)
    struct.pack_into("<IIIII", hdr, 56, 4096, 0xFFFFFFFE, 0, 0xFFFFFFFE, 0)
    difat = [0] + [0xFFFFFFFF] * 108
    struct.pack_into("<109I", hdr, 76, *difat)

    def dent(name, typ, start, size):
        e = bytearray(128)
        nm = name.encode("utf-16-le") + b"\x00\x00"
        e[:len(nm)] = nm
        struct.pack_into("<H", e, 64, len(nm))
        e[66] = typ
        struct.pack_into("<III", e, 68, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF if typ == 2 else 1)
        struct.pack_into("<II", e, 116, start, size)
        return bytes(e)
    d = dent("Root Entry", 5, 0xFFFFFFFE, 0) + dent("Workbook", 2, 2, len(wb)) + b"\x00" * 256
    return bytes(hdr) + struct.pack("<128I", *fat) + d + wb


def _zzenc(n):
    n = (n << 1) ^ (n >> 63)
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _avro_bytes(codec="deflate"):
    schema = {"type": "record", "name": "r", "fields": [
        {"name": "x", "type": "double"}, {"name": "name", "type": "string"},
        {"name": "flag", "type": ["null", "long"]},
        {"name": "color", "type": {"type": "enum", "name": "C", "symbols": ["red", "blue"]}}]}
    recs = b""
    data = [(1.5, "alpha", 1, 0), (2.0, "beta", 0, 1), (-3.25, "alpha", None, 0), (1e6, "gamma", 1, 1)]
    for x, s, f, c in data:
        recs += struct.pack("<d", x) + _zzenc(len(s)) + s.encode()
        recs += _zzenc(0) if f is None else _zzenc(1) + _zzenc(f)
        recs += _zzenc(c)
    if codec == "deflate":
        block = zlib.compress(recs)[2:-4]
    elif codec == "snappy":      # raw snappy (pyarrow's codec as the independent encoder) + big-endian CRC-32
        import pyarrow as pa
        block = pa.compress(recs, codec="snappy", asbytes=True) + (zlib.crc32(recs) & 0xFFFFFFFF).to_bytes(4, "big")
    else:
        block = recs
    sync = bytes(range(16))
    meta = {"avro.schema": json.dumps(schema).encode(), "avro.codec": codec.encode()}
    out = b"Obj\x01" + _zzenc(len(meta))
    for k, v in meta.items():
        out += _zzenc(len(k)) + k.encode() + _zzenc(len(v)) + v
    out += _zzenc(0) + sync + _zzenc(len(data)) + _zzenc(len(block)) + block + sync
    return out


def _check(fr, extra=None):
    df = fr.as_data_frame()
    assert list(df.columns)[:3] == ["x", "name", "flag"]
    np.testing.assert_allclose(df["x"].values, [1.5, 2.0, -3.25, 1e6])
    assert list(df["name"]) == ["alpha", "beta", "alpha", "gamma"]
    assert fr.types["name"] == "enum"
    assert np.isnan(df["flag"].values[2]) and df["flag"].values[0] == 1


@pytest.mark.parametrize("kind", ["xlsx", "xls"])
def test_spreadsheets(tmp_path, kind):
    h2o.init(verbose=False)
    p = tmp_path / f"t.{kind}"
    p.write_bytes(_xlsx_bytes(ROWS) if kind == "xlsx" else _xls_bytes(ROWS))
    _check(h2o.import_file(str(p)))


@pytest.mark.parametrize("codec", ["null", "deflate", "snappy"])
def test_avro(tmp_path, codec):
    h2o.init(verbose=False)
    p = tmp_path / "t.avro"
    p.write_bytes(_avro_bytes(codec))
    fr = h2o.import_file(str(p))
    _check(fr)
    assert list(fr.as_data_frame()["color"]) == ["red", "blue", "red", "blue"]


def test_orc_roundtrip(tmp_path):
    import pandas as pd
    import pyarrow as pa
    import pyarrow.orc as po
    h2o.init(verbose=False)
    p = tmp_path / "t.orc"
    po.write_table(pa.Table.from_pandas(pd.DataFrame({"x": [1.5, 2.0], "name": ["a", "b"]})), str(p))
    df = h2o.import_file(str(p)).as_data_frame()
    assert list(df["x"]) == [1.5, 2.0]


def test_snappy_decoder_matches_pyarrow():
    """The pure-Python raw snappy decoder (Avro snappy blocks) against pyarrow's encoder: literals of every length
    class, overlapping and far back-references."""
    import pyarrow as pa
    from llama_github_io_amd.io.formats import snappy_decompress
    rng = np.random.default_rng(0)
    for data in (b"", b"a", b"abcabcabcabcabcabcabc" * 50, bytes(rng.integers(0, 256, 70000, dtype=np.uint8)),
                 (b"x" * 1000 + bytes(rng.integers(0, 4, 5000, dtype=np.uint8))) * 20):
        assert snappy_decompress(pa.compress(data, codec="snappy", asbytes=True)) == data
