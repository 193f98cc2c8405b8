"""Ingest: ParseSetup guessing + parsers + export (reference: ``water/parser/ParseSetup.java``,
``CsvParser.java``, ``SVMLightParser.java``, ``ARFFParser.java``, ``h2o-parsers/h2o-parquet-parser``,
``water/api/FramesHandler.java`` export, ``water/persist/PersistNFS.java``).

CSV goes through the native multi-threaded tokenizer (``csrc/csv_parser.cpp``): one host pass
produces per-column doubles + kind bytes + text spans, Python only builds enum domains for text
columns (also native) and then moves every numeric/categorical column into HBM in one copy.
Type rules (ParseSetup): a column whose non-NA tokens are all numbers is ``int``/``real``; a column
dominated by text is ``enum`` (numbers inside it become levels), a numeric-majority column turns
stray text into NA; text columns that parse as dates become ``time``; ``col_types`` overrides.
"""
from __future__ import annotations

import ctypes
import glob as _glob
import gzip
import io
import math
import os
import zipfile

import numpy as np
import torch

from ..frame import Column, H2OFrame, _enum_from_values, engine_device

_TYPE_ALIASES = {"numeric": "real", "real": "real", "float": "real", "double": "real", "int": "int", "integer": "int",
                 "enum": "enum", "factor": "enum", "categorical": "enum", "string": "string", "str": "string",
                 "time": "time", "date": "time", "uuid": "uuid"}


# ------------------------------------------------------------------------------------------------
def _read_bytes(path: str, decrypt_tool=None) -> bytes:
    if decrypt_tool is not None:
        # DecryptionTool.decryptInputStream: decrypt the raw file, then unpack a gzip / zip container by its magic
        from .decrypt import get_tool
        with open(path, "rb") as f:
            data = get_tool(decrypt_tool).decrypt(f.read())
        if data[:2] == b"\x1f\x8b":
            return gzip.decompress(data)
        if data[:4] == b"PK\x03\x04":
            with zipfile.ZipFile(io.BytesIO(data)) as z:
                names = [n for n in z.namelist() if not n.endswith("/")]
                return b"".join(z.read(n) for n in names)
        return data
    if path.endswith(".gz"):
        with gzip.open(path, "rb") as f:
            return f.read()
    if path.endswith(".zip"):
        with zipfile.ZipFile(path) as z:
            names = [n for n in z.namelist() if not n.endswith("/")]
            return b"".join(z.read(n) for n in names)
    with open(path, "rb") as f:
        return f.read()


def _expand(path) -> list:
    if isinstance(path, (list, tuple)):
        out = []
        for p in path:
            out += _expand(p)
        return out
    from . import persist_url
    urls = persist_url.resolve(path)        # http(s):// -> fetched whole into the persist cache (PersistEagerHTTP)
    if urls is not None:
        return urls
    path = os.path.expanduser(str(path))
    if path.startswith("file://"):
        path = path[7:]
    if os.path.isdir(path):
        return sorted(p for p in _glob.glob(os.path.join(path, "*")) if os.path.isfile(p))
    if any(ch in path for ch in "*?["):
        return sorted(_glob.glob(path))
    if not os.path.exists(path):
        raise FileNotFoundError(path)
    return [path]


def _plain_name(path: str, decrypt_tool) -> str:
    """The file name parse-type guessing sees: an encrypted file's extension (.aes / .enc) says nothing."""
    if decrypt_tool is None:
        return path
    low = path.lower()
    for ext in (".aes", ".enc", ".encrypted"):
        if low.endswith(ext):
            return path[: -len(ext)]
    return path


def guess_parse_type(path: str, head: bytes) -> str:
    low = path.lower()
    for ext, t in ((".parquet", "PARQUET"), (".svm", "SVMLight"), (".svmlight", "SVMLight"), (".arff", "ARFF"),
                   (".xlsx", "XLSX"), (".xls", "XLS"), (".orc", "ORC"), (".avro", "AVRO"), (".feather", "FEATHER")):
        if low.endswith(ext) or low.endswith(ext + ".gz"):
            return t
    if head[:4] == b"PAR1":
        return "PARQUET"
    txt = head[:4096].decode("utf-8", "replace").lstrip()
    if txt.lower().startswith("@relation"):
        return "ARFF"
    first = txt.splitlines()[0] if txt else ""
    toks = first.split()
    if len(toks) >= 2 and all(":" in t for t in toks[1:]) and all(t.split(":")[0].isdigit() for t in toks[1:]):
        return "SVMLight"
    return "CSV"


def parse_setup(path, destination_frame=None, header=0, separator=None, column_names=None, column_types=None,
                na_strings=None, decrypt_tool=None) -> dict:
    """``/3/ParseSetup``: guess parse type, separator, header, column names and types."""
    files = _expand(path)
    head = _read_bytes(files[0], decrypt_tool)[: 1 << 20]
    ptype = guess_parse_type(_plain_name(files[0], decrypt_tool), head)
    out = dict(source_frames=[{"name": f} for f in files], parse_type=ptype, destination_frame=destination_frame or
               _dest_name(files[0]), check_header=header, separator=None, column_names=None, column_types=None,
               number_columns=0, na_strings=na_strings)
    if ptype == "CSV":
        rt = _rt()
        sep = separator or rt.h2o_csv_guess_sep(head, len(head)).decode("latin-1")
        fr = _parse_csv_bytes(head[: head.rfind(b"\n") + 1] or head, sep, header, column_names, column_types, na_strings,
                              device=torch.device("cpu"))
        out.update(separator=sep, column_names=fr.names, column_types=[_h2o_type(t) for t in fr.types.values()],
                   number_columns=fr.ncols)
    return out


def _h2o_type(t: str) -> str:
    return {"real": "Numeric", "int": "Numeric", "enum": "Enum", "string": "String", "time": "Time"}.get(t, t)


def _dest_name(path: str) -> str:
    b = os.path.basename(path)
    for ext in (".gz", ".zip", ".csv", ".txt", ".svm", ".arff", ".parquet", ".data"):
        if b.lower().endswith(ext):
            b = b[: -len(ext)]
    return b.replace("-", "_").replace(".", "_") + ".hex"


# ------------------------------------------------------------------------------------------------
_rt_lib = None


def _rt():
    global _rt_lib
    if _rt_lib is None:
        from ..ops import _native
        lib = _native.rt()
        c = ctypes
        lib.h2o_csv_guess_sep.argtypes = [c.c_char_p, c.c_int64]
        lib.h2o_csv_guess_sep.restype = c.c_char
        lib.h2o_csv_parse.argtypes = [c.c_char_p, c.c_int64, c.c_char, c.c_int, c.c_char, c.c_int]
        lib.h2o_csv_parse.restype = c.c_void_p
        lib.h2o_csv_nrows.argtypes = [c.c_void_p]
        lib.h2o_csv_nrows.restype = c.c_int64
        lib.h2o_csv_ncols.argtypes = [c.c_void_p]
        lib.h2o_csv_ncols.restype = c.c_int
        lib.h2o_csv_has_header.argtypes = [c.c_void_p]
        lib.h2o_csv_count.argtypes = [c.c_void_p, c.c_int, c.c_int]
        lib.h2o_csv_count.restype = c.c_int64
        lib.h2o_csv_header.argtypes = [c.c_void_p, c.c_int, c.c_char_p, c.c_int]
        lib.h2o_csv_get.argtypes = [c.c_void_p, c.c_int, c.c_void_p, c.c_void_p, c.c_void_p, c.c_void_p]
        lib.h2o_csv_free.argtypes = [c.c_void_p]
        lib.h2o_csv_domain.argtypes = [c.c_void_p, c.c_char_p, c.c_int, c.c_void_p]
        lib.h2o_csv_domain.restype = c.c_void_p
        lib.h2o_domain_size.argtypes = [c.c_void_p]
        lib.h2o_domain_level.argtypes = [c.c_void_p, c.c_int, c.c_char_p, c.c_int]
        lib.h2o_domain_free.argtypes = [c.c_void_p]
        _rt_lib = lib
    return _rt_lib


def _sep_byte(sep) -> bytes:
    return sep.encode() if isinstance(sep, str) else bytes([sep])


def _parse_csv_bytes(buf: bytes, sep, header, column_names, column_types, na_strings, device=None,
                     skipped_columns=None, sharded=False, names_from=None) -> H2OFrame:
    """Parse one CSV buffer. ``sharded``: ``buf`` is this rank's byte range of a file parsed by every rank
    (``ParseDataset``): column kinds, int-ness and categorical domains are agreed over the ranks with
    three small all-gathers, and the frame comes back row-sharded. ``names_from``: column names when
    this chunk carries no header line (ranks > 0)."""
    from ..parallel import collectives as coll, dframe
    rt = _rt()
    device = device or engine_device()
    if sep is None:
        sep = rt.h2o_csv_guess_sep(buf, len(buf)).decode("latin-1")
    hdr = {1: 1, -1: 0, 0: -1}.get(int(header) if header is not None else 0, -1)
    h = rt.h2o_csv_parse(buf, len(buf), _sep_byte(sep), hdr, b'"', 0)
    try:
        n = rt.h2o_csv_nrows(h)
        nc = rt.h2o_csv_ncols(h)
        names = []
        sbuf = ctypes.create_string_buffer(4096)
        for c in range(nc):
            k = rt.h2o_csv_header(h, c, sbuf, 4096) if rt.h2o_csv_has_header(h) else -1
            names.append(sbuf.value.decode("utf-8", "replace").strip().strip('"') if k >= 0 else f"C{c + 1}")
        if names_from is not None:
            names = list(names_from) + names[len(names_from):]
        if column_names:
            names = list(column_names) + names[len(column_names):]
        if sharded:
            nc = max(int(x) for x in coll.all_gather_object(nc))
            names = names + [f"C{c + 1}" for c in range(len(names), nc)]
        ctypes_ = _normalize_types(column_types, names)
        na_set = _na_sets(na_strings, names)
        skip = set(skipped_columns or [])
        cols = []
        num = np.empty(n, dtype=np.float64)
        kind = np.empty(n, dtype=np.uint8)
        counts = np.array([[rt.h2o_csv_count(h, c, 1), rt.h2o_csv_count(h, c, 2)] if c < rt.h2o_csv_ncols(h) else [0, 0]
                           for c in range(nc)], dtype=np.float64).reshape(nc, 2)
        if sharded:     # ParseSetup's column-kind vote over the whole file, not one chunk
            counts = np.sum(coll.all_gather_object(counts), axis=0)
        want = []
        for c in range(nc):
            forced = ctypes_.get(names[c])
            want.append(forced in ("enum", "string") or (forced is None and counts[c, 1] > counts[c, 0]) or
                        bool(na_set.get(names[c])))
        doms = {}
        codes_of = {}
        for c in range(nc):
            if c in skip or names[c] in skip or not want[c]:
                continue
            codes = np.full(n, -1, dtype=np.int32)
            dom = []
            if c < rt.h2o_csv_ncols(h) and n > 0:
                d = rt.h2o_csv_domain(h, buf, c, codes.ctypes.data)
                try:
                    L = rt.h2o_domain_size(d)
                    for k in range(L):
                        ln = rt.h2o_domain_level(d, k, sbuf, 4096)
                        if ln >= 4096:
                            big = ctypes.create_string_buffer(ln + 1)
                            rt.h2o_domain_level(d, k, big, ln + 1)
                            dom.append(big.value.decode("utf-8", "replace"))
                        else:
                            dom.append(sbuf.value.decode("utf-8", "replace"))
                finally:
                    rt.h2o_domain_free(d)
            doms[c], codes_of[c] = dom, codes
        if sharded:     # categorical domain unification: sorted union of every rank's levels
            alld = coll.all_gather_object(doms)
            for c in doms:
                glob = sorted(set().union(*[set(a.get(c, [])) for a in alld]))
                if glob != doms[c]:
                    lut = {v: i for i, v in enumerate(glob)}
                    m = np.array([lut[v] for v in doms[c]] + [-1], dtype=np.int32)
                    codes_of[c] = m[np.where(codes_of[c] < 0, len(doms[c]), codes_of[c])]
                    doms[c] = glob
        num_int = {}
        for c in range(nc):
            if c in skip or names[c] in skip:
                continue
            forced = ctypes_.get(names[c])
            if c < rt.h2o_csv_ncols(h):
                rt.h2o_csv_get(h, c, num.ctypes.data, kind.ctypes.data, None, None)
            else:
                num[:] = np.nan
            nas = na_set.get(names[c])
            want_text = want[c]
            if want_text:
                codes, dom = codes_of[c], doms[c]
                L = len(dom)
                if nas:
                    bad = np.array([s in nas for s in dom] + [True], dtype=bool)
                    codes = np.where(bad[np.where(codes < 0, L, codes)], -1, codes).astype(np.int32)
                    keep = [i for i, s in enumerate(dom) if s not in nas]
                    remap = np.full(L + 1, -1, dtype=np.int32)
                    remap[keep] = np.arange(len(keep), dtype=np.int32)
                    codes = remap[np.where(codes < 0, L, codes)]
                    dom = [dom[i] for i in keep]
                    if forced is None and all(_isnum(s) for s in dom):
                        vals = np.array([float(s) for s in dom] + [np.nan])[np.where(codes < 0, len(dom), codes)]
                        cols.append(Column(names[c], _int_or_real(vals), torch.as_tensor(vals, device=device)))
                        continue
                col = _text_column(names[c], dom, codes, forced, device)
                cols.append(col)
            else:
                vals = num.copy()
                if forced == "time":
                    cols.append(Column(names[c], "time", torch.as_tensor(vals, device=device)))
                else:
                    t = forced if forced in ("int", "real") else _int_or_real(vals)
                    num_int[len(cols)] = t == "int"
                    cols.append(Column(names[c], t, torch.as_tensor(vals, device=device)))
        if sharded:
            # int vs real is a property of the whole column: real on any rank -> real everywhere
            agree = coll.all_gather_object(num_int)
            for i in num_int:
                if not all(a.get(i, True) for a in agree):
                    cols[i].type = "real"
            with dframe.shard_ctx(dframe.make_shard(n)):
                return H2OFrame._from_columns(cols)
        return H2OFrame._from_columns(cols)
    finally:
        rt.h2o_csv_free(h)


def _byte_range(path: str, rank: int, world: int) -> bytes:
    """This rank's whole lines of an uncompressed file: the lines that START in
    [rank*S/W, (rank+1)*S/W) (the first line belongs to rank 0), read with two seeks."""
    size = os.path.getsize(path)
    lo, hi = rank * size // world, (rank + 1) * size // world

    def line_start(f, pos):
        if pos == 0:
            return 0
        f.seek(pos - 1)
        while True:
            chunk = f.read(1 << 16)
            if not chunk:
                return size
            k = chunk.find(b"\n")
            if k >= 0:
                return pos - 1 + k + 1
            pos += len(chunk)
    with open(path, "rb") as f:
        a = line_start(f, lo)
        b = line_start(f, hi) if hi < size else size
        if b <= a:
            return b""
        f.seek(a)
        return f.read(b - a)


def _split_lines(buf: bytes, rank: int, world: int) -> bytes:
    """In-memory version of :func:`_byte_range` for decompressed buffers."""
    size = len(buf)

    def line_start(pos):
        if pos == 0:
            return 0
        k = buf.find(b"\n", pos - 1)
        return size if k < 0 else k + 1
    a = line_start(rank * size // world)
    b = line_start((rank + 1) * size // world) if rank + 1 < world else size
    return buf[a:b] if b > a else b""


def _parse_csv_distributed(path, sep, header, column_names, column_types, na_strings, skipped_columns,
                           markers=None) -> H2OFrame:
    """``ParseDataset`` over the ranks: every rank guesses the setup from the same file head, parses its
    own byte range (plain files are read with seeks, never whole), then the ranks agree on the column
    kinds and domains (:func:`_parse_csv_bytes` with ``sharded=True``)."""
    from ..parallel import collectives as coll
    rt = _rt()
    r, w = coll.rank(), coll.world()
    plain = not (path.endswith(".gz") or path.endswith(".zip")) and not markers
    if plain:
        with open(path, "rb") as f:
            head = f.read(1 << 16)
    else:
        whole = _read_bytes(path)
        if markers:
            whole = b"\n".join(ln for ln in whole.split(b"\n") if not any(ln.startswith(m.encode()) for m in markers))
        head = whole[: 1 << 16]
    head = head[: head.rfind(b"\n") + 1] or head
    if sep is None:
        sep = rt.h2o_csv_guess_sep(head, len(head)).decode("latin-1")
    hdr = {1: 1, -1: 0, 0: -1}.get(int(header) if header is not None else 0, -1)
    hh = rt.h2o_csv_parse(head, len(head), _sep_byte(sep), hdr, b'"', 0)
    try:
        has_header = bool(rt.h2o_csv_has_header(hh))
        sbuf = ctypes.create_string_buffer(4096)
        names = []
        for c in range(rt.h2o_csv_ncols(hh)):
            k = rt.h2o_csv_header(hh, c, sbuf, 4096) if has_header else -1
            names.append(sbuf.value.decode("utf-8", "replace").strip().strip('"') if k >= 0 else f"C{c + 1}")
    finally:
        rt.h2o_csv_free(hh)
    chunk = _byte_range(path, r, w) if plain else _split_lines(whole, r, w)
    my_header = 1 if (r == 0 and has_header) else -1
    return _parse_csv_bytes(chunk, sep, my_header, column_names, column_types, na_strings,
                            skipped_columns=skipped_columns, sharded=True, names_from=names)


def _isnum(s: str) -> bool:
    try:
        float(s)
        return True
    except ValueError:
        return False


def _int_or_real(vals: np.ndarray) -> str:
    fin = vals[np.isfinite(vals)]
    return "int" if fin.size == 0 or bool(np.all(fin == np.round(fin))) and np.abs(fin).max() < 2 ** 53 else "real"


def _text_column(name, dom, codes, forced, device) -> Column:
    if forced == "string":
        arr = np.array(dom + [None], dtype=object)[np.where(codes < 0, len(dom), codes)]
        return Column(name, "string", strings=arr)
    if forced is None and dom and len(dom) <= 100000:
        # date-like text -> time (ParseSetup time guessing)
        sample = dom[: min(len(dom), 50)]
        if all(_looks_like_date(s) for s in sample):
            import pandas as pd
            ts = pd.to_datetime(pd.Series(dom), errors="coerce")
            if not ts.isna().any():
                ms = ts.values.astype("datetime64[ms]").astype(np.int64).astype(np.float64)
                vals = np.append(ms, np.nan)[np.where(codes < 0, len(dom), codes)]
                return Column(name, "time", torch.as_tensor(vals, device=device))
    # H2O orders numeric-looking levels numerically
    if dom and all(_isnum(s) for s in dom):
        order = sorted(range(len(dom)), key=lambda i: float(dom[i]))
        if order != list(range(len(dom))):
            inv = np.empty(len(dom) + 1, dtype=np.int32)
            inv[order] = np.arange(len(dom), dtype=np.int32)
            inv[len(dom)] = -1
            codes = inv[np.where(codes < 0, len(dom), codes)]
            dom = [dom[i] for i in order]
    return Column(name, "enum", torch.as_tensor(codes, device=device), dom)


def _looks_like_date(s: str) -> bool:
    s = s.strip()
    if len(s) < 8 or len(s) > 32:
        return False
    digits = sum(ch.isdigit() for ch in s)
    return digits >= 6 and (s[4:5] in "-/" or s[2:3] in "-/") and s[:2].isdigit()


def _normalize_types(column_types, names) -> dict:
    if not column_types:
        return {}
    if isinstance(column_types, dict):
        return {k: _TYPE_ALIASES.get(str(v).lower(), str(v).lower()) for k, v in column_types.items()}
    return {names[i]: _TYPE_ALIASES.get(str(v).lower(), str(v).lower()) for i, v in enumerate(column_types)
            if i < len(names) and v is not None}


def _na_sets(na_strings, names) -> dict:
    if not na_strings:
        return {}
    if isinstance(na_strings, dict):
        return {k: set(v if isinstance(v, (list, tuple)) else [v]) for k, v in na_strings.items()}
    if all(isinstance(v, str) for v in na_strings):
        return {n: set(na_strings) for n in names}
    return {names[i]: set(v) for i, v in enumerate(na_strings) if v}


# ------------------------------------------------------------------------------------------------
def parse_svmlight(buf: bytes, device=None) -> H2OFrame:
    """``SVMLightParser``: ``label idx:val ...`` (1-based indices) -> C1 = label, C2.. features, 0 fill."""
    device = device or engine_device()
    labels, rows, cols, vals = [], [], [], []
    maxc = 0
    for i, line in enumerate(buf.decode("utf-8", "replace").splitlines()):
        line = line.split("#", 1)[0].strip()
        if not line:
            continue
        toks = line.split()
        r = len(labels)
        labels.append(float(toks[0]))
        for t in toks[1:]:
            k, v = t.split(":", 1)
            if k == "qid":
                continue
            c = int(k)
            maxc = max(maxc, c)
            rows.append(r)
            cols.append(c)
            vals.append(float(v))
    n = len(labels)
    X = np.zeros((n, maxc), dtype=np.float64)
    if rows:
        X[np.asarray(rows), np.asarray(cols) - 1] = np.asarray(vals)
    out = [Column("C1", _int_or_real(np.asarray(labels)), torch.as_tensor(np.asarray(labels), device=device))]
    for j in range(maxc):
        out.append(Column(f"C{j + 2}", _int_or_real(X[:, j]), torch.as_tensor(X[:, j].copy(), device=device)))
    return H2OFrame._from_columns(out)


def parse_arff(buf: bytes, device=None) -> H2OFrame:
    """``ARFFParser``: @attribute declarations give names/types, @data is CSV."""
    device = device or engine_device()
    txt = buf.decode("utf-8", "replace")
    names, types = [], []
    lines = txt.splitlines()
    data_at = len(lines)
    for i, ln in enumerate(lines):
        s = ln.strip()
        low = s.lower()
        if low.startswith("@attribute"):
            rest = s[len("@attribute"):].strip()
            if rest.startswith(("'", '"')):
                q = rest[0]
                j = rest.index(q, 1)
                nm, ty = rest[1:j], rest[j + 1:].strip()
            else:
                nm, ty = rest.split(None, 1)
            names.append(nm)
            tl = ty.lower()
            types.append("enum" if ty.startswith("{") else ("string" if tl.startswith("string") else
                                                            ("time" if tl.startswith("date") else "real")))
        elif low.startswith("@data"):
            data_at = i + 1
            break
    body = "\n".join(ln for ln in lines[data_at:] if ln.strip() and not ln.strip().startswith("%")) + "\n"
    fr = _parse_csv_bytes(body.encode(), ",", -1, names, types, None, device)
    return fr


def parse_parquet(path: str, device=None) -> H2OFrame:
    import pyarrow.parquet as pq
    df = pq.read_table(path).to_pandas()
    return H2OFrame._from_columns(list(H2OFrame(df)._cols.values()))


def import_file(path=None, destination_frame=None, parse=True, header=0, sep=None, col_names=None, col_types=None,
                na_strings=None, pattern=None, skipped_columns=None, custom_non_data_line_markers=None,
                partition_by=None, quotechar=None, escapechar=None, decrypt_tool=None) -> H2OFrame:
    """``h2o.import_file``: file, directory, glob or list; multiple files are row-bound (ParseDataset).
    ``decrypt_tool``: key (or object) of a Decryption Tool (io/decrypt.py) applied to every file first."""
    files = _expand(path)
    if pattern:
        import re
        rx = re.compile(pattern)
        files = [f for f in files if rx.search(os.path.basename(f))]
    if not files:
        raise FileNotFoundError(f"no files match {path}")
    frames = []
    from ..parallel import dframe
    for i, f in enumerate(files):
        # an encrypted file is decrypted whole (ECB / padding), not split into per-rank byte ranges
        dist_parse = dframe.active() and not dframe.in_method() and decrypt_tool is None
        if dist_parse:
            with open(f, "rb") as fh:
                head = fh.read(4096)
            if f.endswith(".gz"):
                head = _read_bytes(f)[:4096]
            ptype = guess_parse_type(f, head)
            if ptype != "CSV":
                dist_parse = False
        if not dist_parse or ptype != "CSV":
            buf = _read_bytes(f, decrypt_tool)
            ptype = guess_parse_type(_plain_name(f, decrypt_tool), buf[:4096])
        if ptype == "SVMLight":
            fr = parse_svmlight(buf)
        elif ptype == "ARFF":
            fr = parse_arff(buf)
        elif ptype == "PARQUET":
            fr = parse_parquet(io.BytesIO(buf) if decrypt_tool is not None else f)
        elif ptype in ("XLS", "XLSX", "AVRO"):
            from . import formats
            grid = {"XLS": formats.read_xls, "XLSX": formats.read_xlsx, "AVRO": formats.read_avro}[ptype](buf)
            fr = formats.to_frame(grid, 1 if ptype == "AVRO" else header, col_types)
        elif ptype in ("ORC", "FEATHER"):
            if ptype == "FEATHER":
                import pyarrow.feather as pf
                fr = H2OFrame(pf.read_table(io.BytesIO(buf)).to_pandas())
            else:
                import pyarrow.orc as po
                fr = H2OFrame(po.ORCFile(io.BytesIO(buf)).read().to_pandas())
        else:
            if dist_parse:
                fr = _parse_csv_distributed(f, sep, header, col_names, col_types, na_strings, skipped_columns,
                                            custom_non_data_line_markers)
                if i > 0 and frames and fr.names != frames[0].names:
                    fr.names = frames[0].names
                frames.append(fr)
                continue
            if custom_non_data_line_markers:
                keep = [ln for ln in buf.split(b"\n") if not any(ln.startswith(m.encode()) for m in custom_non_data_line_markers)]
                buf = b"\n".join(keep)
            # every file after the first repeats the header if the first had one (ParseSetup)
            fr = _parse_csv_bytes(buf, sep, header, col_names, col_types, na_strings, skipped_columns=skipped_columns)
            if i > 0 and frames and fr.names != frames[0].names:
                fr.names = frames[0].names
        frames.append(fr)
    if dframe.active() and not dframe.in_method():
        # non-CSV formats are read whole on every rank: keep this rank's rows
        frames = [fr if fr._shard is not None else dframe.shard_frame(fr) for fr in frames]
    out = frames[0] if len(frames) == 1 else _rbind_sharded(frames)
    _detect_uuid(out, col_types)
    from ..frame import compress_frame
    compress_frame(out)             # integer / short-decimal numeric columns as 8/16/32-bit codes
    dest = destination_frame or _dest_name(files[0])
    from ..core import dkv
    dkv.remove(out.frame_id) if out.frame_id != dest and dkv.contains(out.frame_id) else None
    out.frame_id = dest
    dkv.put(dest, out)
    return out


def _detect_uuid(fr, col_types=None):
    """ParseSetup's UUID type: a string (or enum) column whose every value is a UUID becomes a ``uuid``
    column (two int64 halves per row); an explicit ``col_types`` entry "uuid" forces it."""
    from ..frame import looks_uuid, uuid_column
    forced = set()
    if isinstance(col_types, dict):
        forced = {k for k, v in col_types.items() if str(v).lower() == "uuid"}
    elif isinstance(col_types, (list, tuple)):
        forced = {fr.names[i] for i, v in enumerate(col_types) if i < fr.ncols and str(v).lower() == "uuid"}
    for n in list(fr.names):
        c = fr._col(n)
        if c.type not in ("string", "enum"):
            continue
        vals = c.to_numpy()
        if n in forced or looks_uuid(vals[: 1000]) and looks_uuid(vals):
            dev = c.data.device if c.data is not None else None
            fr._cols[n] = uuid_column(n, list(vals), dev)


def _rbind_sharded(frames):
    """Row-bind per-file frames. Sharded parts are bound rank-locally (each rank keeps its own rows of
    every file), so a multi-file import stays sharded; domains are unified over files and ranks."""
    if all(f._shard is None for f in frames):
        return frames[0].rbind(frames[1:])
    from ..parallel import dframe
    cols = []
    for n, c in frames[0]._cols.items():
        parts = [f._col(n) for f in frames]
        if c.type == "enum":
            dom = sorted(set().union(*[p.domain for p in parts]))
            lut = {s: i for i, s in enumerate(dom)}
            codes = []
            for p in parts:
                m = torch.tensor([lut[s] for s in p.domain] + [-1], dtype=torch.int32, device=p.data.device)
                codes.append(m[torch.where(p.data < 0, torch.full_like(p.data, len(p.domain)), p.data).long()])
            cols.append(Column(n, "enum", torch.cat(codes), dom))
        elif c.type == "string":
            cols.append(Column(n, "string", strings=np.concatenate([p.strings for p in parts])))
        else:
            cols.append(Column(n, c.type if all(p.type == c.type for p in parts) else "real",
                               torch.cat([p.as_float() for p in parts])))
    with dframe.shard_ctx(dframe.make_shard(cols[0].n if cols else 0)):
        return H2OFrame._from_columns(cols)


def upload_file(path, destination_frame=None, header=0, sep=None, col_names=None, col_types=None, na_strings=None,
                skipped_columns=None) -> H2OFrame:
    return import_file(path, destination_frame, header=header, sep=sep, col_names=col_names, col_types=col_types,
                       na_strings=na_strings, skipped_columns=skipped_columns)


def parse_raw_text(text: str, destination_frame=None, header=0, sep=None, col_types=None) -> H2OFrame:
    fr = _parse_csv_bytes(text.encode(), sep, header, None, col_types, None)
    if destination_frame:
        from ..core import dkv
        fr.frame_id = destination_frame
        dkv.put(destination_frame, fr)
    return fr


# ------------------------------------------------------------------------------------------------
def _fmt(v) -> str:
    if v is None:
        return ""
    if isinstance(v, float):
        if math.isnan(v):
            return ""
        if v.is_integer() and abs(v) < 1e15:
            return str(int(v))
        return repr(v)
    s = str(v)
    if any(ch in s for ch in ',"\n'):
        s = '"' + s.replace('"', '""') + '"'
    return s


def export_file(frame: H2OFrame, path: str, force: bool = False, sep: str = ",", header: bool = True,
                quote_header: bool = True, parts: int = 1, compression=None) -> str:
    """``h2o.export_file`` (CSV). ``parts > 1`` writes ``path/part-m-XXXXX`` like the reference."""
    if os.path.exists(path) and not force and parts <= 1:
        raise FileExistsError(f"{path} exists (use force=True)")
    cols = [frame._col(n) for n in frame.names]
    data = []
    for c in cols:
        if c.type == "time":
            import pandas as pd
            v = c.to_numpy()
            data.append([None if np.isnan(x) else str(pd.Timestamp(int(x), unit="ms")) for x in v])
        elif c.type in ("real", "int"):
            data.append([float(x) for x in c.to_numpy()])
        else:
            data.append(list(c.to_numpy()))
    n = frame.nrows

    def write(fh, lo, hi):
        if header:
            fh.write(sep.join((f'"{nm}"' if quote_header else nm) for nm in frame.names) + "\n")
        for r in range(lo, hi):
            fh.write(sep.join(_fmt(col[r]) for col in data) + "\n")

    opener = (lambda p: gzip.open(p, "wt")) if compression == "gzip" else (lambda p: open(p, "w"))
    if parts > 1:
        os.makedirs(path, exist_ok=True)
        for k in range(parts):
            with opener(os.path.join(path, f"part-m-{k:05d}")) as fh:
                write(fh, n * k // parts, n * (k + 1) // parts)
    else:
        with opener(path) as fh:
            write(fh, 0, n)
    return path


# ------------------------------------------------------------------------------------------------
def save_frame(frame: H2OFrame, dir_path: str, force: bool = True) -> str:
    """Binary frame save (``h2o.save_frame``): one safetensors file of device columns + JSON metadata."""
    import json
    from safetensors.torch import save_file
    os.makedirs(dir_path, exist_ok=True)
    meta, tensors = [], {}
    for i, n in enumerate(frame.names):
        c = frame._col(n)
        m = dict(name=n, type=c.type, domain=c.domain)
        if c.type == "string":
            m["strings"] = [None if s is None else str(s) for s in c.strings]
        else:
            tensors[f"c{i}"] = c.data.detach().cpu().contiguous()
        meta.append(m)
    save_file(tensors, os.path.join(dir_path, "columns.safetensors"))
    with open(os.path.join(dir_path, "frame.json"), "w") as f:
        json.dump(dict(frame_id=frame.frame_id, nrows=frame.nrows, columns=meta), f)
    return dir_path


def load_frame(frame_id: str | None, dir_path: str) -> H2OFrame:
    import json
    from safetensors.torch import load_file
    with open(os.path.join(dir_path, "frame.json")) as f:
        meta = json.load(f)
    tens = load_file(os.path.join(dir_path, "columns.safetensors"))
    dev = engine_device()
    cols = []
    for i, m in enumerate(meta["columns"]):
        if m["type"] == "string":
            cols.append(Column(m["name"], "string", strings=np.array(m["strings"], dtype=object)))
        else:
            cols.append(Column(m["name"], m["type"], tens[f"c{i}"].to(dev), m.get("domain")))
    return H2OFrame._from_columns(cols, frame_id or meta["frame_id"])
