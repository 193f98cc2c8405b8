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
                 "time": "time", "date": "time", "uuid": "string"}


# ------------------------------------------------------------------------------------------------
def _read_bytes(path: str) -> bytes:
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
                na_strings=None) -> dict:
    """``/3/ParseSetup``: guess parse type, separator, header, column names and types."""
    files = _expand(path)
    head = _read_bytes(files[0])[: 1 << 20]
    ptype = guess_parse_type(files[0], head)
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
                     skipped_columns=None) -> H2OFrame:
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
        if column_names:
            names = list(column_names) + names[len(column_names):]
        ctypes_ = _normalize_types(column_types, names)
        na_set = _na_sets(na_strings, names)
        skip = set(skipped_columns or [])
        cols = []
        num = np.empty(n, dtype=np.float64)
        kind = np.empty(n, dtype=np.uint8)
        for c in range(nc):
            if c in skip or names[c] in skip:
                continue
            forced = ctypes_.get(names[c])
            rt.h2o_csv_get(h, c, num.ctypes.data, kind.ctypes.data, None, None)
            n_num = rt.h2o_csv_count(h, c, 1)
            n_txt = rt.h2o_csv_count(h, c, 2)
            nas = na_set.get(names[c])
            want_text = forced in ("enum", "string") or (forced is None and n_txt > n_num) or bool(nas)
            if want_text:
                codes = np.empty(n, dtype=np.int32)
                d = rt.h2o_csv_domain(h, buf, c, codes.ctypes.data)
                try:
                    L = rt.h2o_domain_size(d)
                    dom = []
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
                    cols.append(Column(names[c], t, torch.as_tensor(vals, device=device)))
        return H2OFrame._from_columns(cols)
    finally:
        rt.h2o_csv_free(h)


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
                partition_by=None, quotechar=None, escapechar=None) -> H2OFrame:
    """``h2o.import_file``: file, directory, glob or list; multiple files are row-bound (ParseDataset)."""
    files = _expand(path)
    if pattern:
        import re
        rx = re.compile(pattern)
        files = [f for f in files if rx.search(os.path.basename(f))]
    if not files:
        raise FileNotFoundError(f"no files match {path}")
    frames = []
    for i, f in enumerate(files):
        buf = _read_bytes(f)
        ptype = guess_parse_type(f, buf[:4096])
        if ptype == "SVMLight":
            fr = parse_svmlight(buf)
        elif ptype == "ARFF":
            fr = parse_arff(buf)
        elif ptype == "PARQUET":
            fr = parse_parquet(f)
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
            if custom_non_data_line_markers:
                keep = [ln for ln in buf.split(b"\n") if not any(ln.startswith(m.encode()) for m in custom_non_data_line_markers)]
                buf = b"\n".join(keep)
            # every file after the first repeats the header if the first had one (ParseSetup)
            fr = _parse_csv_bytes(buf, sep, header, col_names, col_types, na_strings, skipped_columns=skipped_columns)
            if i > 0 and frames and fr.names != frames[0].names:
                fr.names = frames[0].names
        frames.append(fr)
    out = frames[0] if len(frames) == 1 else frames[0].rbind(frames[1:])
    dest = destination_frame or _dest_name(files[0])
    from ..core import dkv
    dkv.remove(out.frame_id) if out.frame_id != dest and dkv.contains(out.frame_id) else None
    out.frame_id = dest
    dkv.put(dest, out)
    return out


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
