"""Columnar frames resident in device memory (reference: ``water/fvec/Frame.java``, ``Vec.java``,
``RollupStats.java`` and the h2o-py ``H2OFrame`` API, ``h2o-py/h2o/frame.py``).

A :class:`Column` holds one typed vector:

* ``real`` / ``int``  -> float64 tensor, NaN = missing
* ``enum``            -> int32 codes into ``domain`` (sorted level strings), -1 = missing
* ``string``          -> numpy object array (host), None = missing
* ``time``            -> float64 ms since epoch, NaN = missing
* ``uuid``            -> int64 [N, 2] (high, low 64 bits; C16Chunk), both INT64_MIN = missing

Numeric/enum tensors live on the engine device (HBM on MI355X); every reduction and elementwise op
runs there through torch. :meth:`H2OFrame.model_matrix` adapts any frame to a trained model's
``DataInfo`` (column order, categorical level remapping, unseen levels -> NA) and returns the
float32 [F, N] column-major matrix the HIP kernels consume.
"""
from __future__ import annotations

import copy
import math
import re
from collections import OrderedDict

import numpy as np
import torch

from .core import dkv
from .parallel import dframe

_NUMERIC = ("real", "int", "time")


def engine_device():
    from .core import runtime
    return runtime.device()


# ================================================================================================
class Column:
    __slots__ = ("name", "type", "_data", "domain", "strings", "_spilled", "_codec")

    def __init__(self, name, type_, data=None, domain=None, strings=None):
        self.name = name
        self.type = type_
        self._data = data
        self._spilled = None
        self._codec = None
        self.domain = domain
        self.strings = strings

    # device residency: a column spilled by the memory manager comes back on first access; a compressed
    # column (see compress()) is decoded for good on the first ``data`` access (callers may write it)
    @property
    def data(self):
        if self._spilled is not None:
            from .utils import memory
            memory.restore_column(self)
        if self._codec is not None:
            self._data, self._codec = _decode(self._data, self._codec), None
        return self._data

    @data.setter
    def data(self, v):
        self._data = v
        self._spilled = None
        self._codec = None

    def raw_data(self):
        return self._data

    def set_raw_data(self, v, spilled_from=None):
        self._data = v
        self._spilled = spilled_from

    def spilled_device(self):
        return self._spilled

    # ---- chunk compression (water/fvec C1/C2/C4 and the scaled C1S/C2S/C4S chunks)
    def compress(self) -> int:
        """Store a numeric column as 8/16/32-bit integer codes when every value is an integer or a decimal
        with at most 4 places whose scaled range fits (NA = the type's minimum); values decode bit-exactly
        as (code + base) / 10^k. Returns the bytes saved (0: left as is)."""
        if self.type not in ("real", "int") or self._codec is not None or self._spilled is not None:
            return 0
        d = self._data
        if d is None or not torch.is_floating_point(d) or d.dim() != 1:
            return 0
        enc = _encode(d)
        if enc is None:
            return 0
        codes, codec = enc
        saved = d.numel() * d.element_size() - codes.numel() * codes.element_size()
        if saved <= 0:
            return 0
        self._data, self._codec = codes, codec
        return saved

    @property
    def compressed(self) -> bool:
        return self._codec is not None

    def values(self) -> torch.Tensor:
        """Read-only numeric values without decoding the column for good (model matrices, statistics)."""
        if self._codec is None:
            return self.data
        if self._spilled is not None:
            from .utils import memory
            memory.restore_column(self)
        return _decode(self._data, self._codec)

    @property
    def n(self):
        if self._codec is not None:
            return int(self._data.numel())
        if self.type == "string":
            return len(self.strings)
        if self.type == "uuid":
            return int(self.data.shape[0])
        return int(self.data.numel())

    def copy(self):
        return Column(self.name, self.type, None if self.data is None else self.data.clone(),
                      None if self.domain is None else list(self.domain),
                      None if self.strings is None else self.strings.copy())

    def isna(self) -> torch.Tensor:
        if self.type == "uuid":
            return (self.data[:, 0] == _UUID_NA) & (self.data[:, 1] == _UUID_NA)
        if self.type == "enum":
            return self.data < 0
        if self.type == "string":
            return torch.from_numpy(np.array([s is None for s in self.strings], dtype=bool)).to(engine_device())
        return torch.isnan(self.data)

    def as_float(self) -> torch.Tensor:
        """Numeric view: enum -> code (NaN for NA), numeric as is, string -> NaN."""
        if self.type == "enum":
            d = self.data.double()
            return torch.where(self.data < 0, torch.full_like(d, float("nan")), d)
        if self.type == "string":
            vals = np.array([_to_float(s) for s in self.strings], dtype=np.float64)
            return torch.from_numpy(vals).to(engine_device())
        if self.type == "uuid":
            return torch.full((self.n,), float("nan"), dtype=torch.float64, device=self.data.device)
        return self.values()

    def take(self, idx: torch.Tensor):
        if self.type == "string":
            return Column(self.name, self.type, strings=self.strings[idx.cpu().numpy()])
        return Column(self.name, self.type, self.data[idx.to(self.data.device)], self.domain)

    def to_numpy(self):
        if self.type == "string":
            return self.strings
        if self.type == "uuid":
            return uuid_strings(self.data)
        if self.type == "enum":
            codes = self.data.cpu().numpy()
            dom = np.array(self.domain + [None], dtype=object)
            return dom[np.where(codes < 0, len(self.domain), codes)]
        return self.data.cpu().numpy()


_CODEC_MIN_ROWS = 1024


def _encode(x: torch.Tensor):
    """(int codes, (base, k, dtype)) with x == (codes + base) / 10^k bit for bit (NaN <-> the minimum code),
    or None. Tries k = 0..4 decimal places, the narrowest of int8 / int16 / int32."""
    if x.numel() < _CODEC_MIN_ROWS or bool(torch.isinf(x).any()):
        return None
    fin = ~torch.isnan(x)
    v = x[fin].double()
    if v.numel() == 0 or bool(((v == 0) & torch.signbit(v)).any()):
        return None                  # empty, or a -0.0 that integer codes would decode as +0.0
    for k in range(5):
        p = float(10 ** k)
        sv = torch.round(v * p)
        if float(sv.abs().max()) >= 2.0 ** 52:
            return None
        if not torch.equal((sv / p).to(x.dtype), x[fin]):
            continue
        lo, hi = float(sv.min()), float(sv.max())
        for dt, bits in ((torch.int8, 8), (torch.int16, 16), (torch.int32, 32)):
            half = 2 ** (bits - 1)
            if hi - lo <= 2 * half - 2:
                base = lo + half - 1
                codes = torch.full(x.shape, -half, dtype=dt, device=x.device)
                codes[fin] = (sv - base).to(dt)
                return codes, (base, k, x.dtype)
        return None
    return None


def _decode(codes: torch.Tensor, codec) -> torch.Tensor:
    base, k, dt = codec
    na = codes == torch.iinfo(codes.dtype).min
    v = (codes.double() + base) / float(10 ** k)
    return torch.where(na, torch.full_like(v, float("nan")), v).to(dt)


def compress_frame(fr) -> int:
    """Compress every numeric column of a frame (parse-time default, as the reference's chunk encodings);
    H2O_COMPRESS=0 turns it off. Returns the bytes saved."""
    import os
    if os.environ.get("H2O_COMPRESS", "1") == "0":
        return 0
    return sum(c.compress() for c in fr._cols.values())


_UUID_NA = -(1 << 63)
_UUID_RX = re.compile(r"^[0-9a-fA-F]{8}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{4}-[0-9a-fA-F]{12}$")


def _signed(v: int) -> int:
    return v - (1 << 64) if v >= (1 << 63) else v


def uuid_column(name, values, device=None) -> "Column":
    """UUID strings -> a ``uuid`` column (two signed 64-bit halves per row, C16Chunk layout)."""
    import uuid as _uuid
    out = np.full((len(values), 2), _UUID_NA, dtype=np.int64)
    for i, v in enumerate(values):
        if v is None or (isinstance(v, float) and math.isnan(v)) or str(v).strip() == "":
            continue
        u = _uuid.UUID(str(v).strip()).int
        out[i, 0], out[i, 1] = _signed(u >> 64), _signed(u & ((1 << 64) - 1))
    return Column(name, "uuid", torch.as_tensor(out, device=device or engine_device()))


def uuid_strings(data: torch.Tensor):
    import uuid as _uuid
    a = data.cpu().numpy()
    out = np.empty(a.shape[0], dtype=object)
    for i, (hi, lo) in enumerate(a.tolist()):
        out[i] = None if hi == _UUID_NA and lo == _UUID_NA else str(_uuid.UUID(int=((hi % (1 << 64)) << 64) | (lo % (1 << 64))))
    return out


def looks_uuid(values) -> bool:
    vals = [v for v in values if v is not None and not (isinstance(v, float) and math.isnan(v)) and str(v) != ""]
    return bool(vals) and all(isinstance(v, str) and _UUID_RX.match(v.strip()) for v in vals)


def _to_float(s):
    try:
        return float(s)
    except (TypeError, ValueError):
        return float("nan")


def _infer_column(name, values, device, force_type=None) -> Column:
    """Build a column from a python/numpy/pandas sequence (ParseSetup-like type guessing)."""
    if isinstance(values, torch.Tensor):
        arr = values.detach()
        if force_type == "enum":
            return _enum_from_values(name, arr.cpu().numpy(), device)
        t = "int" if not torch.is_floating_point(arr) else "real"
        return Column(name, force_type or t, arr.to(device=device, dtype=torch.float64))
    arr = np.asarray(values, dtype=object) if not isinstance(values, np.ndarray) else values
    if force_type in ("enum", "factor", "categorical"):
        return _enum_from_values(name, arr, device)
    if force_type == "string":
        return Column(name, "string", strings=np.array([None if _isnull(v) else str(v) for v in arr], dtype=object))
    if force_type == "uuid":
        return uuid_column(name, list(arr), device)
    if arr.dtype.kind in "biuf":
        t = "int" if arr.dtype.kind in "biu" else "real"
        if force_type == "time":
            t = "time"
        return Column(name, t, torch.as_tensor(arr.astype(np.float64), device=device))
    if arr.dtype.kind == "M":
        ms = arr.astype("datetime64[ms]").astype(np.int64).astype(np.float64)
        ms[np.isnat(arr)] = np.nan
        return Column(name, "time", torch.as_tensor(ms, device=device))
    # object: numeric if every non-null parses
    vals = np.empty(len(arr), dtype=np.float64)
    numeric = True
    for i, v in enumerate(arr):
        if _isnull(v):
            vals[i] = np.nan
            continue
        if isinstance(v, (bool, np.bool_)):
            vals[i] = float(v)
            continue
        if isinstance(v, (int, float, np.integer, np.floating)):
            vals[i] = float(v)
            continue
        f = _to_float(v)
        if math.isnan(f) and str(v).strip().lower() not in ("nan", "na"):
            numeric = False
            break
        vals[i] = f
    if numeric and force_type != "string":
        isint = bool(np.all(np.isnan(vals) | (vals == np.round(vals))))
        return Column(name, "int" if isint else "real", torch.as_tensor(vals, device=device))
    return _enum_from_values(name, arr, device)


def _isnull(v):
    if v is None:
        return True
    if isinstance(v, float) and math.isnan(v):
        return True
    try:
        import pandas as pd
        return bool(pd.isna(v)) if not isinstance(v, (list, tuple, np.ndarray)) else False
    except Exception:  # noqa: BLE001
        return False


def _enum_from_values(name, arr, device) -> Column:
    strs = np.array([None if _isnull(v) else _level_str(v) for v in arr], dtype=object)
    mask = np.array([s is not None for s in strs], dtype=bool)
    dom = sorted(set(strs[mask].tolist()), key=_level_key)
    lut = {s: i for i, s in enumerate(dom)}
    codes = np.full(len(strs), -1, dtype=np.int32)
    codes[mask] = [lut[s] for s in strs[mask]]
    return Column(name, "enum", torch.as_tensor(codes, device=device), dom)


def _level_str(v):
    if isinstance(v, (float, np.floating)) and float(v).is_integer():
        return str(int(v))
    return str(v)


def _level_key(s):
    # H2O sorts numeric-looking levels numerically when all are numbers, else lexicographically
    return s


# ================================================================================================
class H2OFrame:
    """Distributed-in-HBM frame with the h2o-py ``H2OFrame`` API surface."""

    @property
    def frame_id(self):
        """The frame's key in the DKV (reference ``h2o-py/h2o/frame.py:392``)."""
        return self.__dict__.get("_frame_id")

    @frame_id.setter
    def frame_id(self, newid):
        # assigning a new id renames the frame's DKV entry (the reference's setter issues a Rapids ``rename``)
        # A frame a running job write-locks cannot be renamed (the reference's Rapids rename fails on a locked key):
        # the rename raises and the frame keeps its one key.
        old = self.__dict__.get("_frame_id")
        if old is not None and newid != old and dkv.contains(old) and dkv.get(old) is self:
            dkv.remove(old)          # RuntimeError while write-locked: nothing changed
            self.__dict__["_frame_id"] = newid
            dkv.put(newid, self)
            return
        self.__dict__["_frame_id"] = newid

    def __init__(self, python_obj=None, destination_frame=None, header=0, separator=",", column_names=None,
                 column_types=None, na_strings=None, skipped_columns=None):
        self._cols: "OrderedDict[str, Column]" = OrderedDict()
        self._shard = None
        self.frame_id = destination_frame or dkv.new_key("py_frame")
        if python_obj is not None:
            self._from_python(python_obj, column_names, column_types)
            if dframe.active() and not dframe.in_method() and self._cols and self._nlocal > 1:
                # a user-built frame under torchrun: every rank was handed the same object (SPMD); keep
                # this rank's row range (ParseDataset distributes rows the same way)
                cols, self._shard = dframe.shard_columns(list(self._cols.values()), self._nlocal)
                self._cols = OrderedDict((c.name, c) for c in cols)
        dkv.put(self.frame_id, self)

    # ---- construction
    @classmethod
    def _from_columns(cls, cols, frame_id=None) -> "H2OFrame":
        f = cls.__new__(cls)
        f._cols = OrderedDict()
        f._shard = dframe.current_ctx()
        for c in cols:
            name = c.name
            k = 0
            while name in f._cols:
                k += 1
                name = f"{c.name}{k}"
            c.name = name
            f._cols[name] = c
        f.frame_id = frame_id or dkv.new_key("frame")
        dkv.put(f.frame_id, f)
        return f

    def _from_python(self, obj, column_names=None, column_types=None):
        dev = engine_device()
        types = column_types or {}
        try:
            import pandas as pd
        except ImportError:  # pragma: no cover
            pd = None
        if pd is not None and isinstance(obj, pd.DataFrame):
            names = [str(c) for c in obj.columns]
            cols = []
            for n, orig in zip(names, obj.columns):
                s = obj[orig]
                ft = types.get(n) if isinstance(types, dict) else None
                if str(s.dtype) == "category":
                    ft = ft or "enum"
                    cols.append(_infer_column(n, s.astype(object).values, dev, ft))
                else:
                    cols.append(_infer_column(n, s.values, dev, ft))
            for c in cols:
                self._cols[c.name] = c
            return
        if isinstance(obj, dict):
            for n, v in obj.items():
                ft = types.get(n) if isinstance(types, dict) else None
                c = _infer_column(str(n), v if not isinstance(v, (int, float, str)) else [v], dev, ft)
                self._cols[c.name] = c
            return
        if isinstance(obj, torch.Tensor):
            obj = obj.detach().cpu().numpy()
        if isinstance(obj, np.ndarray) and obj.ndim == 2:
            names = column_names or [f"C{i + 1}" for i in range(obj.shape[1])]
            for i, n in enumerate(names):
                ft = types[i] if isinstance(types, (list, tuple)) and i < len(types) else (types.get(n) if isinstance(types, dict) else None)
                c = _infer_column(n, obj[:, i], dev, ft)
                self._cols[n] = c
            return
        if isinstance(obj, (list, tuple)):
            if len(obj) and isinstance(obj[0], (list, tuple)):
                rows = obj
                ncol = max(len(r) for r in rows)
                names = column_names or [f"C{i + 1}" for i in range(ncol)]
                for i, n in enumerate(names):
                    vals = [r[i] if i < len(r) else None for r in rows]
                    ft = types[i] if isinstance(types, (list, tuple)) and i < len(types) else None
                    c = _infer_column(n, vals, dev, ft)
                    self._cols[n] = c
            else:
                n = (column_names or ["C1"])[0]
                self._cols[n] = _infer_column(n, list(obj), dev)
            return
        raise TypeError(f"cannot build an H2OFrame from {type(obj)}")

    @staticmethod
    def from_predictions(P: torch.Tensor, category: str, domain, threshold=None, names=None,
                         labels=None) -> "H2OFrame":
        dev = P.device
        if names is not None:
            P2 = P if P.dim() == 2 else P.reshape(-1, 1)
            return H2OFrame._from_columns([Column(n, "real", P2[:, i].double()) for i, n in enumerate(names)])
        if category == "Binomial":
            p1 = P[:, 1].double()
            th = 0.5 if threshold is None else threshold
            lab = (p1 >= th).int()
            cols = [Column("predict", "enum", lab.to(torch.int32), list(domain))]
            cols += [Column(str(d), "real", P[:, i].double()) for i, d in enumerate(domain)]
            return H2OFrame._from_columns(cols)
        if category == "Multinomial":
            lab = (P.argmax(1) if labels is None else labels).to(torch.int32)
            cols = [Column("predict", "enum", lab, list(domain))]
            cols += [Column(str(d), "real", P[:, i].double()) for i, d in enumerate(domain)]
            return H2OFrame._from_columns(cols)
        if P.dim() == 2 and P.shape[1] > 1:
            return H2OFrame._from_columns([Column(f"C{i + 1}", "real", P[:, i].double()) for i in range(P.shape[1])])
        return H2OFrame._from_columns([Column("predict", "real", P.reshape(-1).double())])

    @staticmethod
    def from_tensor(t: torch.Tensor, names=None) -> "H2OFrame":
        t = t if t.dim() == 2 else t.reshape(-1, 1)
        names = names or [f"C{i + 1}" for i in range(t.shape[1])]
        return H2OFrame._from_columns([Column(n, "real", t[:, i].double().to(engine_device())) for i, n in enumerate(names)])

    # ---- shape / metadata
    @property
    def names(self):
        return list(self._cols.keys())

    @names.setter
    def names(self, value):
        self.set_names(value)

    columns = names

    @property
    def col_names(self):
        return self.names

    @property
    def nrows(self):
        if self._shard is not None:
            return self._shard.n_global
        return self._nlocal

    @property
    def _nlocal(self):
        """Rows held by this rank (== nrows unless the frame is row-sharded)."""
        return next(iter(self._cols.values())).n if self._cols else 0

    @property
    def is_sharded(self):
        return self._shard is not None

    def gather(self):
        """Replicated copy of a sharded frame (every rank gets every row); self if not sharded."""
        return dframe.gather_frame(self)

    def reshard(self):
        """Sharded copy of a replicated frame under a multi-rank cloud (self otherwise)."""
        return dframe.shard_frame(self)

    nrow = nrows

    @property
    def ncols(self):
        return len(self._cols)

    ncol = ncols

    @property
    def shape(self):
        return (self.nrows, self.ncols)

    def dim(self):
        return [self.nrows, self.ncols]

    @property
    def types(self):
        return {n: c.type for n, c in self._cols.items()}

    @property
    def dtypes(self):
        return [c.type for c in self._cols.values()]

    def type(self, col):
        return self._col(col).type

    def columns_by_type(self, coltype="numeric"):
        out = []
        for i, c in enumerate(self._cols.values()):
            if (coltype == "numeric" and c.type in ("real", "int")) or (coltype == "categorical" and c.type == "enum") \
                    or (coltype == "string" and c.type == "string") or (coltype == "time" and c.type == "time"):
                out.append(float(i))
        return out

    def __len__(self):
        return self.nrows

    def _col(self, c) -> Column:
        if isinstance(c, (int, np.integer)):
            return list(self._cols.values())[int(c)]
        return self._cols[c]

    def _resolve(self, item):
        if isinstance(item, str):
            return [item]
        if isinstance(item, (int, np.integer)):
            return [self.names[int(item)]]
        if isinstance(item, slice):
            return self.names[item]
        if isinstance(item, (list, tuple)):
            if all(isinstance(x, (bool, np.bool_)) for x in item):
                return [n for n, b in zip(self.names, item) if b]
            return [self.names[int(x)] if isinstance(x, (int, np.integer)) else x for x in item]
        raise KeyError(item)

    def set_names(self, names):
        assert len(names) == self.ncols
        self._cols = OrderedDict((n, c) for n, c in zip(names, self._cols.values()))
        for n, c in self._cols.items():
            c.name = n
        return self

    def set_name(self, col=None, name=None):
        old = self._col(col if col is not None else 0).name
        newcols = OrderedDict()
        for n, c in self._cols.items():
            if n == old:
                c.name = name
                newcols[name] = c
            else:
                newcols[n] = c
        self._cols = newcols
        return self

    def rename(self, columns=None):
        for old, new in (columns or {}).items():
            self.set_name(old, new)
        return self

    # ---- indexing
    def __getitem__(self, item):
        if isinstance(item, tuple) and len(item) == 2:
            rows, cols = item
            fr = self[cols] if not (isinstance(cols, slice) and cols == slice(None)) else self
            return fr._rows(rows)
        if isinstance(item, H2OFrame):  # boolean mask
            return self._rows(item)
        with dframe.shard_ctx(self._shard):
            return H2OFrame._from_columns([self._col(n) for n in self._resolve(item)])

    def _rows(self, rows):
        if self._shard is not None or (isinstance(rows, H2OFrame) and rows._shard is not None):
            return self._rows_sharded(rows)
        n = self.nrows
        dev = engine_device()
        if isinstance(rows, H2OFrame):
            m = rows._col(0).as_float()
            idx = torch.nonzero(torch.nan_to_num(m, nan=0.0) != 0).reshape(-1)
        elif isinstance(rows, slice):
            idx = torch.arange(n, device=dev)[rows]
        elif isinstance(rows, (int, np.integer)):
            idx = torch.tensor([int(rows) % n], device=dev)
        elif isinstance(rows, torch.Tensor):
            idx = torch.nonzero(rows).reshape(-1) if rows.dtype == torch.bool else rows.long()
        else:
            idx = torch.as_tensor(np.asarray(rows), device=dev).long()
        return H2OFrame._from_columns([c.take(idx) for c in self._cols.values()])

    def _rows_sharded(self, rows):
        """Row selection on a sharded frame: masks and ascending global indices / slices stay local
        (the new shard's offsets come from one all-gather of the kept counts); anything that reorders
        rows runs on the gathered frame."""
        me = self
        if me._shard is None:
            me = dframe.shard_frame(me) if me.nrows == rows.nrows else me
        sh = me._shard
        dev = engine_device()
        local = None
        if isinstance(rows, H2OFrame):
            if rows._shard != sh:
                if rows._shard is None and rows.nrows == me.nrows:
                    rows = dframe.shard_frame(rows)
                else:
                    return dframe.gather_frame(me)._rows(dframe.gather_frame(rows))
            m = rows._col(0).as_float()
            local = torch.nonzero(torch.nan_to_num(m, nan=0.0) != 0).reshape(-1)
        elif isinstance(rows, torch.Tensor) and rows.dtype == torch.bool and rows.numel() == sh.n_local:
            local = torch.nonzero(rows).reshape(-1).to(dev)
        elif isinstance(rows, slice) and (rows.step or 1) > 0:
            g = range(sh.n_global)[rows]
            lo, hi = max(g.start, sh.offset), min(g.stop, sh.offset + sh.n_local)
            st = g.step
            first = lo + ((g.start - lo) % st) if lo > g.start else g.start
            local = torch.arange(first - sh.offset, max(hi - sh.offset, first - sh.offset), st, device=dev)
        elif isinstance(rows, (int, np.integer, list, np.ndarray)) or (isinstance(rows, torch.Tensor) and rows.dtype != torch.bool):
            idx = np.atleast_1d(rows.cpu().numpy() if isinstance(rows, torch.Tensor) else np.asarray(rows)).astype(np.int64)
            idx = np.where(idx < 0, idx + sh.n_global, idx)
            if idx.size > 1 and np.any(np.diff(idx) <= 0):
                return dframe.gather_frame(me)._rows(idx)
            sel = idx[(idx >= sh.offset) & (idx < sh.offset + sh.n_local)] - sh.offset
            local = torch.as_tensor(sel, device=dev)
        else:
            return dframe.gather_frame(me)._rows(rows)
        with dframe.shard_ctx(dframe.make_shard(int(local.numel()))):
            return H2OFrame._from_columns([c.take(local) for c in me._cols.values()])

    def __setitem__(self, key, value):
        n = self._nlocal if self._cols else None
        if self._shard is not None and isinstance(value, H2OFrame) and value._shard is None and \
                value.nrows == self.nrows and self.nrows > 1:
            value = dframe.shard_frame(value)
        if self._shard is not None and isinstance(key, tuple) and isinstance(key[0], H2OFrame) and \
                key[0]._shard is None and key[0].nrows == self.nrows:
            key = (dframe.shard_frame(key[0]), key[1])
        if self._shard is not None and not isinstance(value, (H2OFrame, int, float, str)) and value is not None \
                and hasattr(value, "__len__") and len(value) == self.nrows:
            lo, hi = dframe.bounds(self.nrows)
            value = value[lo:hi]
        dev = engine_device()
        if isinstance(key, tuple):  # (row mask, col) assignment
            rows, col = key
            c = self._col(col)
            mask = rows._col(0).as_float().nan_to_num(0) != 0 if isinstance(rows, H2OFrame) else rows
            v = value._col(0).as_float() if isinstance(value, H2OFrame) else torch.full((c.n,), float(value), dtype=torch.float64, device=dev)
            if c.type == "enum" and isinstance(value, str):
                code = c.domain.index(value) if value in c.domain else None
                if code is None:
                    c.domain = c.domain + [value]
                    code = len(c.domain) - 1
                c.data = torch.where(mask, torch.full_like(c.data, code), c.data)
            else:
                base = c.as_float()
                c.data = torch.where(mask, v, base)
                c.type = "real" if c.type == "enum" else c.type
                c.domain = None
            return
        name = key if isinstance(key, str) else self.names[int(key)]
        if isinstance(value, H2OFrame):
            c = value._col(0)
            c = Column(name, c.type, c.data, c.domain, c.strings)
        elif isinstance(value, (int, float)):
            c = Column(name, "real", torch.full((n,), float(value), dtype=torch.float64, device=dev))
        elif isinstance(value, str):
            c = Column(name, "enum", torch.zeros(n, dtype=torch.int32, device=dev), [value])
        else:
            c = _infer_column(name, value, dev)
        self._cols[name] = c

    def __delitem__(self, key):
        for n in self._resolve(key):
            del self._cols[n]

    def drop(self, index, axis=1):
        if axis == 0:
            if self._shard is not None:
                return dframe.gather_frame(self).drop(index, axis)
            keep = torch.ones(self.nrows, dtype=torch.bool, device=engine_device())
            keep[torch.as_tensor(np.atleast_1d(index), device=keep.device).long()] = False
            return self._rows(keep)
        names = set(self._resolve(index))
        with dframe.shard_ctx(self._shard):
            return H2OFrame._from_columns([c for n, c in self._cols.items() if n not in names])

    def pop(self, i):
        n = self._resolve(i)[0]
        c = self._cols.pop(n)
        with dframe.shard_ctx(self._shard):
            return H2OFrame._from_columns([c])

    # ---- conversion
    def as_data_frame(self, use_pandas=True, header=True, use_multi_thread=False):
        if self._shard is not None:
            return dframe.gather_frame(self).as_data_frame(use_pandas, header, use_multi_thread)
        import pandas as pd
        data = OrderedDict()
        for n, c in self._cols.items():
            v = c.to_numpy()
            if c.type == "time":
                v = pd.to_datetime(v, unit="ms")
            elif c.type == "int":
                v = v.copy()
            data[n] = v
        df = pd.DataFrame(data)
        if not use_pandas:
            return [self.names] + df.values.tolist() if header else df.values.tolist()
        return df

    def as_tensor(self, cols=None, dtype=torch.float32) -> torch.Tensor:
        names = cols or self.names
        return torch.stack([self._col(n).as_float() for n in names], 1).to(dtype)

    def get_frame_data(self):
        return self.as_data_frame().to_csv(index=False)

    def head(self, rows=10, cols=200):
        out = self[: min(rows, self.nrows), :][self.names[:cols]]
        return dframe.gather_frame(out)

    def tail(self, rows=10, cols=200):
        out = self[max(0, self.nrows - rows):, :][self.names[:cols]]
        return dframe.gather_frame(out)

    def __repr__(self):
        if self._shard is not None:      # no collectives in repr (a rank may print alone)
            sh = self._shard
            return (f"<H2OFrame {self.frame_id} [{sh.n_global} rows x {self.ncols} columns], row-sharded: this rank "
                    f"holds rows [{sh.offset}, {sh.offset + sh.n_local})>")
        try:
            return repr(self.head().as_data_frame()) + f"\n\n[{self.nrows} rows x {self.ncols} columns]"
        except Exception:  # noqa: BLE001
            return f"<H2OFrame {self.frame_id} {self.shape}>"

    def show(self, *a, **k):
        print(repr(self))

    # ---- type conversion
    def asfactor(self):
        cols = []
        sharded = self._shard is not None
        for c in self._cols.values():
            if c.type == "enum":
                cols.append(c)
            elif c.type == "string":
                e = _enum_from_values(c.name, c.strings, engine_device())
                if sharded:                      # ParseDataset-style domain unification over the ranks
                    e.data, e.domain = dframe.unify_domain(e.data, e.domain, _level_key)
                cols.append(e)
            else:
                cols.append(_num_to_enum(c, sharded))
        with dframe.shard_ctx(self._shard):
            return H2OFrame._from_columns(cols)

    def asnumeric(self):
        cols = []
        for c in self._cols.values():
            if c.type == "enum":
                # H2O: numeric-looking levels become their numbers, else the codes
                try:
                    lv = torch.tensor([float(x) for x in c.domain], dtype=torch.float64, device=c.data.device)
                    v = torch.where(c.data < 0, torch.full(c.data.shape, float("nan"), dtype=torch.float64, device=c.data.device), lv[c.data.clamp(min=0).long()])
                except ValueError:
                    v = c.as_float()
                cols.append(Column(c.name, "real", v))
            else:
                cols.append(Column(c.name, "real" if c.type != "int" else "int", c.as_float()))
        return H2OFrame._from_columns(cols)

    def ascharacter(self):
        return H2OFrame._from_columns([Column(c.name, "string", strings=np.array(
            [None if v is None or (isinstance(v, float) and math.isnan(v)) else _level_str(v) for v in c.to_numpy()], dtype=object))
            for c in self._cols.values()])

    def isfactor(self):
        return [c.type == "enum" for c in self._cols.values()]

    def isnumeric(self):
        return [c.type in ("real", "int") for c in self._cols.values()]

    def isstring(self):
        return [c.type == "string" for c in self._cols.values()]

    def levels(self):
        return [list(c.domain) if c.type == "enum" else [] for c in self._cols.values()]

    def nlevels(self):
        return [len(c.domain) if c.type == "enum" else 0 for c in self._cols.values()]

    def set_levels(self, levels):
        c = self._col(0)
        assert c.type == "enum" and len(levels) == len(c.domain)
        c.domain = list(levels)
        return self

    def relevel(self, y):
        c = self._col(0)
        k = c.domain.index(y)
        order = [k] + [i for i in range(len(c.domain)) if i != k]
        remap = torch.empty(len(order), dtype=torch.int32, device=c.data.device)
        remap[torch.tensor(order, device=c.data.device)] = torch.arange(len(order), dtype=torch.int32, device=c.data.device)
        codes = torch.where(c.data < 0, c.data, remap[c.data.clamp(min=0).long()])
        return H2OFrame._from_columns([Column(c.name, "enum", codes, [c.domain[i] for i in order])])

    # ---- stats (RollupStats)
    def _num(self, col=0):
        return self._col(col).as_float()

    def _moments(self):
        """Per-column global moments (one all-gather of per-rank partials when sharded)."""
        return [dframe.moments(c.as_float(), self._shard is not None) for c in self._cols.values()]

    def _reduce(self, fn, na_rm=True, return_frame=False):
        if self._shard is not None:
            kind = {torch.sum: "sum", torch.mean: "mean", torch.max: "max", torch.min: "min"}.get(fn)
            if kind is None:
                return dframe.gather_frame(self)._reduce(fn, na_rm, return_frame)
            out = []
            for m in self._moments():
                if not na_rm and m["nas"] > 0:
                    out.append(float("nan"))
                elif m["n"] == 0:
                    out.append(float("nan") if kind != "sum" else 0.0)
                else:
                    out.append(float(m[kind]))
            return out if (len(out) > 1 or return_frame) else out[0]
        out = []
        for c in self._cols.values():
            v = c.as_float()
            if na_rm:
                v = v[~torch.isnan(v)]
            out.append(float(fn(v)) if v.numel() else float("nan"))
        return out if (len(out) > 1 or return_frame) else out[0]

    def mean(self, skipna=True, axis=0, return_frame=False):
        if axis == 1:
            X = torch.stack([c.as_float() for c in self._cols.values()], 1)
            return H2OFrame.from_tensor(torch.nanmean(X, 1) if skipna else X.mean(1), ["mean"])
        r = self._reduce(torch.mean, skipna, True)
        return H2OFrame._from_columns([Column(n, "real", torch.tensor([v], dtype=torch.float64, device=engine_device()))
                                       for n, v in zip(self.names, r)]) if return_frame else (r if len(r) > 1 else r)

    def sum(self, skipna=True, axis=0, return_frame=False):
        r = self._reduce(torch.sum, skipna, True)
        return r if len(r) > 1 else r[0]

    def max(self):
        return self._reduce(torch.max)

    def min(self):
        return self._reduce(torch.min)

    def sd(self, na_rm=True):
        if self._shard is not None:
            return [math.sqrt(m["m2"] / (m["n"] - 1)) if m["n"] > 1 else float("nan") for m in self._moments()]
        return self._reduce(lambda v: torch.std(v, unbiased=True), na_rm, True)

    std = sd

    def var(self, y=None, na_rm=True, use=None):
        if self._shard is not None and y is None and self.ncols == 1:
            m = self._moments()[0]
            return m["m2"] / (m["n"] - 1) if m["n"] > 1 else float("nan")
        if self._shard is not None or (y is not None and y._shard is not None):
            return dframe.gather_frame(self).var(dframe.gather_frame(y), na_rm, use)
        if y is None and self.ncols == 1:
            return self._reduce(lambda v: torch.var(v, unbiased=True))
        X = self.as_tensor(dtype=torch.float64)
        Y = X if y is None else y.as_tensor(dtype=torch.float64)
        Xc, Yc = X - X.mean(0), Y - Y.mean(0)
        return H2OFrame.from_tensor(Xc.T @ Yc / (X.shape[0] - 1), names=(y or self).names)

    def median(self, na_rm=True):
        return self._reduce(lambda v: torch.quantile(v, 0.5))

    def nacnt(self):
        cnt = [int(c.isna().sum()) for c in self._cols.values()]
        if self._shard is not None:
            cnt = [int(x) for x in coll_all_reduce_np(cnt)]
        return cnt

    def isna(self):
        return H2OFrame._from_columns([Column(f"isNA({c.name})", "int", c.isna().double()) for c in self._cols.values()])

    def any(self):
        r = bool(torch.nan_to_num(self._num(), nan=0).ne(0).any())
        return bool(coll_all_reduce_np([r])[0] > 0) if self._shard is not None else r

    def all(self):
        r = bool(torch.nan_to_num(self._num(), nan=1).ne(0).all())
        return bool(coll_all_reduce_np([not r])[0] == 0) if self._shard is not None else r

    def quantile(self, prob=None, combine_method="interpolate", weights_column=None):
        """Column quantiles (``hex/quantile/Quantile.java``): combine_method interpolate | average | low |
        high, optional observation weights; computed on device by one sort per column."""
        from .models.quantile import weighted_quantiles
        prob = prob or [0.001, 0.01, 0.1, 0.25, 0.333, 0.5, 0.667, 0.75, 0.9, 0.99, 0.999]
        wcol = None
        if weights_column is not None:
            wcol = (weights_column if isinstance(weights_column, H2OFrame) else self[weights_column])._col(0).as_float()
        cols = [Column("Probs", "real", torch.tensor(prob, dtype=torch.float64, device=engine_device()))]
        for c in self._cols.values():
            if c.type not in _NUMERIC or (isinstance(weights_column, str) and c.name == weights_column):
                continue
            q = weighted_quantiles(c.data, prob, combine_method, wcol)
            cols.append(Column(c.name + "Quantiles", "real", q.to(engine_device())))
        return H2OFrame._from_columns(cols)

    def summary(self, return_data=False):
        out = {}
        sharded = self._shard is not None
        for n, c in self._cols.items():
            d = dict(type=c.type, missing=int(c.isna().sum()))
            if sharded:
                d["missing"] = int(coll_all_reduce_np([d["missing"]])[0])
            if c.type in _NUMERIC:
                m = dframe.moments(c.data, sharded)
                if m["n"]:
                    d.update(mean=m["mean"], sd=math.sqrt(m["m2"] / (m["n"] - 1)) if m["n"] > 1 else 0.0, min=m["min"],
                             max=m["max"], zeros=int(m["zeros"]))
            elif c.type == "enum":
                d.update(cardinality=len(c.domain))
            out[n] = d
        if return_data:
            return out
        import pandas as pd
        print(pd.DataFrame(out))
        return None

    describe = summary

    def table(self, data2=None, dense=True):
        c = self._col(0)
        if data2 is None:
            if c.type == "enum":
                cnt = torch.bincount(c.data[c.data >= 0].long(), minlength=len(c.domain))
                return H2OFrame({c.name: list(c.domain), "Count": cnt.cpu().numpy()})
            v, cnt = torch.unique(c.data[~torch.isnan(c.data)], return_counts=True)
            return H2OFrame({c.name: v.cpu().numpy(), "Count": cnt.cpu().numpy()})
        a, b = c.to_numpy(), data2._col(0).to_numpy()
        import pandas as pd
        df = pd.DataFrame({c.name: a, data2.names[0]: b}).groupby([c.name, data2.names[0]]).size().reset_index(name="Counts")
        return H2OFrame(df)

    def unique(self, include_nas=False):
        c = self._col(0)
        if c.type == "enum":
            codes = torch.unique(c.data[c.data >= 0])
            return H2OFrame._from_columns([Column("C1", "enum", codes.to(torch.int32), list(c.domain))])
        v = torch.unique(c.data[~torch.isnan(c.data)])
        return H2OFrame._from_columns([Column("C1", c.type, v)])

    def hist(self, breaks="sturges", plot=False):
        v = self._num()
        v = v[~torch.isnan(v)]
        nb = int(math.ceil(math.log2(max(v.numel(), 2)) + 1)) if breaks == "sturges" else int(breaks)
        h = torch.histc(v.float(), bins=nb, min=float(v.min()), max=float(v.max()))
        edges = torch.linspace(float(v.min()), float(v.max()), nb + 1, dtype=torch.float64)
        return H2OFrame({"breaks": edges[1:].numpy(), "counts": h.cpu().numpy().astype(np.float64)})

    def cor(self, y=None, na_rm=False, use=None, method="Pearson"):
        X = self.as_tensor(dtype=torch.float64)
        Y = X if y is None else y.as_tensor(dtype=torch.float64)
        if method.lower() == "spearman":
            X = X.argsort(0).argsort(0).double(); Y = Y.argsort(0).argsort(0).double()
        Xc, Yc = X - X.mean(0), Y - Y.mean(0)
        c = (Xc.T @ Yc) / torch.outer(Xc.norm(dim=0), Yc.norm(dim=0))
        if c.numel() == 1:
            return float(c)
        return H2OFrame.from_tensor(c, names=(y or self).names)

    # ---- elementwise ops
    def _binop(self, other, fn, name=None, logical=False):
        cols = []
        if isinstance(other, H2OFrame):
            oc = list(other._cols.values())
            for i, c in enumerate(self._cols.values()):
                o = oc[i if len(oc) > 1 else 0]
                a, b = _op_operand(c, o), _op_operand(o, c)
                cols.append(Column(c.name, "real", fn(a, b).double()))
        else:
            for c in self._cols.values():
                if c.type == "enum" and isinstance(other, str):
                    code = c.domain.index(other) if other in c.domain else -2
                    a = c.data.double()
                    r = fn(a, torch.full_like(a, float(code)))
                    r = torch.where(c.data < 0, torch.full_like(r.double(), float("nan")), r.double())
                    cols.append(Column(c.name, "real", r))
                elif isinstance(other, str) and (c.type == "string" or bool(torch.isnan(c.as_float()).all())):
                    # string compare (AstBinOp string ops: a missing string equals ""); ranks in the sorted
                    # union keep <, > lexicographic
                    vals = ["" if v is None or (isinstance(v, float) and math.isnan(v)) else str(v)
                            for v in (c.strings if c.type == "string" else [None] * self._nlocal)]
                    lut = {s: i for i, s in enumerate(sorted(set(vals) | {other}))}
                    a = torch.tensor([float(lut[v]) for v in vals], dtype=torch.float64, device=engine_device())
                    cols.append(Column(c.name, "real", fn(a, torch.full_like(a, float(lut[other]))).double()))
                else:
                    cols.append(Column(c.name, "real", fn(c.as_float(), torch.as_tensor(float(other), dtype=torch.float64)).double()))
        for c in cols:
            if logical:
                c.type = "int"
        return H2OFrame._from_columns(cols)

    def __add__(self, o): return self._binop(o, torch.add)
    def __radd__(self, o): return self._binop(o, lambda a, b: b + a)
    def __sub__(self, o): return self._binop(o, torch.sub)
    def __rsub__(self, o): return self._binop(o, lambda a, b: b - a)
    def __mul__(self, o): return self._binop(o, torch.mul)
    def __rmul__(self, o): return self._binop(o, lambda a, b: b * a)
    def __truediv__(self, o): return self._binop(o, torch.div)
    def __rtruediv__(self, o): return self._binop(o, lambda a, b: b / a)
    def __floordiv__(self, o): return self._binop(o, lambda a, b: torch.floor(a / b))
    def __mod__(self, o): return self._binop(o, torch.remainder)
    def __pow__(self, o): return self._binop(o, torch.pow)
    def __rpow__(self, o): return self._binop(o, lambda a, b: torch.pow(b, a))
    def _cmp(self, o, fn):
        def f(a, b):
            r = fn(a, b).double()
            return torch.where(torch.isnan(a) | torch.isnan(b), torch.full_like(r, float("nan")), r)
        return self._binop(o, f, logical=True)
    def __eq__(self, o): return self._cmp(o, torch.eq)  # noqa: E301
    def __ne__(self, o): return self._cmp(o, torch.ne)
    def __lt__(self, o): return self._cmp(o, torch.lt)
    def __le__(self, o): return self._cmp(o, torch.le)
    def __gt__(self, o): return self._cmp(o, torch.gt)
    def __ge__(self, o): return self._cmp(o, torch.ge)
    def __and__(self, o): return self._binop(o, lambda a, b: ((a != 0) & (b != 0)).double(), logical=True)
    def __or__(self, o): return self._binop(o, lambda a, b: ((a != 0) | (b != 0)).double(), logical=True)
    def __invert__(self): return self._unop(lambda v: (v == 0).double())
    def __neg__(self): return self._unop(torch.neg)
    def __abs__(self): return self._unop(torch.abs)
    __hash__ = object.__hash__

    def _unop(self, fn, name=None):
        return H2OFrame._from_columns([Column(c.name, "real", fn(c.as_float()).double()) for c in self._cols.values()])

    def log(self): return self._unop(torch.log)
    def log10(self): return self._unop(torch.log10)
    def log2(self): return self._unop(torch.log2)
    def log1p(self): return self._unop(torch.log1p)
    def exp(self): return self._unop(torch.exp)
    def expm1(self): return self._unop(torch.expm1)
    def sqrt(self): return self._unop(torch.sqrt)
    def abs(self): return self._unop(torch.abs)
    def ceil(self): return self._unop(torch.ceil)
    def floor(self): return self._unop(torch.floor)
    def trunc(self): return self._unop(torch.trunc)
    def sign(self): return self._unop(torch.sign)
    def sin(self): return self._unop(torch.sin)
    def cos(self): return self._unop(torch.cos)
    def tan(self): return self._unop(torch.tan)
    def tanh(self): return self._unop(torch.tanh)
    def round(self, digits=0): return self._unop(lambda v: torch.round(v * 10 ** digits) / 10 ** digits)
    def signif(self, digits=6): return self._unop(lambda v: torch.where(v == 0, v, torch.round(v / 10 ** (torch.floor(torch.log10(v.abs())) - digits + 1)) * 10 ** (torch.floor(torch.log10(v.abs())) - digits + 1)))
    def cumsum(self, axis=0): return self._unop(lambda v: torch.cumsum(v, 0))
    def cumprod(self, axis=0): return self._unop(lambda v: torch.cumprod(v, 0))
    def cummax(self, axis=0): return self._unop(lambda v: torch.cummax(v, 0).values)
    def cummin(self, axis=0): return self._unop(lambda v: torch.cummin(v, 0).values)

    def ifelse(self, yes, no):
        cond = torch.nan_to_num(self._num(), nan=0) != 0
        dev = cond.device
        def val(x):
            if isinstance(x, H2OFrame):
                return x._num()
            return torch.full(cond.shape, float(x), dtype=torch.float64, device=dev)
        return H2OFrame._from_columns([Column("C1", "real", torch.where(cond, val(yes), val(no)))])

    def which(self):
        idx = torch.nonzero(torch.nan_to_num(self._num(), nan=0) != 0).reshape(-1)
        return H2OFrame._from_columns([Column("which", "int", idx.double())])

    def fillna(self, method="forward", axis=0, maxlen=1):
        cols = []
        for c in self._cols.values():
            if c.type not in _NUMERIC:
                cols.append(c)
                continue
            v = c.data.cpu().numpy().copy()
            import pandas as pd
            s = pd.Series(v)
            s = s.ffill(limit=maxlen) if method == "forward" else s.bfill(limit=maxlen)
            cols.append(Column(c.name, c.type, torch.as_tensor(s.values, device=engine_device())))
        return H2OFrame._from_columns(cols)

    def impute(self, column=-1, method="mean", combine_method="interpolate", by=None, group_by_frame=None, values=None):
        targets = self.names if column in (-1, None) else self._resolve(column)
        if by not in (None, [], ()):
            return self._impute_by(targets, method, by)
        res = []
        if self._shard is not None:
            # global statistics (collectives), applied to each shard in place
            for n in targets:
                c = self._cols[n]
                if c.type == "enum":
                    cnt = torch.bincount(c.data[c.data >= 0].long(), minlength=len(c.domain)).double().cpu().numpy()
                    mode = int(np.argmax(coll_all_reduce_np(cnt)))
                    c.data = torch.where(c.data < 0, torch.full_like(c.data, mode), c.data)
                    res.append(mode)
                elif c.type in _NUMERIC:
                    if method == "mean":
                        fill = dframe.moments(c.data, True)["mean"]
                    else:
                        g = dframe.gather_tensor(c.data)
                        gv = g[~torch.isnan(g)]
                        fill = float(torch.quantile(gv, 0.5)) if method != "mode" else float(torch.mode(gv).values)
                    c.data = torch.nan_to_num(c.data, nan=fill)
                    res.append(fill)
            return res
        for n in targets:
            c = self._cols[n]
            if c.type == "enum":
                cnt = torch.bincount(c.data[c.data >= 0].long(), minlength=len(c.domain))
                mode = int(cnt.argmax())
                c.data = torch.where(c.data < 0, torch.full_like(c.data, mode), c.data)
                res.append(mode)
            elif c.type in _NUMERIC:
                v = c.data[~torch.isnan(c.data)]
                fill = float(v.mean() if method == "mean" else torch.quantile(v, 0.5)) if method != "mode" else float(torch.mode(v).values)
                c.data = torch.nan_to_num(c.data, nan=fill)
                res.append(fill)
        return res

    def _impute_by(self, targets, method, by):
        """Group-wise imputation (AstImpute.java:205-257): each NA of a target column takes the aggregate of its
        group of the ``by`` columns — mean / median of a numeric column, mode of a categorical one, NAs removed
        ("rm"); a group whose aggregate is NA keeps its NAs. NA keys form a group of their own (AstGroup). Row
        sharded frames gather the key and target columns, aggregate once, and write their own rows back.
        Returns {target: {group key tuple: fill}}."""
        bys = self._resolve(by if isinstance(by, (list, tuple)) else [by])
        sharded = self._shard is not None
        if sharded:
            from .parallel import collectives as coll
            n_local = int(next(iter(self._cols.values())).data.shape[0])     # this rank's rows (nrows is global)
            row0 = coll.row_offset(n_local)

        def full(t):
            return dframe.gather_tensor(t) if sharded else t
        keys = torch.stack([full(self._cols[b].as_float()).double() for b in bys], 1)
        keys = torch.nan_to_num(keys, nan=float("inf"))          # NA keys: one group
        uk, inv = torch.unique(keys, dim=0, return_inverse=True)
        G = uk.shape[0]
        out = {}
        for n in targets:
            if n in bys:
                raise ValueError(f"column {n} is both imputed and a group-by column")
            c = self._cols[n]
            if c.type not in _NUMERIC and c.type != "enum":
                continue
            v = full(c.data.double() if c.type != "enum" else torch.where(c.data < 0, torch.nan, c.data.double()))
            ok = ~torch.isnan(v)
            if c.type == "enum" or method == "mode":
                fill = torch.full((G,), float("nan"), dtype=torch.float64, device=v.device)
                for gi in range(G):
                    vv = v[ok & (inv == gi)]
                    if vv.numel():
                        fill[gi] = float(torch.mode(vv).values)
            elif method == "median":
                fill = torch.full((G,), float("nan"), dtype=torch.float64, device=v.device)
                for gi in range(G):
                    vv = v[ok & (inv == gi)]
                    if vv.numel():
                        fill[gi] = float(torch.quantile(vv, 0.5))
            else:
                s = torch.zeros(G, dtype=torch.float64, device=v.device).index_add_(0, inv[ok], v[ok])
                k = torch.zeros(G, dtype=torch.float64, device=v.device).index_add_(0, inv[ok], torch.ones_like(v[ok]))
                fill = s / k
            filled = torch.where(ok, v, fill[inv])
            if sharded:
                filled = filled[row0:row0 + n_local]
            if c.type == "enum":
                c.data = torch.where(torch.isnan(filled), -1, filled).to(c.data.dtype)
            else:
                c.data = filled.to(c.data.dtype)
            ukc = uk.cpu().tolist()
            out[n] = {tuple(None if math.isinf(x) else x for x in ukc[gi]): float(fill[gi]) for gi in range(G)}
        return out

    def scale(self, center=True, scale=True):
        cols = []
        if self._shard is not None:
            for c, m in zip(self._cols.values(), self._moments()):
                v = c.as_float()
                if center:
                    v = v - m["mean"]
                if scale:
                    v = v / math.sqrt(m["m2"] / (m["n"] - 1))
                cols.append(Column(c.name, "real", v))
            with dframe.shard_ctx(self._shard):
                return H2OFrame._from_columns(cols)
        for c in self._cols.values():
            v = c.as_float()
            if center:
                v = v - torch.nanmean(v)
            if scale:
                vv = v[~torch.isnan(v)]
                v = v / vv.std()
            cols.append(Column(c.name, "real", v))
        return H2OFrame._from_columns(cols)

    def cut(self, breaks, labels=None, include_lowest=False, right=True, dig_lab=3):
        v = self._num()
        b = torch.tensor(breaks, dtype=torch.float64, device=v.device)
        idx = torch.bucketize(v, b, right=not right) - 1
        if include_lowest:
            idx = torch.where(v == b[0], torch.zeros_like(idx), idx)
        nb = len(breaks) - 1
        bad = (idx < 0) | (idx >= nb) | torch.isnan(v)
        labels = labels or [f"({breaks[i]},{breaks[i + 1]}]" if right else f"[{breaks[i]},{breaks[i + 1]})" for i in range(nb)]
        return H2OFrame._from_columns([Column(self.names[0], "enum", torch.where(bad, torch.full_like(idx, -1), idx).to(torch.int32), list(labels))])

    # ---- string ops
    def _strs(self):
        c = self._col(0)
        return c.strings if c.type == "string" else c.to_numpy()

    def _str_map(self, fn, type_="string"):
        s = self._strs()
        out = np.array([None if v is None else fn(str(v)) for v in s], dtype=object)
        if type_ == "string":
            return H2OFrame._from_columns([Column(self.names[0], "string", strings=out)])
        return H2OFrame._from_columns([Column(self.names[0], "int", torch.as_tensor(np.array([np.nan if v is None else v for v in out], dtype=np.float64), device=engine_device()))])

    def tolower(self): return self._enum_or_str(str.lower)
    def toupper(self): return self._enum_or_str(str.upper)
    def trim(self): return self._enum_or_str(str.strip)
    def lstrip(self, set=" "): return self._enum_or_str(lambda s: s.lstrip(set))
    def rstrip(self, set=" "): return self._enum_or_str(lambda s: s.rstrip(set))
    def nchar(self): return self._str_map(len, "int")
    def gsub(self, pattern, replacement, ignore_case=False): return self._enum_or_str(lambda s: re.sub(pattern, replacement, s, flags=re.I if ignore_case else 0))
    def sub(self, pattern, replacement, ignore_case=False): return self._enum_or_str(lambda s: re.sub(pattern, replacement, s, count=1, flags=re.I if ignore_case else 0))
    def substring(self, start_index, end_index=None): return self._enum_or_str(lambda s: s[start_index:end_index])
    def grep(self, pattern, ignore_case=False, invert=False, output_logical=False):
        s = self._strs()
        rx = re.compile(pattern, re.I if ignore_case else 0)
        m = np.array([(v is not None and bool(rx.search(str(v)))) != invert for v in s])
        if output_logical:
            return H2OFrame._from_columns([Column("C1", "int", torch.as_tensor(m.astype(np.float64), device=engine_device()))])
        return H2OFrame._from_columns([Column("C1", "int", torch.as_tensor(np.nonzero(m)[0].astype(np.float64), device=engine_device()))])
    def countmatches(self, pattern): return self._str_map(lambda s: sum(s.count(p) for p in ([pattern] if isinstance(pattern, str) else pattern)), "int")
    def strsplit(self, pattern):
        s = self._strs()
        parts = [None if v is None else re.split(pattern, str(v)) for v in s]
        k = max((len(p) for p in parts if p), default=1)
        return H2OFrame._from_columns([Column(f"C{j + 1}", "string", strings=np.array([p[j] if p and j < len(p) else None for p in parts], dtype=object)).__class__ and
                                       _enum_from_values(f"C{j + 1}", np.array([p[j] if p and j < len(p) else None for p in parts], dtype=object), engine_device()) for j in range(k)])
    def entropy(self):
        def ent(s):
            if not s:
                return 0.0
            _, cnt = np.unique(list(s), return_counts=True)
            p = cnt / cnt.sum()
            return float(-(p * np.log2(p)).sum())
        return self._str_map(ent, "int")

    def _enum_or_str(self, fn):
        c = self._col(0)
        if c.type == "enum":
            return H2OFrame._from_columns([_enum_from_values(c.name, np.array([None if v is None else fn(v) for v in c.to_numpy()], dtype=object), engine_device())])
        return self._str_map(fn)

    # ---- time ops
    def _time(self, fn):
        ms = self._num()
        import pandas as pd
        t = pd.to_datetime(ms.cpu().numpy(), unit="ms")
        return H2OFrame._from_columns([Column(self.names[0], "int", torch.as_tensor(np.asarray(fn(t), dtype=np.float64), device=engine_device()))])

    def year(self): return self._time(lambda t: t.year)
    def month(self): return self._time(lambda t: t.month)
    def day(self): return self._time(lambda t: t.day)
    def hour(self): return self._time(lambda t: t.hour)
    def minute(self): return self._time(lambda t: t.minute)
    def second(self): return self._time(lambda t: t.second)
    def week(self): return self._time(lambda t: t.isocalendar().week.values)
    def dayOfWeek(self): return self._time(lambda t: t.dayofweek)

    def as_date(self, format):
        import pandas as pd
        s = pd.to_datetime(pd.Series(self._strs()), format=format.replace("%", "%") if "%" in format else None, errors="coerce")
        ms = s.values.astype("datetime64[ms]").astype(np.int64).astype(np.float64)
        ms[s.isna().values] = np.nan
        return H2OFrame._from_columns([Column(self.names[0], "time", torch.as_tensor(ms, device=engine_device()))])

    # ---- combining
    def cbind(self, data):
        others = data if isinstance(data, (list, tuple)) else [data]
        cols = list(self._cols.values())
        for o in others:
            if isinstance(o, (int, float)):
                cols.append(Column(f"C{len(cols) + 1}", "real", torch.full((self._nlocal,), float(o), dtype=torch.float64, device=engine_device())))
            else:
                cols += list(o._cols.values())
        return H2OFrame._from_columns([Column(c.name, c.type, c.data, c.domain, c.strings) for c in cols])

    def rbind(self, data):
        others = data if isinstance(data, (list, tuple)) else [data]
        cols = []
        for n, c in self._cols.items():
            parts = [c] + [o._col(n) for o in others]
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
                cols.append(Column(n, c.type, torch.cat([p.as_float() for p in parts])))
        return H2OFrame._from_columns(cols)

    def merge(self, other, all_x=False, all_y=False, by_x=None, by_y=None, method="auto"):
        left, right = self.as_data_frame(), other.as_data_frame()
        on_x = by_x or [n for n in self.names if n in other.names]
        on_y = by_y or on_x
        how = "outer" if all_x and all_y else ("left" if all_x else ("right" if all_y else "inner"))
        df = left.merge(right, left_on=on_x, right_on=on_y, how=how)
        return H2OFrame(df)

    def sort(self, by, ascending=True):
        by = self._resolve(by)
        asc = ascending if isinstance(ascending, (list, tuple)) else [ascending] * len(by)
        idx = torch.arange(self.nrows, device=engine_device())
        for n, a in reversed(list(zip(by, asc))):
            v = self._cols[n].as_float()[idx]
            key = torch.nan_to_num(v, nan=float("-inf"))
            o = torch.argsort(key, descending=not a, stable=True)
            idx = idx[o]
        return self._rows(idx)

    def group_by(self, by):
        from .frame_ops import GroupBy
        return GroupBy(self, by)

    def _row_uniform(self, seed):
        """Per-row uniforms keyed by the GLOBAL row index: the same draw for a row however the frame is
        sharded (a SPMD program gets the same split on 1 or N ranks)."""
        from .parallel import collectives as coll
        s = int(seed) if seed not in (None, -1) else int(coll.broadcast_object(np.random.randint(1 << 30)))
        off = self._shard.offset if self._shard is not None else 0
        return coll.row_uniform(s, 0x5EED, off, self._nlocal, engine_device())

    def split_frame(self, ratios=None, destination_frames=None, seed=None):
        ratios = ratios or [0.75]
        r = self._row_uniform(seed)
        cuts = np.cumsum([0.0] + list(ratios) + [1.0 - sum(ratios)])
        out = []
        for i in range(len(cuts) - 1):
            m = (r >= cuts[i]) & (r < cuts[i + 1]) if i < len(cuts) - 2 else (r >= cuts[i])
            fr = self._rows(m)
            if destination_frames and i < len(destination_frames):
                dkv.put(destination_frames[i], fr)
                fr.frame_id = destination_frames[i]
            out.append(fr)
        return out

    def runif(self, seed=None):
        with dframe.shard_ctx(self._shard):
            return H2OFrame._from_columns([Column("rnd", "real", self._row_uniform(seed))])

    def kfold_column(self, n_folds=3, seed=-1):
        u = self._row_uniform(seed)
        with dframe.shard_ctx(self._shard):
            return H2OFrame._from_columns([Column("fold", "int", torch.floor(u * n_folds).clamp(max=n_folds - 1))])

    def modulo_kfold_column(self, n_folds=3):
        off = self._shard.offset if self._shard is not None else 0
        with dframe.shard_ctx(self._shard):
            return H2OFrame._from_columns([Column("fold", "int", (torch.arange(off, off + self._nlocal, device=engine_device()) % n_folds).double())])

    def stratified_kfold_column(self, n_folds=3, seed=-1):
        c = self._col(0)
        g = np.random.default_rng(None if seed in (None, -1) else int(seed))
        y = c.to_numpy()
        fold = np.zeros(len(y))
        keys = np.array([str(v) for v in y])
        for k in np.unique(keys):
            idx = np.nonzero(keys == k)[0]
            g.shuffle(idx)
            fold[idx] = np.arange(len(idx)) % n_folds
        return H2OFrame._from_columns([Column("fold", "int", torch.as_tensor(fold, device=engine_device()))])

    def stratified_split(self, test_frac=0.2, seed=-1):
        f = self.stratified_kfold_column(int(round(1 / test_frac)), seed)
        v = f._num()
        lab = np.array(["train"] * self.nrows, dtype=object)
        lab[(v == 0).cpu().numpy()] = "test"
        return H2OFrame._from_columns([_enum_from_values("test_train_split", lab, engine_device())])

    def apply(self, fun, axis=0):
        X = self.as_tensor(dtype=torch.float64)
        if axis == 0:
            return H2OFrame.from_tensor(torch.stack([torch.as_tensor(fun(X[:, j])) for j in range(X.shape[1])]).reshape(1, -1).double(), self.names)
        return H2OFrame.from_tensor(torch.stack([torch.as_tensor(fun(X[i])) for i in range(X.shape[0])]).double())

    def transpose(self):
        return H2OFrame.from_tensor(self.as_tensor(dtype=torch.float64).T)

    def mult(self, matrix):
        return H2OFrame.from_tensor(self.as_tensor(dtype=torch.float64) @ matrix.as_tensor(dtype=torch.float64))

    def flatten(self):
        c = self._col(0)
        v = c.to_numpy()[0]
        return v

    def topN(self, column=0, nPercent=10, grabTopN=-1):
        v = self._col(column).as_float()
        k = max(1, int(round(v.numel() * nPercent / 100)))
        vals, idx = torch.topk(torch.nan_to_num(v, nan=float("-inf")), k, largest=grabTopN == -1)
        return H2OFrame._from_columns([Column("Row Indices", "int", idx.double()), Column(self.names[column] if isinstance(column, int) else column, "real", vals)])

    def drop_duplicates(self, columns, keep="first"):
        df = self.as_data_frame()
        return H2OFrame(df.drop_duplicates(subset=self._resolve(columns), keep=keep).reset_index(drop=True))

    def na_omit(self):
        m = torch.ones(self._nlocal, dtype=torch.bool, device=engine_device())
        for c in self._cols.values():
            m &= ~c.isna().to(m.device)
        return self._rows(m)

    def pivot(self, index, column, value):
        df = self.as_data_frame()
        return H2OFrame(df.pivot_table(index=index, columns=column, values=value, aggfunc="mean").reset_index())

    def melt(self, id_vars, value_vars=None, var_name="variable", value_name="value", skipna=False):
        df = self.as_data_frame().melt(id_vars=id_vars, value_vars=value_vars, var_name=var_name, value_name=value_name)
        if skipna:
            df = df.dropna(subset=[value_name])
        return H2OFrame(df)

    def difflag1(self):
        v = self._num()
        return H2OFrame._from_columns([Column(self.names[0], "real", torch.cat([torch.full((1,), float("nan"), dtype=torch.float64, device=v.device), v[1:] - v[:-1]]))])

    def interaction(self, factors, pairwise, max_factors, min_occurrence, destination_frame=None):
        from .frame_ops import interaction
        return interaction(self, factors, pairwise, max_factors, min_occurrence)

    def refresh(self):
        return self

    @property
    def key(self):
        return self.frame_id

    def __iter__(self):
        return iter(self.names)

    def __contains__(self, item):
        return item in self._cols

    # ---- model adaptation (Model.adaptTestForTrain)
    def model_matrix(self, info, device=None):
        device = device or engine_device()
        N = self._nlocal
        X = torch.empty(info.F, N, dtype=torch.float32, device=device)
        for j, n in enumerate(info.x):
            if n not in self._cols:
                X[j] = float("nan")
                continue
            c = self._cols[n]
            if info.domains[j] is not None:
                X[j] = _remap_codes(c, info.domains[j], device)
            else:
                X[j] = c.as_float().to(device=device, dtype=torch.float32)
        offset = None
        if info.offset and info.offset in self._cols:
            offset = self._cols[info.offset].as_float().to(device=device, dtype=torch.float32)
        return X, offset

    def response_tensor(self, info, device=None):
        device = device or engine_device()
        if info.response not in self._cols:
            return None
        c = self._cols[info.response]
        if info.response_domain is not None:
            return _remap_codes(c, info.response_domain, device)
        return c.as_float().to(device=device, dtype=torch.float32)

    def weights_tensor(self, info, device=None):
        if not info.weights or info.weights not in self._cols:
            return None
        return self._cols[info.weights].as_float().to(device=device or engine_device(), dtype=torch.float32)


def coll_all_reduce_np(a):
    from .parallel import collectives as coll
    if not coll.world_active():
        return np.asarray(a, dtype=np.float64)
    with_ = coll.all_gather_object(np.asarray(a, dtype=np.float64))
    return np.sum(with_, axis=0)


def _op_operand(c: Column, other: Column):
    if c.type == "enum" and other.type == "enum" and c.domain != other.domain:
        return c.data.double()
    return c.as_float()


def _num_to_enum(c: Column, sharded: bool = False) -> Column:
    v = c.data
    ok = ~torch.isnan(v)
    u = dframe.global_unique(v) if sharded else torch.unique(v[ok])
    dom = [_level_str(x) for x in u.cpu().numpy().tolist()]
    codes = torch.full(v.shape, -1, dtype=torch.int32, device=v.device)
    codes[ok] = torch.bucketize(v[ok], u).to(torch.int32)
    return Column(c.name, "enum", codes, dom)


def _remap_codes(c: Column, domain, device) -> torch.Tensor:
    """Column -> float codes in ``domain`` order (unseen levels / NA -> NaN)."""
    if c.type == "enum":
        if list(c.domain) == list(domain):
            codes = c.data.to(device)
            return torch.where(codes < 0, torch.full(codes.shape, float("nan"), device=device), codes.float())
        lut = {s: i for i, s in enumerate(domain)}
        m = torch.tensor([lut.get(s, -1) for s in c.domain] + [-1], dtype=torch.float32, device=device)
        codes = c.data.to(device).long()
        r = m[torch.where(codes < 0, torch.full_like(codes, len(c.domain)), codes)]
        return torch.where(r < 0, torch.full_like(r, float("nan")), r)
    # numeric response/feature used as categorical: map by string value
    lut = {s: i for i, s in enumerate(domain)}
    vals = c.to_numpy()
    out = np.array([lut.get(_level_str(v) if v is not None and not (isinstance(v, float) and math.isnan(v)) else None, np.nan)
                    for v in vals], dtype=np.float32)
    return torch.as_tensor(out, device=device)


# distribution class of every H2OFrame method (row-local / collective / gathered): parallel/dframe.py
from . import frame_more as _frame_more  # noqa: E402

_frame_more.install(H2OFrame)
dframe.LOCAL.update({"acos", "acosh", "asin", "asinh", "atan", "atanh", "cosh", "sinh", "cospi", "sinpi", "tanpi",
                     "gamma", "lgamma", "digamma", "trigamma", "logical_negation"})
dframe.install(H2OFrame)
