"""The rest of the h2o-py ``H2OFrame`` surface (reference ``h2o-py/h2o/frame.py``): trigonometric /
special functions, statistics (skewness, kurtosis, prod, idxmax), level manipulation
(set_level, append_levels, relevel_by_frequency), matching (match, isin), string tools (tokenize,
strdistance, num_valid_substrings), time constructors (mktime, moment), iSAX, ranking within groups,
top/bottom-N, distance matrices, and the object helpers (get_frame, from_python, save, structure,
summaries, detach, concat, DMatrix conversion). Every numeric method runs through the same Rapids
primitive the REST ``/99/Rapids`` endpoint uses, so local calls and wire calls agree."""
from __future__ import annotations

import math

import numpy as np
import torch


def _prim(name, *args):
    from .rapids import Session
    global _SESSION
    try:
        sess = _SESSION
    except NameError:
        sess = _SESSION = Session()
    return sess.prims[name](*args)


def _unary(name):
    def f(self):
        return _prim(name, self)
    f.__name__ = name
    f.__doc__ = f"Element-wise ``{name}`` (Rapids primitive ``{name}``)."
    return f


def install(cls):
    for nm in ("acos", "acosh", "asin", "asinh", "atan", "atanh", "cosh", "sinh", "cospi", "sinpi", "tanpi",
               "gamma", "lgamma", "digamma", "trigamma"):
        setattr(cls, nm, _unary(nm))

    def logical_negation(self):
        return ~self

    def skewness(self, na_rm=False):
        return _prim("skewness", self, int(bool(na_rm)))

    def kurtosis(self, na_rm=False):
        return _prim("kurtosis", self, int(bool(na_rm)))

    def prod(self, na_rm=False):
        return _prim("prod.na" if na_rm else "prod", self)

    def any_na_rm(self):
        """True if any value (NAs skipped) is non-zero."""
        X = self.as_tensor(dtype=torch.float64)
        return bool(torch.nan_to_num(X, nan=0.0).ne(0).any())

    def anyfactor(self):
        return any(self.type(n) == "enum" for n in self.names)

    def ischaracter(self):
        return [self.type(n) == "string" for n in self.names]

    def categories(self):
        if self.ncols != 1:
            raise ValueError("categories() needs a single-column frame")
        return list(self._col(self.names[0]).domain or [])

    def idxmax(self, skipna=True, axis=0):
        return _prim("which.max", self, int(bool(skipna)), int(axis))

    def idxmin(self, skipna=True, axis=0):
        return _prim("which.min", self, int(bool(skipna)), int(axis))

    def set_level(self, level):
        return _prim("setLevel", self, level)

    def append_levels(self, levels):
        return _prim("appendLevels", self, list(levels), 0)

    def relevel_by_frequency(self, weights_column=None, top_n=-1):
        """Reorder every categorical column's levels by (weighted) frequency, most frequent first
        (AstRelevelByFreq); ``top_n`` > 0 moves only the top levels to the front."""
        from .frame import Column, H2OFrame
        w = self._col(weights_column).as_float().double() if weights_column else None
        cols = []
        for n in self.names:
            c = self._col(n)
            if c.type != "enum" or n == weights_column:
                cols.append(c)
                continue
            L = len(c.domain)
            codes = c.data.long()
            ok = codes >= 0
            cnt = torch.zeros(L, dtype=torch.float64, device=codes.device).index_add_(
                0, codes[ok], (w[ok] if w is not None else torch.ones_like(codes[ok], dtype=torch.float64)))
            order = sorted(range(L), key=lambda i: (-float(cnt[i]), i))
            if top_n is not None and int(top_n) > 0:
                top = order[:int(top_n)]
                order = top + [i for i in range(L) if i not in top]
            new_of_old = torch.empty(L, dtype=torch.long, device=codes.device)
            new_of_old[torch.tensor(order, device=codes.device)] = torch.arange(L, device=codes.device)
            nc = torch.where(ok, new_of_old[codes.clamp(min=0)], codes)
            cols.append(Column(n, "enum", nc.to(c.data.dtype), [c.domain[i] for i in order]))
        return H2OFrame._from_columns(cols)

    def match(self, table, nomatch=0):
        return _prim("match", self, table if isinstance(table, list) else [table], nomatch)

    def isin(self, item):
        """Row-wise membership of each value in ``item`` (a value, list, or single-column frame)."""
        from .frame import H2OFrame
        if isinstance(item, H2OFrame):
            item = [v for v in item._col(item.names[0]).to_numpy().tolist()]
        items = item if isinstance(item, (list, tuple, set)) else [item]
        outs = [(_prim("match", self[n], list(items), 0) > 0) for n in self.names]
        out = outs[0]
        for o in outs[1:]:
            out = out | o
        return out

    def distance(self, y, measure=None):
        return _prim("distance", self, y, measure or "l2")

    def strdistance(self, y, measure=None, compare_empty=True):
        return _prim("strDistance", self, y, measure or "lv", int(bool(compare_empty)))

    def tokenize(self, split):
        return _prim("tokenize", self, split)

    def num_valid_substrings(self, path_to_words):
        return _prim("num_valid_substrings", self, path_to_words)

    def isax(self, num_words, max_cardinality, optimize_card=False):
        return _prim("isax", self, num_words, max_cardinality, int(bool(optimize_card)))

    def rank_within_group_by(self, group_by_cols, sort_cols, ascending=[], new_col_name="New_Rank_column",
                             sort_cols_sorted=False):
        idx = lambda cs: [self.names.index(c) if isinstance(c, str) else int(c)  # noqa: E731
                          for c in (cs if isinstance(cs, (list, tuple)) else [cs])]
        s = idx(sort_cols)
        asc = [1 if a else 0 for a in ascending] if ascending else [1] * len(s)
        return _prim("rank_within_groupby", self, idx(group_by_cols), s, asc, new_col_name, int(bool(sort_cols_sorted)))

    def topNBottomN(self, column=0, nPercent=10, grabTopN=-1):
        col = self.names.index(column) if isinstance(column, str) else int(column)
        return _prim("topn", self, col, nPercent, grabTopN)

    def bottomN(self, column=0, nPercent=10):
        return topNBottomN(self, column, nPercent, -1)

    def rep_len(self, length_out):
        return _prim("rep_len", self, length_out)

    def filter_na_cols(self, frac=0.2):
        return _prim("filterNACols", self, frac)

    def getrow(self):
        if self.nrows != 1:
            raise ValueError("getrow() is only for single-row frames")
        return [v for v in self.as_data_frame().iloc[0].tolist()]

    def insert_missing_values(self, fraction=0.1, seed=None):
        """In place, like h2o-py (MissingInserter)."""
        from .frame_ops import insert_missing_values as imv
        out = imv(self, fraction, seed)
        for n in out.names:
            self._cols[n] = out._col(n)
        return self

    def concat(self, frames, axis=1):
        fs = [self] + list(frames if isinstance(frames, (list, tuple)) else [frames])
        out = fs[0]
        for f in fs[1:]:
            out = out.cbind(f) if axis == 1 else out.rbind(f)
        return out

    def structure(self):
        lines = [f"H2OFrame '{self.frame_id}':\t {self.nrows} obs. of {self.ncols} variables(s)"]
        for n in self.names:
            c = self._col(n)
            if c.type == "enum":
                lines.append(f"$ {n}: Factor w/ {len(c.domain)} level(s) " + ",".join(f'"{d}"' for d in c.domain[:10]))
            else:
                vals = self[n].head(10).as_data_frame()[n].tolist()
                lines.append(f"$ {n}: {c.type} " + " ".join(str(v) for v in vals))
        print("\n".join(lines))

    def get_summary(self):
        return self.summary(return_data=True) if "return_data" in self.summary.__code__.co_varnames else self.summary()

    def show_summary(self):
        print(self.summary())

    def detach(self):
        """Drop the local handle's link to its key (the data stays in the store)."""
        self._detached = True

    def save(self, path, force=True):
        from .io.parse import save_frame
        return save_frame(self, path, force)

    def save_to_hive(self, jdbc_url, table_name, format="csv", table_path=None, tmp_path=None):
        raise NotImplementedError("Hive is not available in this single-node MI355X engine; use export_file")

    def convert_H2OFrame_2_DMatrix(self, predictors, yresp, h2oXGBoostModel, return_pandas=False):
        """Design matrix of an XGBoost model's encoding (one-hot categoricals with an NA slot, then
        numerics) as a pandas frame (``return_pandas``) or a SciPy CSR matrix plus the response."""
        import pandas as pd
        import scipy.sparse as sp
        m = getattr(h2oXGBoostModel, "_model", h2oXGBoostModel)
        X, _ = self.model_matrix(m.info)
        cols, names = [], []
        for j, n in enumerate(m.info.x):
            v = X[j].double().cpu().numpy()
            if m.info.iscat[j]:
                dom = m.info.domains[j]
                for i, lv in enumerate(dom):
                    cols.append((v == i).astype(np.float64))
                    names.append(f"{n}.{lv}")
                cols.append(np.isnan(v).astype(np.float64))
                names.append(f"{n}.missing(NA)")
            else:
                cols.append(v)
                names.append(n)
        D = np.stack(cols, 1) if cols else np.zeros((self.nrows, 0))
        y = self._col(yresp).as_float().double().cpu().numpy() if yresp in self.names else None
        if return_pandas:
            df = pd.DataFrame(D, columns=names)
            if y is not None:
                df[yresp] = y
            return df
        return sp.csr_matrix(np.nan_to_num(D)), y

    for f in (logical_negation, skewness, kurtosis, prod, any_na_rm, anyfactor, ischaracter, categories, idxmax,
              idxmin, set_level, append_levels, relevel_by_frequency, match, isin, distance, strdistance, tokenize,
              num_valid_substrings, isax, rank_within_group_by, topNBottomN, bottomN, rep_len, filter_na_cols,
              getrow, insert_missing_values, concat, structure, get_summary, show_summary, detach, save,
              save_to_hive, convert_H2OFrame_2_DMatrix):
        if not hasattr(cls, f.__name__) or f.__name__ in ("insert_missing_values",):
            setattr(cls, f.__name__, f)

    def mktime(year=1970, month=0, day=0, hour=0, minute=0, second=0, msec=0):
        return _prim("mktime", year, month, day, hour, minute, second, msec)

    def moment(year=None, month=None, day=None, hour=None, minute=None, second=None, msec=None, date=None, time=None):
        """A time column from parts (month 1-12, day 1-31), or from ``date``/``time`` python objects."""
        if date is not None:
            year, month, day = date.year, date.month, date.day
        if time is not None:
            hour, minute, second, msec = time.hour, time.minute, time.second, time.microsecond // 1000
        return _prim("moment", year if year is not None else 1970, month or 1, day or 1, hour or 0, minute or 0,
                     second or 0, msec or 0)

    def get_frame(frame_id, rows=10, rows_offset=0, cols=-1, full_cols=-1, cols_offset=0, light=False):
        from .core import dkv
        return dkv.get(frame_id)

    def from_python(python_obj, destination_frame=None, header=0, separator=",", column_names=None,
                    column_types=None, na_strings=None):
        return cls(python_obj, destination_frame=destination_frame, header=header, separator=separator,
                   column_names=column_names, column_types=column_types, na_strings=na_strings)

    for nm, f in (("mktime", mktime), ("moment", moment), ("get_frame", get_frame), ("from_python", from_python)):
        if not hasattr(cls, nm):
            setattr(cls, nm, staticmethod(f))

    if not hasattr(cls, "dtype"):
        cls.dtype = property(lambda self: {n: self.type(n) for n in self.names} if self.ncols != 1 else self.type(self.names[0]))
