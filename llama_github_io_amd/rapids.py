"""Rapids expression evaluator (reference: ``water/rapids/Rapids.java`` (parser), ``Env.java``,
``ast/prims/**`` — mungers, math, reducers, operators, search, string, time, assign).

The REST ``/99/Rapids`` endpoint and the Python facade share this evaluator. An expression is an
s-expression: ``(op arg ...)``; atoms are numbers, "strings", frame/model ids, lists ``[1 2 3]``
(also ``[0:5]`` spans), and the special words ``TRUE FALSE NA``. Every primitive maps to the
device-resident :class:`H2OFrame` implementation, so Rapids munging runs on the GPU tensors.
"""
from __future__ import annotations

import math
import re

import numpy as np
import torch

from .core import dkv
from .frame import Column, H2OFrame, engine_device

_TOKEN = re.compile(r'\s*(\(|\)|\[|\]|"(?:[^"\\]|\\.)*"|\'(?:[^\'\\]|\\.)*\'|[^\s()\[\]]+)')


def tokenize(s: str):
    pos, out = 0, []
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise SyntaxError(f"bad rapids near {s[pos:pos + 20]!r}")
        out.append(m.group(1))
        pos = m.end()
        while pos < len(s) and s[pos].isspace():
            pos += 1
    return out


def parse(tokens, i=0):
    t = tokens[i]
    if t == "(":
        lst = []
        i += 1
        while tokens[i] != ")":
            node, i = parse(tokens, i)
            lst.append(node)
        return ("call", lst), i + 1
    if t == "[":
        lst = []
        i += 1
        while tokens[i] != "]":
            node, i = parse(tokens, i)
            lst.append(node)
        return ("list", lst), i + 1
    if t[0] in "\"'":
        return ("str", bytes(t[1:-1], "utf-8").decode("unicode_escape")), i + 1
    if t in ("TRUE", "FALSE"):
        return ("num", 1.0 if t == "TRUE" else 0.0), i + 1
    if t == "NA":
        return ("num", float("nan")), i + 1
    m = re.fullmatch(r"(-?\d+):(\d+)", t)
    if m:
        a, n = int(m.group(1)), int(m.group(2))
        return ("span", (a, n)), i + 1
    try:
        return ("num", float(t)), i + 1
    except ValueError:
        return ("id", t), i + 1


def _frame(v):
    if isinstance(v, H2OFrame):
        return v
    if isinstance(v, (int, float)):
        return H2OFrame._from_columns([Column("C1", "real", torch.tensor([float(v)], dtype=torch.float64, device=engine_device()))])
    raise TypeError(f"expected a frame, got {type(v)}")


def _idx_list(v, n=None):
    if isinstance(v, (int, float)):
        return [int(v)]
    out = []
    for x in v:
        if isinstance(x, tuple):
            out += list(range(x[0], x[0] + x[1]))
        else:
            out.append(x if isinstance(x, str) else int(x))
    return out


def _binop(fn):
    def f(a, b):
        if isinstance(a, H2OFrame):
            return a._binop(b, fn)
        if isinstance(b, H2OFrame):
            return b._binop(a, lambda x, y: fn(y, x))
        return float(fn(torch.tensor(float(a)), torch.tensor(float(b))))
    return f


def _cmp(fn):
    def f(a, b):
        if isinstance(a, H2OFrame):
            return a._cmp(b, fn)
        if isinstance(b, H2OFrame):
            return b._cmp(a, lambda x, y: fn(y, x))
        return float(fn(torch.tensor(float(a)), torch.tensor(float(b))))
    return f


def _unary(name):
    def f(a):
        if isinstance(a, H2OFrame):
            return getattr(a, name)()
        return float(getattr(torch, name)(torch.tensor(float(a))))
    return f


def _reduce(name):
    def f(a, *rest):
        fr = _frame(a)
        if name == "sum":
            v = fr.sum()
        elif name == "mean":
            v = fr.mean()
        elif name == "min":
            v = fr.min()
        elif name == "max":
            v = fr.max()
        elif name == "sd":
            v = fr.sd()
        elif name == "var":
            v = fr.var()
        elif name == "median":
            v = fr.median()
        else:
            raise ValueError(name)
        if isinstance(v, (list, tuple)):
            return float(v[0]) if len(v) == 1 else [float(x) for x in v]
        return float(v)
    return f


def _rows(fr, sel):
    fr = _frame(fr)
    if isinstance(sel, H2OFrame):
        return fr[sel]
    idx = _idx_list(sel)
    neg = [i for i in idx if isinstance(i, int) and i < 0]
    if neg and len(neg) == len(idx):
        drop = {-i - 1 for i in neg}
        idx = [i for i in range(fr.nrows) if i not in drop]
    return fr._rows(torch.as_tensor(idx, dtype=torch.long, device=engine_device()))


def _cols(fr, sel):
    fr = _frame(fr)
    if isinstance(sel, (int, float, str)):
        sel = [sel]
    idx = _idx_list(sel)
    if idx and all(isinstance(i, int) and i < 0 for i in idx):
        drop = {-i - 1 for i in idx}
        idx = [i for i in range(fr.ncols) if i not in drop]
    return fr[idx if len(idx) != 1 else idx[0:1]]


class Session:
    """Rapids session: temp names live in the DKV like ``Env`` globals."""

    def __init__(self):
        self.prims = {
            "+": _binop(torch.add), "-": _binop(torch.sub), "*": _binop(torch.mul), "/": _binop(torch.div),
            "^": _binop(torch.pow), "%": _binop(torch.remainder), "%%": _binop(torch.remainder),
            "intDiv": _binop(lambda a, b: torch.floor(a / b)),
            "==": _cmp(torch.eq), "!=": _cmp(torch.ne), "<": _cmp(torch.lt), "<=": _cmp(torch.le),
            ">": _cmp(torch.gt), ">=": _cmp(torch.ge),
            "&": lambda a, b: _frame(a) & b, "|": lambda a, b: _frame(a) | b, "&&": lambda a, b: _frame(a) & b,
            "||": lambda a, b: _frame(a) | b, "!": lambda a: ~_frame(a), "not": lambda a: ~_frame(a),
            **{n: _unary(n) for n in ("log", "exp", "sqrt", "abs", "ceiling", "floor", "trunc", "sign", "sin", "cos",
                                      "tan", "tanh", "log10", "log2", "log1p", "expm1")},
            "ceiling": lambda a: _frame(a).ceil(),
            **{n: _reduce(n) for n in ("sum", "mean", "min", "max", "sd", "var", "median")},
            "sumNA": _reduce("sum"), "maxNA": _reduce("max"), "minNA": _reduce("min"),
            "nrow": lambda a: float(_frame(a).nrows), "ncol": lambda a: float(_frame(a).ncols),
            "dim": lambda a: [float(_frame(a).nrows), float(_frame(a).ncols)],
            "rows": _rows, "cols": _cols, "cols_py": _cols,
            "cbind": lambda *fs: _frame(fs[0]).cbind([_frame(f) for f in fs[1:]]) if len(fs) > 1 else _frame(fs[0]),
            "rbind": lambda *fs: _frame(fs[0]).rbind([_frame(f) for f in fs[1:]]) if len(fs) > 1 else _frame(fs[0]),
            "as.factor": lambda a: _frame(a).asfactor(), "as.numeric": lambda a: _frame(a).asnumeric(),
            "as.character": lambda a: _frame(a).ascharacter(), "is.na": lambda a: _frame(a).isna(),
            "is.factor": lambda a: [float(x) for x in np.atleast_1d(_frame(a).isfactor())],
            "ifelse": lambda t, y, n: _frame(t).ifelse(y, n), "unique": lambda a, *r: _frame(a).unique(),
            "table": lambda a, *r: _frame(a).table(), "levels": lambda a: _frame(a).levels(),
            "nlevels": lambda a: _frame(a).nlevels(), "h2o.runif": lambda a, seed=-1: _frame(a).runif(int(seed)),
            "sort": lambda fr, by, asc=None: _frame(fr).sort(_idx_list(by), [bool(x) for x in asc] if isinstance(asc, list) else True),
            "quantile": lambda fr, probs, *r: _frame(fr).quantile(list(probs) if isinstance(probs, list) else [probs]),
            "scale": lambda fr, c=1, s=1: _frame(fr).scale(bool(c), bool(s)),
            "cumsum": lambda a, *r: _frame(a).cumsum(), "cumprod": lambda a, *r: _frame(a).cumprod(),
            "cummax": lambda a, *r: _frame(a).cummax(), "cummin": lambda a, *r: _frame(a).cummin(),
            "tolower": lambda a: _frame(a).tolower(), "toupper": lambda a: _frame(a).toupper(),
            "trim": lambda a: _frame(a).trim(), "strlen": lambda a: _frame(a).nchar(),
            "gsub": lambda pat, rep, a, ic=0: _frame(a).gsub(pat, rep, bool(ic)),
            "sub": lambda pat, rep, a, ic=0: _frame(a).sub(pat, rep, bool(ic)),
            "year": lambda a: _frame(a).year(), "month": lambda a: _frame(a).month(), "day": lambda a: _frame(a).day(),
            "hour": lambda a: _frame(a).hour(), "dayOfWeek": lambda a: _frame(a).dayOfWeek(),
            "na.omit": lambda a: _frame(a).na_omit(), "colnames=": self._colnames,
            "columnsByType": lambda fr, t: [float(i) for i in _col_idx_by_type(_frame(fr), t)],
            "merge": lambda l, r, ax, ay, bx, by, m="auto": _frame(l).merge(_frame(r), bool(ax), bool(ay),
                                                                              [_frame(l).names[int(i)] for i in bx] or None,
                                                                              [_frame(r).names[int(i)] for i in by] or None),
            "GB": self._groupby, "tmp=": self._assign, "assign": self._assign, "rm": self._rm,
            "cor": lambda a, b=None, *r: _frame(a).cor(None if b is None or isinstance(b, str) else _frame(b)),
            "transpose": lambda a: _frame(a).transpose(), "x": lambda a, b: _frame(a).mult(_frame(b)),
            "which": lambda a: _frame(a).which(), "h2o.impute": self._impute,
            "append": lambda fr, v, name: _frame(fr).cbind(_frame(v).set_names([name]) if isinstance(v, H2OFrame) else v),
            "comma": lambda *a: a[-1], ",": lambda *a: a[-1],
        }

    # ---- special forms
    def _assign(self, name, value):
        if isinstance(value, H2OFrame):
            dkv.put(name, value)
            value.frame_id = name
        return value

    def _rm(self, name):
        dkv.remove(name if isinstance(name, str) else name.frame_id)
        return 0.0

    def _colnames(self, fr, idx, names):
        fr = _frame(fr)
        idx = _idx_list(idx)
        names = names if isinstance(names, list) else [names]
        new = list(fr.names)
        for i, n in zip(idx, names):
            new[int(i)] = n
        fr.set_names(new)
        return fr

    def _groupby(self, fr, by, *aggs):
        from .frame_ops import GroupBy
        fr = _frame(fr)
        g = GroupBy(fr, [fr.names[int(i)] for i in _idx_list(by)])
        ops = {"nrow": "count", "mean": "mean", "sum": "sum", "min": "min", "max": "max", "sdev": "sd", "sd": "sd",
               "var": "var", "median": "median", "mode": "mode", "sumSquares": "ss"}
        for k in range(0, len(aggs), 3):
            op, col, na = aggs[k], aggs[k + 1], aggs[k + 2]
            fn = ops[op]
            if fn == "count":
                g.count(na)
            else:
                getattr(g, fn)(fr.names[int(col)], na)
        return g.get_frame()

    def _impute(self, fr, col, method, combine, by, *rest):
        fr = _frame(fr)
        fr.impute(int(col), method)
        return [0.0]

    # ---- evaluation
    def eval_node(self, node):
        kind, v = node
        if kind == "num":
            return v
        if kind == "str":
            return v
        if kind == "span":
            return [v]
        if kind == "list":
            out = []
            for x in v:
                r = self.eval_node(x)
                out += r if isinstance(r, list) and x[0] == "span" else [r]
            return out
        if kind == "id":
            val = dkv.get(v)
            return val if val is not None else v
        op = v[0]
        if op[0] != "id":
            raise SyntaxError("call head must be an operator")
        name = op[1]
        if name in ("tmp=", "assign"):
            return self._assign(v[1][1], self.eval_node(v[2]))
        fn = self.prims.get(name)
        if fn is None:
            raise NotImplementedError(f"rapids primitive {name!r}")
        return fn(*[self.eval_node(a) for a in v[1:]])

    def exec(self, expr: str):
        toks = tokenize(expr)
        node, _ = parse(toks, 0)
        return self.eval_node(node)


def _col_idx_by_type(fr, t):
    t = t.lower()
    out = []
    for i, n in enumerate(fr.names):
        ty = fr.type(n)
        if (t == "numeric" and ty in ("real", "int")) or (t == "categorical" and ty == "enum") or \
                (t == "string" and ty == "string") or (t == "time" and ty == "time") or t == "all":
            out.append(i)
    return out


_session = Session()


def rapids(expr: str):
    return _session.exec(expr)
