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

# commas separate list items like blanks do (h2o-py renders string lists with %r: ['a', 'b'])
_TOKEN = re.compile(r'[\s,]*(\(|\)|\[|\]|\{|\}|"(?:[^"\\]|\\.)*"|\'(?:[^\'\\]|\\.)*\'|[^\s,()\[\]{}]+)')


def tokenize(s: str):
    pos, out = 0, []
    s = s.strip()
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise SyntaxError(f"bad rapids near {s[pos:pos + 20]!r}")
        out.append(m.group(1))
        pos = m.end()
        while pos < len(s) and (s[pos].isspace() or s[pos] == ","):
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
    if t == "{":                       # lambda: { arg1 arg2 . body }
        params = []
        i += 1
        while tokens[i] != ".":
            params.append(tokens[i])
            i += 1
        body, i = parse(tokens, i + 1)
        if tokens[i] != "}":
            raise SyntaxError("lambda body must be one expression followed by '}'")
        return ("fun", (params, body)), i + 1
    if t[0] in "\"'":
        return ("str", bytes(t[1:-1], "utf-8").decode("unicode_escape")), i + 1
    if t in ("TRUE", "FALSE"):
        return ("num", 1.0 if t == "TRUE" else 0.0), i + 1
    if t == "NA":
        return ("num", float("nan")), i + 1
    # ASTNumList span "start:count[:stride]"; a NaN count is open-ended (h2o-py renders x[1:] this way)
    m = re.fullmatch(r"(-?\d+):(\d+|nan|NaN)(?::(\d+))?", t)
    if m:
        a = int(m.group(1))
        n = None if m.group(2).lower() == "nan" else int(m.group(2))
        return ("span", (a, n, int(m.group(3) or 1))), i + 1
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
    if isinstance(v, tuple):
        v = [v]
    out = []
    for x in v:
        if isinstance(x, tuple):
            a, cnt, st = (tuple(x) + (1,))[:3]
            if cnt is None:
                if n is None:
                    raise ValueError("an open-ended span needs the extent of the indexed axis")
                cnt = max(0, -(-(n - a) // st))
            out += list(range(a, a + cnt * st, st))
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


def _as_frame(v):
    """A Rapids value as a frame: list of lists -> one column each (padded with NA; string levels ->
    enum columns like AstLevels), flat list -> one row, scalar / string -> 1x1."""
    import numpy as np
    if isinstance(v, H2OFrame):
        return v
    if isinstance(v, (list, tuple)) and v and all(isinstance(x, (list, tuple)) for x in v):
        L = max((len(x) for x in v), default=0)
        data = {}
        for j, col in enumerate(v):
            vals = list(col) + [None] * (L - len(col))
            data[f"C{j + 1}"] = vals
        types = {k: ("enum" if any(isinstance(x, str) for x in c) else None) for k, c in data.items()}
        return H2OFrame(data, column_types={k: t for k, t in types.items() if t})
    if isinstance(v, (list, tuple)):
        return H2OFrame({f"C{j + 1}": [x] for j, x in enumerate(v)})
    if isinstance(v, str):
        return H2OFrame({"C1": [v]}, column_types={"C1": "string"})
    return H2OFrame({"C1": [float("nan") if v is None else float(v)]})


def _mean(a, na_rm=1, axis=0, *rest):
    """AstMean: ``(mean fr na_rm axis)`` -> a 1-row frame of column means (axis 0) or a column of row
    means (axis 1); a scalar argument passes through."""
    if not isinstance(a, H2OFrame):
        return float(a)
    skip = bool(na_rm) if not isinstance(na_rm, str) else na_rm.upper() == "TRUE"
    if int(axis or 0) == 1:
        return a.mean(skipna=skip, axis=1)
    return a.mean(skipna=skip, return_frame=True)


def _reduce_na(name):
    """sumNA / maxNA / minNA (AstSumNA ...): like sum / max / min but any missing value -> NaN."""
    base = _reduce(name)

    def f(a, *rest):
        fr = _frame(a)
        if any(n > 0 for n in fr.nacnt()):
            return float("nan")
        return base(a, *rest)
    return f


def _rows(fr, sel):
    fr = _frame(fr)
    if isinstance(sel, H2OFrame):
        return fr[sel]
    idx = _idx_list(sel, fr.nrows)
    neg = [i for i in idx if isinstance(i, int) and i < 0]
    if neg and len(neg) == len(idx):
        drop = {-i - 1 for i in neg}
        idx = [i for i in range(fr.nrows) if i not in drop]
    return fr._rows(torch.as_tensor(idx, dtype=torch.long, device=engine_device()))


def _cols(fr, sel):
    fr = _frame(fr)
    if isinstance(sel, (int, float, str)):
        sel = [sel]
    idx = _idx_list(sel, fr.ncols)
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
            **{n: _reduce(n) for n in ("sum", "min", "max", "sd", "var", "median")},
            "mean": _mean,
            "sumNA": _reduce_na("sum"), "maxNA": _reduce_na("max"), "minNA": _reduce_na("min"),
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
        self.prims.update(_extended_prims(self))
        from .rapids_more import more_prims
        self.prims.update(more_prims(self))
        self.scopes = []

    # ---- special forms
    def _assign(self, name, value):
        """``(tmp= name expr)`` / ``(assign name expr)``: the value becomes a named frame in the DKV (Java
        Rapids always assigns frames: scalars become 1x1 frames, lists of lists one column per list)."""
        if not isinstance(value, H2OFrame):
            value = _as_frame(value)
        elif value.frame_id != name and dkv.get(value.frame_id) is value:
            # the source keeps its own key (AstAssign builds a new Frame over the same vecs)
            from .parallel import dframe
            with dframe.shard_ctx(value._shard):      # a row-sharded source stays sharded under its new name
                value = H2OFrame._from_columns([value._col(n) for n in value.names])
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
        """(h2o.impute data col method combine_method groupby groupByFrame values) — AstImpute.java:86."""
        fr = _frame(fr)
        by = [int(b) for b in (by if isinstance(by, list) else ([] if by in (None, "_") else [by]))]
        col = int(col)
        r = fr.impute(-1 if col < 0 else col, str(method).lower(), str(combine).lower(),
                      by=[fr.names[b] for b in by] or None)
        return [0.0] if by else [float(x) for x in r] or [0.0]

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
            for sc in reversed(self.scopes):
                if v in sc:
                    return sc[v]
            val = dkv.get(v)
            return val if val is not None else v
        if kind == "fun":
            from .rapids_more import RapidsFunction
            return RapidsFunction(self, *v)
        op = v[0]
        if op[0] != "id":
            raise SyntaxError("call head must be an operator")
        name = op[1]
        if name in ("tmp=", "assign"):
            return self._assign(v[1][1], self.eval_node(v[2]))
        if name == "rm" and v[1][0] in ("id", "str"):
            return self._rm(v[1][1])           # by key: the object may also live under another key
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


# ================================================================================================
# the long tail of ast/prims/** (advmath, math, reducers, mungers, search, string, time, matrix, misc)
def _elementwise(fn):
    """Unary math over every numeric column (scalars pass straight through)."""
    def f(a):
        if isinstance(a, H2OFrame):
            return a._unop(fn)
        return float(fn(torch.tensor(float(a), dtype=torch.float64)))
    return f


def _num_cols(fr):
    return [n for n in fr.names if fr.type(n) in ("real", "int", "time")]


def _col_tensor(fr, i=0):
    return fr.as_tensor(dtype=torch.float64)[:, i]


def _moment(fr, k, central=True):
    out = []
    X = fr[_num_cols(fr)].as_tensor(dtype=torch.float64)
    for j in range(X.shape[1]):
        v = X[:, j]
        v = v[~torch.isnan(v)]
        mu = v.mean()
        out.append(float(((v - mu) ** k).mean()) if central else float((v ** k).mean()))
    return out


def _skew(fr, na_rm=1):
    X = fr[_num_cols(fr)].as_tensor(dtype=torch.float64)
    out = []
    for j in range(X.shape[1]):
        v = X[:, j]
        if na_rm:
            v = v[~torch.isnan(v)]
        n = v.numel()
        m = v.mean()
        s2 = ((v - m) ** 2).mean()
        out.append(float(((v - m) ** 3).mean() / s2 ** 1.5) if n > 2 else float("nan"))
    return out


def _kurt(fr, na_rm=1):
    X = fr[_num_cols(fr)].as_tensor(dtype=torch.float64)
    out = []
    for j in range(X.shape[1]):
        v = X[:, j]
        if na_rm:
            v = v[~torch.isnan(v)]
        m = v.mean()
        s2 = ((v - m) ** 2).mean()
        out.append(float(((v - m) ** 4).mean() / s2 ** 2))
    return out


def _mad(fr, combine="interpolate", const=1.4826):
    v = _col_tensor(fr)
    v = v[~torch.isnan(v)]
    med = torch.quantile(v, 0.5)
    return float(const * torch.quantile((v - med).abs(), 0.5))


def _frame_of(cols: dict):
    dev = engine_device()
    return H2OFrame._from_columns([Column(n, "real", torch.as_tensor(np.asarray(v, dtype=np.float64), device=dev))
                                   for n, v in cols.items()])


def _seq(a, b, by=1):
    return _frame_of({"C1": np.arange(float(a), float(b) + (1e-9 if by > 0 else -1e-9), float(by))})


def _rep_len(x, n):
    n = int(n)
    if isinstance(x, H2OFrame):
        v = _col_tensor(x).cpu().numpy()
        return _frame_of({x.names[0]: np.resize(v, n)})
    return _frame_of({"C1": np.full(n, float(x))})


def _match(fr, table, nomatch=float("nan"), *rest):
    c = fr._col(0)
    vals = table if isinstance(table, list) else [table]
    if c.type == "enum":
        dom = c.domain
        lut = {str(v): i + 1 for i, v in reversed(list(enumerate(vals)))}
        codes = c.data.cpu().numpy()
        out = np.array([lut.get(dom[int(k)], nomatch) if not np.isnan(k) else nomatch for k in codes], dtype=np.float64)
    else:
        v = c.data.double().cpu().numpy()
        lut = {float(x): i + 1 for i, x in reversed(list(enumerate(vals)))}
        out = np.array([lut.get(float(x), nomatch) for x in v], dtype=np.float64)
    return _frame_of({"C1": out})


def _which_mm(fr, na_rm=1, axis=0, want_max=True):
    X = fr[_num_cols(fr)].as_tensor(dtype=torch.float64)
    fill = -math.inf if want_max else math.inf
    Xf = torch.where(torch.isnan(X), torch.full_like(X, fill), X)
    if int(axis) == 0:
        idx = (Xf.argmax(0) if want_max else Xf.argmin(0)).double()
        return _frame_of({n: [float(i)] for n, i in zip(_num_cols(fr), idx.tolist())})
    idx = (Xf.argmax(1) if want_max else Xf.argmin(1)).double()
    return _frame_of({"which.max" if want_max else "which.min": idx.cpu().numpy()})


def _sumaxis(fr, na_rm=0, axis=0):
    X = fr[_num_cols(fr)].as_tensor(dtype=torch.float64)
    if int(na_rm):
        X = torch.nan_to_num(X, nan=0.0)
    if int(axis) == 0:
        return _frame_of({n: [float(v)] for n, v in zip(_num_cols(fr), X.sum(0).tolist())})
    return _frame_of({"sum": X.sum(1).cpu().numpy()})


def _prod(fr, na_rm=0):
    X = fr[_num_cols(fr)].as_tensor(dtype=torch.float64)
    if na_rm:
        X = torch.nan_to_num(X, nan=1.0)
    return float(X.prod())


def _distance(a, b, measure="l2"):
    A, B = a.as_tensor(dtype=torch.float64), b.as_tensor(dtype=torch.float64)
    m = measure.lower()
    if m == "l1":
        D = torch.cdist(A, B, p=1)
    elif m == "l2":
        D = torch.cdist(A, B, p=2)
    elif m == "cosine":
        D = (A @ B.T) / (A.norm(dim=1)[:, None] * B.norm(dim=1)[None, :]).clamp(min=1e-300)
    elif m == "cosine_sq":
        D = ((A @ B.T) / (A.norm(dim=1)[:, None] * B.norm(dim=1)[None, :]).clamp(min=1e-300)) ** 2
    else:
        raise ValueError(f"unknown distance measure {measure}")
    return H2OFrame.from_tensor(D.float(), [f"C{i + 1}" for i in range(D.shape[1])])


def _str_distance(a, b, measure="lv", compare_empty=1):
    def lev(x, y):
        prev = list(range(len(y) + 1))
        for i, cx in enumerate(x, 1):
            cur = [i]
            for j, cy in enumerate(y, 1):
                cur.append(min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (cx != cy)))
            prev = cur
        return prev[-1]
    xa = a._col(0).to_numpy()
    xb = b._col(0).to_numpy()
    out = []
    for x, y in zip(xa, xb):
        if x is None or y is None or (isinstance(x, float) and math.isnan(x)) or (isinstance(y, float) and math.isnan(y)):
            out.append(float("nan"))
            continue
        x, y = str(x), str(y)
        if not compare_empty and (x == "" or y == ""):
            out.append(float("nan"))
            continue
        if measure == "lv":
            out.append(float(lev(x, y)))
        elif measure == "jaccard":
            sx, sy = set(x), set(y)
            out.append(len(sx & sy) / max(1, len(sx | sy)))
        else:
            out.append(1.0 - lev(x, y) / max(1, max(len(x), len(y))))
    return _frame_of({"C1": out})


def _tokenize(fr, regex):
    out = []
    for col in fr.names:
        for v in fr._col(col).to_numpy():
            if v is None or (isinstance(v, float) and math.isnan(v)):
                continue
            out += [t for t in re.split(regex, str(v)) if t != ""] + [None]
    return H2OFrame._from_columns([Column("C1", "string", strings=np.array(out, dtype=object))])


def _na_cnt(fr):
    return [float(x) for x in fr.nacnt()]


def _filter_na_cols(fr, frac):
    n = max(1, fr.nrows)
    return [float(i) for i, c in enumerate(fr.nacnt()) if c / n <= float(frac)]


def _rank_within_groupby(fr, groups, sorts, asc, new_name="New_Rank_column", sort_cols_order=0):
    g = [fr.names[int(i)] for i in _idx_list(groups)]
    sc = [fr.names[int(i)] for i in _idx_list(sorts)]
    asc = [bool(int(x)) for x in (asc if isinstance(asc, list) else [asc])]
    df = fr.as_data_frame()
    df["__i"] = np.arange(len(df))
    ds = df.sort_values(g + sc, ascending=[True] * len(g) + asc, kind="mergesort")
    ok = ds[sc].notna().all(axis=1)
    rank = np.full(len(df), np.nan)
    r = ds[ok].groupby(g, sort=False).cumcount().values + 1
    rank[ds[ok]["__i"].values] = r
    out = fr.cbind(_frame_of({new_name: rank}))
    return out


def _set_domain(fr, inplace, dom):
    c = fr._col(0)
    newdom = dom if isinstance(dom, list) else [dom]
    c.domain = [str(x) for x in newdom]
    return fr


def _relevel_by_freq(fr, weights=None, top_n=-1):
    out = []
    for n in fr.names:
        c = fr._col(n)
        if c.type != "enum":
            out.append(c)
            continue
        codes = c.data.long()
        ok = codes >= 0
        cnt = torch.bincount(codes[ok], minlength=len(c.domain)).cpu().numpy()
        order = sorted(range(len(c.domain)), key=lambda k: (-cnt[k], k))
        if int(top_n) > 0:
            order = order[:int(top_n)] + sorted(set(range(len(c.domain))) - set(order[:int(top_n)]))
        remap = torch.empty(len(c.domain), dtype=torch.long, device=codes.device)
        remap[torch.as_tensor(order, device=codes.device)] = torch.arange(len(order), device=codes.device)
        newc = torch.where(codes >= 0, remap[codes.clamp(min=0)], codes).to(c.data.dtype)
        out.append(Column(n, "enum", torch.where(torch.isnan(c.data), c.data, newc), [c.domain[k] for k in order]))
    return H2OFrame._from_columns(out)


def _append_levels(fr, levels, inplace=0):
    c = fr._col(0)
    c.domain = list(c.domain) + [str(x) for x in (levels if isinstance(levels, list) else [levels])]
    return fr


def _getrow(fr):
    if fr.nrows != 1:
        raise ValueError("getrow needs a single-row frame")
    return [float(v) for v in fr.as_tensor(dtype=torch.float64)[0].tolist()]


def _minus1(v):
    return v - 1 if isinstance(v, H2OFrame) else float(v) - 1


def _mktime(yr, mo, dy, hr, mi, se, ms):
    import pandas as pd
    parts = [yr, mo, dy, hr, mi, se, ms]
    n = max(p.nrows if isinstance(p, H2OFrame) else 1 for p in parts)
    vals = [(_col_tensor(p).cpu().numpy() if isinstance(p, H2OFrame) else np.full(n, float(p))) for p in parts]
    ts = pd.to_datetime(dict(year=vals[0], month=vals[1] + 1, day=vals[2] + 1, hour=vals[3], minute=vals[4],
                             second=vals[5], ms=vals[6]), errors="coerce")
    ms_ = (ts.astype("int64") // 1_000_000).astype(np.float64).values
    return H2OFrame._from_columns([Column("C1", "time", torch.as_tensor(ms_, device=engine_device()))])


def _as_fn(sess, f):
    from .rapids_more import as_function
    return as_function(sess, f)


def _extended_prims(sess):
    fr = _frame
    pi = math.pi
    return {
        # math / advmath
        "acos": _elementwise(torch.acos), "acosh": _elementwise(torch.acosh), "asin": _elementwise(torch.asin),
        "asinh": _elementwise(torch.asinh), "atan": _elementwise(torch.atan), "atanh": _elementwise(torch.atanh),
        "cosh": _elementwise(torch.cosh), "sinh": _elementwise(torch.sinh),
        "cospi": _elementwise(lambda v: torch.cos(pi * v)), "sinpi": _elementwise(lambda v: torch.sin(pi * v)),
        "tanpi": _elementwise(lambda v: torch.tan(pi * v)), "lgamma": _elementwise(torch.lgamma),
        "gamma": _elementwise(lambda v: torch.exp(torch.lgamma(v)) * torch.where(
            (v < 0) & (torch.floor(v).remainder(2) == 0), -torch.ones_like(v), torch.ones_like(v))),
        "digamma": _elementwise(torch.digamma), "trigamma": _elementwise(lambda v: torch.polygamma(1, v)),
        "round": lambda a, d=0: fr(a).round(int(d)) if isinstance(a, H2OFrame) else float(round(a, int(d))),
        "signif": lambda a, d=6: fr(a).signif(int(d)),
        "none": lambda a: a,
        # AstMoment: a time column from year, month (1-12), day (1-31), hour, minute, second, msec (UTC)
        "moment": lambda yr, mo, dy, hr, mi, se, ms: _mktime(yr, _minus1(mo), _minus1(dy), hr, mi, se, ms),
        "skewness": lambda a, na_rm=1: _skew(fr(a), na_rm), "kurtosis": lambda a, na_rm=1: _kurt(fr(a), na_rm),
        "h2o.mad": lambda a, combine="interpolate", const=1.4826: _mad(fr(a), combine, float(const)),
        "prod": lambda a: _prod(fr(a)), "prod.na": lambda a: _prod(fr(a), True),
        "sumaxis": lambda a, na_rm=0, axis=0: _sumaxis(fr(a), na_rm, axis),
        "mode": lambda a: float(torch.mode(fr(a)._col(0).data[~torch.isnan(fr(a)._col(0).data)]).values),
        # reducers over predicates
        "any": lambda a: float(bool(fr(a).any())), "all": lambda a: float(bool(fr(a).all())),
        "any.na": lambda a: float(any(c > 0 for c in fr(a).nacnt())),
        "any.factor": lambda a: float(any(fr(a).type(n) == "enum" for n in fr(a).names)),
        "naCnt": lambda a: _na_cnt(fr(a)),
        "is.character": lambda a: [float(fr(a).type(n) == "string") for n in fr(a).names],
        "is.numeric": lambda a: [float(fr(a).type(n) in ("real", "int")) for n in fr(a).names],
        "which.max": lambda a, na_rm=1, axis=0: _which_mm(fr(a), na_rm, axis, True),
        "which.min": lambda a, na_rm=1, axis=0: _which_mm(fr(a), na_rm, axis, False),
        # mungers
        "cut": lambda a, breaks, labels=None, lowest=0, right=1, dig=3: fr(a).cut(
            list(breaks), None if not isinstance(labels, list) or not labels else labels, bool(lowest), bool(right), int(dig)),
        "h2o.fillna": lambda a, method="forward", axis=0, maxlen=1: fr(a).fillna(method, int(axis), int(maxlen)),
        "difflag1": lambda a: fr(a).difflag1(), "flatten": lambda a: fr(a).flatten(),
        "dropdup": lambda a, cols, keep="first": fr(a).drop_duplicates([fr(a).names[int(i)] for i in _idx_list(cols)], keep),
        "getrow": lambda a: _getrow(fr(a)),
        "melt": lambda a, ids, vals, var="variable", val="value", skipna=0: fr(a).melt(
            [fr(a).names[int(i)] for i in _idx_list(ids)],
            None if not vals else [fr(a).names[int(i)] for i in _idx_list(vals)], var, val, bool(skipna)),
        "pivot": lambda a, index, column, value: fr(a).pivot(index, column, value),
        "rank_within_groupby": lambda a, g, s, asc, name="New_Rank_column", o=0: _rank_within_groupby(fr(a), g, s, asc, name, o),
        "relevel": lambda a, lvl: fr(a).relevel(lvl),
        "relevel.by.freq": lambda a, w=None, top_n=-1: _relevel_by_freq(fr(a), w, top_n),
        "rename": lambda old, new: sess._assign(new, dkv.get(old) if isinstance(old, str) else old),
        "rep_len": lambda x, n: _rep_len(x, n),
        "seq": lambda a, b, by=1: _seq(a, b, by), "seq_len": lambda n: _seq(1, n),
        "setDomain": lambda a, inplace, dom: _set_domain(fr(a), inplace, dom),
        "setLevel": lambda a, lvl: _set_level(fr(a), lvl),
        "appendLevels": lambda a, lv, inplace=0: _append_levels(fr(a), lv, inplace),
        "filterNACols": lambda a, frac: _filter_na_cols(fr(a), frac),
        "apply": lambda a, margin, f: fr(a).apply(_as_fn(sess, f), 0 if int(margin) == 2 else 1),  # R margins
        "t": lambda a: fr(a).transpose(), "topn": lambda a, col, pct, top=1: fr(a).topN(int(col), float(pct), int(top)),
        "hist": lambda a, breaks="sturges": fr(a).hist(breaks if isinstance(breaks, str) else list(breaks)),
        "kfold_column": lambda a, k, seed=-1: fr(a).kfold_column(int(k), int(seed)),
        "modulo_kfold_column": lambda a, k: fr(a).modulo_kfold_column(int(k)),
        "stratified_kfold_column": lambda a, k, seed=-1: fr(a).stratified_kfold_column(int(k), int(seed)),
        "h2o.random_stratified_split": lambda a, frac, seed=-1: fr(a).stratified_split(float(frac), int(seed)),
        "match": lambda a, table, nomatch=float("nan"), *r: _match(fr(a), table, nomatch),
        "distance": lambda a, b, m="l2": _distance(fr(a), fr(b), m),
        "ls": lambda: H2OFrame._from_columns([Column("key", "string", strings=np.array(list(dkv.keys()), dtype=object))]),
        # strings
        "lstrip": lambda a, s=" ": fr(a).lstrip(s), "rstrip": lambda a, s=" ": fr(a).rstrip(s),
        "substring": lambda a, s, e=None: fr(a).substring(int(s), None if e is None or (isinstance(e, float) and math.isnan(e)) else int(e)),
        "grep": lambda a, pat, ic=0, inv=0, logical=0: fr(a).grep(pat, bool(ic), bool(inv), bool(logical)),
        "countmatches": lambda a, pat: fr(a).countmatches(pat), "strsplit": lambda a, pat: fr(a).strsplit(pat),
        "entropy": lambda a: fr(a).entropy(), "tokenize": lambda a, rx: _tokenize(fr(a), rx),
        "replacefirst": lambda a, pat, rep, ic=0: fr(a).sub(pat, rep, bool(ic)),
        "replaceall": lambda a, pat, rep, ic=0: fr(a).gsub(pat, rep, bool(ic)),
        "strDistance": lambda a, b, m="lv", ce=1: _str_distance(fr(a), fr(b), m, int(ce)),
        "num_valid_substrings": lambda a, path: _num_valid_substrings(fr(a), path),
        # time
        "minute": lambda a: fr(a).minute(), "second": lambda a: fr(a).second(), "week": lambda a: fr(a).week(),
        "millis": lambda a: fr(a)._unop(lambda v: torch.remainder(v, 1000.0)),
        "as.Date": lambda a, f: fr(a).as_date(f),
        "mktime": _mktime,
        "getTimeZone": lambda: "UTC", "listTimeZones": lambda: H2OFrame._from_columns([Column("C1", "string", strings=np.array(["UTC"], dtype=object))]),
        "setTimeZone": lambda tz: tz,
        # assignment / models / misc
        ":=": lambda dst, src, cols, rows=None: _assign_cols(fr(dst), src, cols, rows),
        "tf-idf": lambda a, doc=0, text=1, pre=1, cs=1: _tfidf(fr(a), int(doc), int(text), bool(pre), bool(cs)),
        "perfectAUC": lambda p, y: _perfect_auc(fr(p), fr(y)),
        "model.reset.threshold": lambda m, t: _reset_threshold(m, float(t)),
        "PermutationVarImp": lambda m, f, metric="AUTO", n_samples=-1, n_repeats=1, features=None, seed=-1:
            _permutation_varimp(m, fr(f), metric, int(n_repeats), int(seed)),
        "setproperty": lambda k, v: _PROPS.__setitem__(k, v) or v,
        "makeLeaderboard": lambda models, frame=None, sort="AUTO", extra=None, scoring="AUTO":
            _leaderboard(models, frame, sort),
        "transform": lambda m, f, *r: _model_obj(m).transform(fr(f)),
        "result": lambda m: _model_obj(m).output.get("result_frame"),
    }


_PROPS = {}


def _model_obj(m):
    obj = dkv.get(m) if isinstance(m, str) else m
    return getattr(obj, "_model", obj)


def _assign_cols(dst, src, cols, rows=None):
    """``(:= dst src cols rows)``: overwrite columns (optionally rows) of dst in place (AstRectangleAssign)."""
    idx = _idx_list(cols, dst.ncols)
    names = [dst.names[int(i)] if not isinstance(i, str) else i for i in idx]
    for k, n in enumerate(names):
        if isinstance(src, H2OFrame):
            sc = src._col(min(k, src.ncols - 1))
            newv = sc.data.double()
        else:
            newv = torch.full((dst.nrows,), float(src), dtype=torch.float64, device=engine_device())
        if rows is None or (isinstance(rows, list) and not rows):
            if isinstance(src, H2OFrame) and sc.type in ("enum", "string"):
                dst._cols[n] = Column(n, sc.type, sc.data.clone() if sc.data is not None else None, sc.domain,
                                      sc.strings)
                continue
            dst._cols[n] = Column(n, "real", newv.clone())
        else:
            ridx = torch.as_tensor(_idx_list(rows, dst.nrows), dtype=torch.long, device=engine_device())
            cur = dst._col(n).data.double().clone()
            cur[ridx] = newv if newv.numel() == ridx.numel() else newv[0]
            dst._cols[n] = Column(n, "real", cur)
    return dst


def _tfidf(fr, doc, text, preprocess, case_sensitive):
    from .frame_ops import tf_idf
    return tf_idf(fr, doc, text, preprocess, case_sensitive)


def _perfect_auc(p, y):
    from . import metrics as mm
    yv = y.as_tensor(dtype=torch.float64)[:, 0]
    pv = p.as_tensor(dtype=torch.float64)[:, 0]
    return float(mm.binomial_metrics(yv, pv).get("AUC"))


def _reset_threshold(m, t):
    obj = _model_obj(m)
    old = obj.default_threshold()
    for k in ("training_metrics", "validation_metrics"):
        if obj.output.get(k):
            obj.output[k]["max_f1_threshold"] = t
    return [float(old) if old is not None else float("nan")]


def _permutation_varimp(m, frame, metric="AUTO", n_repeats=1, seed=-1):
    """Permutation importance (hex/PermutationVarImp.java): metric degradation when one predictor's values
    are shuffled; returns a frame of (Variable, Relative, Scaled, Percentage)."""
    obj = _model_obj(m)
    X, off = frame.model_matrix(obj.info, device=obj.device)
    y = frame.response_tensor(obj.info, device=obj.device)
    base = obj.metrics_for(X, y, None, off)
    mname = {"AUTO": "AUC" if obj.model_category == "Binomial" else ("logloss" if obj.model_category == "Multinomial"
                                                                    else "MSE")}.get(metric, metric)
    higher = mname.upper() in ("AUC", "AUCPR", "PR_AUC", "R2")
    b0 = float(base.get(mname) if hasattr(base, "get") else base[mname])
    g = torch.Generator(device="cpu").manual_seed(seed if seed >= 0 else 1234)
    imp = []
    for j in range(X.shape[0]):
        acc = 0.0
        for _ in range(max(1, n_repeats)):
            Xp = X.clone()
            perm = torch.randperm(X.shape[1], generator=g).to(X.device)
            Xp[j] = X[j][perm]
            mv = obj.metrics_for(Xp, y, None, off)
            v = float(mv.get(mname) if hasattr(mv, "get") else mv[mname])
            acc += (b0 - v) if higher else (v - b0)
        imp.append(acc / max(1, n_repeats))
    imp = np.maximum(np.asarray(imp), 0.0)
    mx, tot = max(imp.max(), 1e-300), max(imp.sum(), 1e-300)
    order = np.argsort(-imp, kind="stable")
    dev = engine_device()
    return H2OFrame._from_columns([
        Column("Variable", "string", strings=np.array([obj.info.x[i] for i in order], dtype=object)),
        Column("Relative Importance", "real", torch.as_tensor(imp[order], device=dev)),
        Column("Scaled Importance", "real", torch.as_tensor(imp[order] / mx, device=dev)),
        Column("Percentage", "real", torch.as_tensor(imp[order] / tot, device=dev))])


def _leaderboard(models, frame, sort):
    from .automl import leaderboard_frame
    ms = [_model_obj(k) for k in (models if isinstance(models, list) else [models])]
    return leaderboard_frame(ms, None if frame is None or isinstance(frame, (str, list)) else _frame(frame), sort)


def _set_level(fr, lvl):
    c = fr._col(0)
    k = c.domain.index(lvl)
    data = torch.full_like(c.data, float(k))
    return H2OFrame._from_columns([Column(c.name, "enum", data, list(c.domain))])


def _num_valid_substrings(fr, path):
    with open(path) as f:
        words = {w.strip() for w in f if w.strip()}
    out = []
    for v in fr._col(0).to_numpy():
        if v is None or (isinstance(v, float) and math.isnan(v)):
            out.append(float("nan"))
            continue
        s = str(v)
        out.append(float(sum(1 for i in range(len(s)) for j in range(i + 2, len(s) + 1) if s[i:j] in words)))
    return _frame_of({"C1": out})


_session = Session()


def rapids(expr: str):
    return _session.exec(expr)
