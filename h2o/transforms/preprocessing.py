"""Assembly transforms (reference ``h2o-py/h2o/transforms/preprocessing.py``): H2OScaler, H2OColSelect,
H2OColOp, H2OBinaryOp.

The in-process frames are eager, so a step's Rapids AST (what the reference client captures by applying the
operation to a lazy placeholder frame) is rendered here from the operation's name and arguments; the engine's
Assembly (``llama_github_io_amd/assembly.py``) then runs exactly what the REST ``/99/Assembly`` route runs."""
from __future__ import annotations

import warnings

from .transform_base import H2OTransformer

# H2OFrame method -> Rapids primitive (where the names differ)
_RAPIDS_NAMES = {"gsub": "replaceall", "sub": "replacefirst", "asnumeric": "as.numeric", "ascharacter": "as.character",
                 "asfactor": "as.factor", "isna": "is.na", "__add__": "+", "__radd__": "+", "__sub__": "-",
                 "__rsub__": "-", "__mul__": "*", "__rmul__": "*", "__truediv__": "/", "__rtruediv__": "/",
                 "__floordiv__": "intDiv", "__mod__": "%", "__pow__": "^", "__lt__": "<", "__le__": "<=",
                 "__gt__": ">", "__ge__": ">=", "__eq__": "==", "__ne__": "!=", "__and__": "&", "__or__": "|",
                 "strdistance": "strDistance", "trim": "trim", "lstrip": "lstrip", "rstrip": "rstrip"}


def _lit(v) -> str:
    """A Python value as a Rapids literal."""
    if isinstance(v, H2OCol):
        return v.ast()
    if isinstance(v, bool):
        return "TRUE" if v else "FALSE"
    if isinstance(v, (int, float)):
        return repr(v)
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(_lit(x) for x in v) + "]"
    return "'" + str(v).replace("\\", "\\\\").replace("'", "\\'") + "'"


def _op_name(fun) -> str:
    n = getattr(fun, "__name__", str(fun))
    return _RAPIDS_NAMES.get(n, n)


class H2OScaler(H2OTransformer):
    """Center / scale every column (fitted means and standard deviations, or given lists)."""

    def __init__(self, center=True, scale=True):
        self.parms = dict(center=center, scale=scale)
        if center is None or scale is None:
            raise ValueError("centers and scales must not be None.")
        self._means = None
        self._stds = None

    @property
    def means(self):
        return self._means

    @property
    def stds(self):
        return self._stds

    def fit(self, X, y=None, **params):
        if isinstance(self.parms["center"], (tuple, list)):
            self._means = list(self.parms["center"])
        if isinstance(self.parms["scale"], (tuple, list)):
            self._stds = list(self.parms["scale"])
        if self._means is None:
            self._means = [float(X[n].mean()[0]) for n in X.names] if self.parms["center"] else False
        if self._stds is None:
            self._stds = [float(X[n].sd()[0]) for n in X.names] if self.parms["scale"] else False
        return self

    def transform(self, X, y=None, **params):
        return X.scale(self.means, self.stds)

    def inverse_transform(self, X, y=None, **params):
        for i in range(X.ncol):
            X[i] = self.means[i] + self.stds[i] * X[i]
        return X

    def to_rest(self, step_name):
        return super().to_rest([step_name, "H2OScaler", "(cols_py dummy [])", False, "|"])


class H2OColSelect(H2OTransformer):
    def __init__(self, cols):
        self.cols = cols
        self.parms = dict(cols=cols)

    def fit(self, X, y=None, **params):
        return self

    def transform(self, X, y=None, **params):
        return X[self.cols]

    def to_rest(self, step_name):
        return super().to_rest([step_name, "H2OColSelect", "(cols_py dummy %r)" % self.cols, False, "|"])


class H2OCol:
    """A reference to another column of the frame in a binary operation."""

    def __init__(self, column):
        self.col = column

    def ast(self):
        return "(cols_py dummy %s)" % _lit(self.col)


class H2OColOp(H2OTransformer):
    """A column operation; ``inplace``: replace the column, else append the result (named ``new_col_name`` or
    uniquely after the column)."""

    def __init__(self, op, col=None, inplace=True, new_col_name=None, **params):
        self.fun = op
        self.col = col
        self.inplace = inplace
        self.params = params
        self.new_col_name = new_col_name
        self.parms = dict(op=op, col=col, inplace=inplace, new_col_name=new_col_name, **params)
        if inplace and new_col_name is not None:
            warnings.warn("inplace was False, but new_col_name was not empty. Ignoring new_col_name.")
        if isinstance(col, (list, tuple)):
            raise ValueError("col must be None or a single column.")

    def fit(self, X, y=None, **params):
        return self

    def _args(self):
        return [_lit(v) for v in self.params.values()]

    def _ast(self):
        target = "(cols_py dummy %s)" % _lit(self.col) if self.col is not None else "dummy"
        return "(%s %s)" % (_op_name(self.fun), " ".join([target] + self._args()))

    def transform(self, X, y=None, **params):
        res = self.fun(X[self.col], **self.params) if self.col is not None else self.fun(X, **self.params)
        if self.inplace:
            X[self.col] = res
            return X
        return X.cbind(res)

    def to_rest(self, step_name):
        names = self.new_col_name
        if names is None:
            names = ["|"]
        elif not isinstance(names, (list, tuple)):
            names = [names]
        return super().to_rest([step_name, self.__class__.__name__, self._ast(), self.inplace, "|".join(names)])


class H2OBinaryOp(H2OColOp):
    """A binary operation between a column and ``left`` / ``right`` (a constant or :class:`H2OCol`)."""

    def __init__(self, op, col, inplace=True, new_col_name=None, left=None, right=None, **params):
        super().__init__(op, col, inplace, new_col_name, **params)
        self.left_is_col = isinstance(left, H2OCol)
        self.right_is_col = isinstance(right, H2OCol)
        self.left = left
        self.right = right
        if left is None and right is None:
            raise ValueError("left and right cannot both be None")

    def _ast(self):
        col = "(cols_py dummy %s)" % _lit(self.col)
        if self.left is None:
            a, b = col, _lit(self.right)
        else:
            a, b = _lit(self.left), col
        return "(%s %s %s)" % (_op_name(self.fun), a, b)

    def transform(self, X, y=None, **params):
        other = lambda v: X[v.col] if isinstance(v, H2OCol) else v  # noqa: E731
        res = self.fun(X[self.col], other(self.right)) if self.left is None else self.fun(other(self.left), X[self.col])
        if self.inplace:
            X[self.col] = res
            return X
        return X.cbind(res)
