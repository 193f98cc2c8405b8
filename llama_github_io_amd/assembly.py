"""Munging pipelines: Assembly (reference: ``h2o-core/src/main/java/water/rapids/Assembly.java``,
``water/rapids/transforms/{Transform,H2OColSelect,H2OColOp,H2OBinaryOp,H2OScaler}.java``,
``water/api/AssemblyHandler.java``; client ``h2o-py/h2o/assembly.py``, ``h2o-py/h2o/transforms/*``).

An assembly is an ordered list of transforms, each a Rapids expression over a placeholder frame ``dummy``
(``(cos (cols_py dummy 'x'))``). ``fit`` runs them in order on a frame — every step is an ordinary Rapids
evaluation on the device-resident columns — and records each step's input/output schema; ``to_java`` then
emits the reference's per-row ``GenMunger`` POJO source (``hex.genmodel.GenMunger`` steps) from that schema.

Steps arrive from the REST client in the reference wire form ``name__Class__ast__inplace__newnames``
(``|`` = no new names), the form ``h2o-py``'s ``H2OTransformer.to_rest`` produces.
"""
from __future__ import annotations

import itertools
import uuid

from .core import dkv
from .frame import H2OFrame

PLACEHOLDER = "dummy"


def _types(fr: H2OFrame) -> list:
    """Vec type strings as Frame.typesStr: Numeric / Enum / String / Time / UUID."""
    m = {"real": "Numeric", "int": "Numeric", "enum": "Enum", "string": "String", "time": "Time", "uuid": "UUID"}
    return [m.get(fr.type(n), "Numeric") for n in fr.names]


def _java_list(strs) -> str:
    if not strs:
        return '"null"'
    return ",".join(f'"{s}"' for s in strs)


def _subst(ast: str, key: str) -> str:
    """Replace the placeholder frame id (a whole token outside quotes) by ``key``."""
    from .rapids import tokenize
    return " ".join(key if t == PLACEHOLDER else t for t in tokenize(ast))


def _run(ast: str, fr: H2OFrame) -> H2OFrame:
    """Evaluate a step's Rapids AST with the placeholder bound to ``fr`` (registered under its frame id)."""
    from .rapids import rapids
    if dkv.get(fr.frame_id) is not fr:
        dkv.put(fr.frame_id, fr)
    out = rapids(_subst(ast, fr.frame_id))
    if not isinstance(out, H2OFrame):
        raise ValueError(f"assembly step {ast!r} did not produce a frame")
    return out


def _parse_call(ast: str):
    """Head operator and argument nodes of a Rapids call."""
    from .rapids import parse, tokenize
    node, _ = parse(tokenize(ast), 0)
    if node[0] != "call" or not node[1] or node[1][0][0] != "id":
        raise ValueError(f"assembly step is not a Rapids call: {ast!r}")
    return node[1][0][1], node[1][1:]


def _old_col(node):
    """The column a (cols_py dummy <name>) sub-expression selects (H2OColOp.findOldName), breadth first."""
    queue = [node]
    while queue:
        n = queue.pop(0)
        if n[0] != "call":
            continue
        v = n[1]
        if (len(v) == 3 and v[0] == ("id", "cols_py") and v[1] == ("id", PLACEHOLDER)):
            return v[2][1] if v[2][0] in ("str", "id") else str(v[2][1])
        queue += [a for a in v[1:] if a[0] == "call"]
    return None


def _render(n) -> str:
    """Rapids text of a parsed argument node (for the POJO's _params)."""
    if n[0] == "str":
        return n[1]
    if n[0] == "num":
        v = n[1]
        return str(int(v)) if float(v).is_integer() else repr(v)
    if n[0] == "list":
        return "[" + " ".join(_render(a) for a in n[1]) + "]"
    return str(n[1])


class Transform:
    """One assembly step (Transform.java): name, Rapids AST over ``dummy``, inplace flag, new column names."""

    def __init__(self, name: str, ast: str, inplace: bool, new_names):
        self.name, self.ast, self.inplace = name, ast, bool(inplace)
        self.new_names = list(new_names) if new_names else None
        self.params = {}                  # name -> rendered value (Transform._params)
        self.in_names = self.in_types = self.out_names = self.out_types = None

    def fit(self, fr: H2OFrame) -> "Transform":
        return self

    def transform(self, fr: H2OFrame) -> H2OFrame:
        self.in_names, self.in_types = list(fr.names), _types(fr)
        out = self._transform(fr)
        self.out_names, self.out_types = list(out.names), _types(out)
        return out

    def fit_transform(self, fr: H2OFrame) -> H2OFrame:
        return self.fit(fr).transform(fr)

    def _transform(self, fr):
        raise NotImplementedError

    def gen_class(self) -> str:
        """Transform.genClass: the step's nested class of the munging POJO."""
        if self.in_names is None:
            raise ValueError(f"assembly step {self.name} was never fitted")
        s = [f"  class {self.name} extends Step<{self.name}> {{\n",
             f"    public {self.name}() {{ super(new String[]{{{_java_list(self.in_names)}}},\n",
             f"                                new String[]{{{_java_list(self.in_types)}}},"
             f"                                new String[]{{{_java_list(self.out_names)}}});\n"]
        for k, v in self.params.items():
            vv = v.replace("\\", "\\\\").replace('"', '\\"')
            s.append(f'    _params.put("{k}", new String[]{{"{vv}"}});\n')
        s.append("  }\n")
        return "".join(s) + self.gen_class_impl() + "  }\n"

    def gen_class_impl(self) -> str:
        raise NotImplementedError(f"{type(self).__name__} has no POJO form")


class H2OColSelect(Transform):
    """(cols_py dummy [names]) — keep a subset of the columns (H2OColSelect.java)."""

    def __init__(self, name, ast, inplace, new_names):
        super().__init__(name, ast, inplace, new_names)
        _, args = _parse_call(ast)
        sel = args[1] if len(args) > 1 else None
        if sel is None:
            self.cols = None
        elif sel[0] == "list":
            self.cols = [a[1] for a in sel[1]]
        else:
            self.cols = [sel[1]]

    def _transform(self, fr):
        return _run(self.ast, fr)

    def gen_class_impl(self):
        s = ["    @Override public RowData transform(RowData row) {\n", "      RowData colSelect = new RowData();\n"]
        for c in self.cols or []:
            s.append(f'      colSelect.put("{c}", row.get("{c}"));\n')
        s.append("      return colSelect;\n    }\n")
        return "".join(s)


class H2OColOp(Transform):
    """A column operation (H2OColOp.java): the result replaces the column (inplace) or is appended under a new,
    unique name; several result columns are appended one by one."""

    def __init__(self, name, ast, inplace, new_names):
        super().__init__(name, ast, inplace, new_names)
        self.fun, args = _parse_call(ast)
        self.old_col = None
        for a in args:
            if a[0] == "call":
                self.old_col = _old_col(a)
                break
        self.multi = False
        self.new_cols = None
        self.new_type = "Numeric"
        if len(args) > 1:                               # H2OColOp.setupParams: the first argument is the frame
            for i, a in enumerate(args):
                self._param(_arg_name(self.fun, i), a)

    def _param(self, name, a):
        if a[0] != "call":
            self.params[name] = _render(a)

    def _transform(self, fr):
        res = _run(self.ast, fr)
        out = _copy(fr)
        self.new_type = _types(res)[0] if res.ncols else "Numeric"
        self.multi = res.ncols > 1
        if self.multi:
            names = self.new_names or []
            self.new_cols = []
            for i in range(res.ncols):
                nm = names[i] if i < len(names) else _uniquify(out, self.new_cols[-1] if i else self.old_col)
                self.new_cols.append(nm)
                out = out.cbind(_renamed(res[:, i], nm))
            if self.inplace and self.old_col in out.names:
                out = out.drop(self.old_col)
            return out
        if self.inplace:
            nm = self.old_col
            self.new_cols = [nm]
            out[nm] = res
            return out
        nm = (self.new_names or [None])[0] or _uniquify(out, self.old_col)
        self.new_cols = [nm]
        return out.cbind(_renamed(res, nm))

    def _lookup(self):
        return self.fun.replace(".", "")

    def _row_param(self):
        return ""

    def gen_class_impl(self):
        if self.old_col not in (self.in_names or []):
            raise ValueError(f"Unknown column {self.old_col} (known: {self.in_names})")
        cast = "Double" if self.in_types[self.in_names.index(self.old_col)] == "Numeric" else "String"
        jt = "String" if self.new_type in ("String", "Enum") else "double"
        call = f'GenMunger.{self._lookup()}(({cast})row.get("{self.old_col}"), _params)'
        s = ["    @Override public RowData transform(RowData row) {\n", self._row_param()]
        if self.multi:
            s.append(f"     {jt}[] res = {call};\n")
            for i, c in enumerate(self.new_cols):
                s.append(f'      row.put("{c}",({i}>=res.length)?"":res[{i}]);\n')
        else:
            s.append(f"      {jt} res = {call};\n")
            s.append(f'      row.put("{self.new_cols[0]}", res);\n')
        s.append("      return row;\n    }\n")
        return "".join(s)


_BINOPS = {"+": "plus", "-": "minus", "*": "multiply", "/": "divide", "<": "lessThan", "<=": "lessThanEquals",
           ">": "greaterThan", ">=": "greaterThanEquals", "==": "equals", "!=": "notEquals", "^": "pow", "%": "mod",
           "%%": "mod", "&": "and", "&&": "and", "|": "or", "||": "or", "intDiv": "intDiv",
           "strDistance": "strDistance"}


class H2OBinaryOp(H2OColOp):
    """A binary operator between a column and a constant or a second column (H2OBinaryOp.java)."""

    def __init__(self, name, ast, inplace, new_names):
        self.left_is_col = self.right_is_col = False
        self.bin_col = None
        super().__init__(name, ast, inplace, new_names)

    def _param(self, name, a):
        # H2OBinaryOp.setupParamsImpl: a column operand marks its side and names the column the POJO reads per row
        if a[0] == "call":
            if self.fun not in _BINOPS:
                raise NotImplementedError(f"unimpl: {self._lookup()}")
            if name in ("leftArg", "ary_x"):
                self.left_is_col = True
            elif name in ("rightArg", "ary_y"):
                self.right_is_col = True
            self.bin_col = _old_col(a)
            self.params[name] = self.bin_col
        else:
            super()._param(name, a)

    def _lookup(self):
        return _BINOPS.get(self.fun, self.fun)

    def _row_param(self):
        if not (self.left_is_col or self.right_is_col):
            return ""
        k = "rightArg" if self.right_is_col else "leftArg"
        return (f'      _params.put("{k}", new String[]{{String.valueOf(row.get("{self.bin_col}"))}}); '
                "// write over the previous value\n")


class H2OScaler(Transform):
    """Center and scale every column by its fitted mean / sd (H2OScaler.java); no POJO form, as in the reference."""

    def fit(self, fr):
        from .parallel import collectives as coll
        self.means, self.sdevs = [], []
        for n in fr.names:
            x = fr._col(n).as_float()
            ok = ~x.isnan()
            v = coll.all_reduce_np([float(x[ok].sum()), float((x[ok] ** 2).sum()), float(ok.sum())]) \
                if fr._shard is not None else [float(x[ok].sum()), float((x[ok] ** 2).sum()), float(ok.sum())]
            mu = v[0] / max(v[2], 1.0)
            self.means.append(mu)
            self.sdevs.append(((v[1] - v[2] * mu * mu) / max(v[2] - 1.0, 1.0)) ** 0.5)
        return self

    def _transform(self, fr):
        return fr.scale(self.means, self.sdevs)


_CLASSES = {c.__name__: c for c in (H2OColSelect, H2OColOp, H2OBinaryOp, H2OScaler)}

# argument names of common Rapids primitives (their AstPrimitive.args()), the keys of a step's POJO _params
_ARGS = {"countmatches": ["ary", "pattern"], "replaceall": ["ary", "pattern", "replacement", "ignore_case"],
         "replacefirst": ["ary", "pattern", "replacement", "ignore_case"], "strsplit": ["ary", "split"],
         "substring": ["ary", "startIndex", "endIndex"], "lstrip": ["ary", "set"], "rstrip": ["ary", "set"],
         "grep": ["ary", "regex", "ignore_case", "invert", "output_logical"], "num_valid_substrings": ["ary", "words"],
         "strDistance": ["ary_x", "ary_y", "measure", "compare_empty"], "round": ["ary", "digits"],
         "signif": ["ary", "digits"], "cut": ["ary", "breaks", "labels", "include.lowest", "right", "digits"]}


def _arg_name(fun, i):
    if fun in _BINOPS and fun != "strDistance":
        return ("leftArg", "rightArg")[i] if i < 2 else f"arg{i}"
    names = _ARGS.get(fun, ["ary"])
    return names[i] if i < len(names) else f"arg{i}"


def _uniquify(fr, name):
    """Frame.uniquify: ``name`` if free, else name0, name1, ..."""
    base = name or "C"
    if base not in fr.names:
        return base
    for i in itertools.count():
        if f"{base}{i}" not in fr.names:
            return f"{base}{i}"


def _copy(fr: H2OFrame, frame_id=None) -> H2OFrame:
    from .parallel import dframe
    with dframe.shard_ctx(fr._shard):
        return H2OFrame._from_columns([c.copy() for c in fr._cols.values()], frame_id)


def _renamed(fr: H2OFrame, name) -> H2OFrame:
    """The first column of ``fr`` as a one-column frame named ``name``."""
    from .frame import Column
    from .parallel import dframe
    c = fr._col(0)
    with dframe.shard_ctx(fr._shard):
        return H2OFrame._from_columns([Column(name, c.type, c.data, c.domain, c.strings)])


class Assembly:
    """A keyed pipeline of transforms (Assembly.java)."""

    def __init__(self, steps, key=None):
        self.steps = list(steps)
        self.key = key or f"assembly_{uuid.uuid4().hex}"

    @staticmethod
    def from_rest(step_strings) -> "Assembly":
        """AssemblyHandler.fit: ``name__Class__ast__inplace__names`` per step."""
        steps = []
        for st in step_strings:
            s = st.split("__")
            if len(s) != 5:
                raise ValueError(f"assembly step {st!r} is not of the form name__class__ast__inplace__names")
            cls = _CLASSES.get(s[1])
            if cls is None:
                raise ValueError(f"unknown assembly transform class {s[1]!r}")
            steps.append(cls(s[0], s[2], s[3].strip().lower() == "true", None if s[4] == "|" else s[4].split("|")))
        return Assembly(steps)

    def names(self):
        return [s.name for s in self.steps]

    def fit(self, fr: H2OFrame) -> H2OFrame:
        for step in self.steps:
            fr = step.fit_transform(fr)
        return fr

    def to_java(self, pojo_name: str | None = None) -> str:
        pojo_name = pojo_name or "GeneratedMungingPojo"
        s = ["import hex.genmodel.GenMunger;\n", "import hex.genmodel.easy.RowData;\n\n",
             f"public class {pojo_name} extends GenMunger {{\n", f"  public {pojo_name}() {{\n",
             f"    _steps = new Step[{len(self.steps)}];\n"]
        for i, st in enumerate(self.steps):
            s.append(f"    _steps[{i}] = new {st.name}();\n")
        s.append("  }\n")
        for st in self.steps:
            s.append(st.gen_class())
        s.append("}\n")
        return "".join(s)


def fit_rest(step_strings, frame: H2OFrame):
    """POST /99/Assembly: build, fit and register the assembly; returns (assembly, result frame)."""
    asm = Assembly.from_rest(step_strings)
    out = asm.fit(frame)
    out = _copy(out, f"{asm.key}_result")
    dkv.put(asm.key, asm)
    return asm, out

