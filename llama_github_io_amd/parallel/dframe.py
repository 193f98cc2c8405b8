"""Row-sharded frames: the distributed data plane (reference: ``water/fvec/Frame.java`` /
``Vec.java`` (a Vec's chunks are spread over the cloud, ``Vec.espc`` = the element-start of each
chunk), ``water/MRTask.java`` (map over the local chunks, reduce the results up a tree) and
``water/parser/ParseDataset.java`` (each node parses its own byte ranges, then the categorical
domains are unified cluster-wide)).

MI355X design: one process per GPU; a sharded :class:`~llama_github_io_amd.frame.H2OFrame` keeps
only its rank's contiguous row range in that GPU's HBM and carries a :class:`Shard` record
``(offset, n_local, n_global)`` — the one-chunk-per-node form of ``espc``. Invariants:

* every rank holds the same columns, types and (for categoricals) the SAME domain, so a level code
  means the same thing everywhere and per-rank histograms / Grams can be summed;
* rows are split in rank order: global row ``offset + i`` is local row ``i``.

Frame methods fall in three classes (installed by :func:`install` on ``H2OFrame``):

* **row-local** (element-wise math, comparisons, column selection, masks, string/time maps,
  ``cbind``, ``model_matrix``): run on the shard, no communication, the result carries the same
  shard (a mask filter re-derives its offsets with one tiny all-gather);
* **collective reductions** (``nrow``, ``mean``/``sum``/``min``/``max``/``sd``/``var``/``nacnt``,
  ``asfactor`` domain union, ``impute``/``scale`` statistics, ``head``): an all-reduce / all-gather
  of per-rank partials — the MRTask map/reduce;
* **global re-orderings** (``sort``, ``merge``, ``group_by``, cumulative ops, ``pivot``/``melt``, …):
  gather the shards (all-gather over RCCL/xGMI), run on the full rows, return a replicated frame.

A replicated frame is a valid frame everywhere (every rank holds all rows); trainers shard or
gather their inputs as they need (``models/builder.py``).
"""
from __future__ import annotations

import contextlib
import functools
import threading
from dataclasses import dataclass

import numpy as np
import torch

from . import collectives as coll

_tls = threading.local()


@dataclass(frozen=True)
class Shard:
    offset: int        # global index of this rank's first row
    n_local: int
    n_global: int


def current_ctx():
    """Shard that frames built by ``_from_columns`` right now belong to (None = replicated)."""
    return getattr(_tls, "shard", None)


@contextlib.contextmanager
def shard_ctx(shard):
    prev = getattr(_tls, "shard", None)
    _tls.shard = shard
    try:
        yield
    finally:
        _tls.shard = prev


def in_method() -> bool:
    return getattr(_tls, "depth", 0) > 0


@contextlib.contextmanager
def _method():
    _tls.depth = getattr(_tls, "depth", 0) + 1
    try:
        yield
    finally:
        _tls.depth -= 1


def active() -> bool:
    """A multi-rank cloud exists: user-built frames are sharded."""
    return coll.world_active()


def bounds(n_global: int, rank: int | None = None, world: int | None = None) -> tuple:
    r = coll.rank() if rank is None else rank
    w = coll.world() if world is None else world
    return r * n_global // w, (r + 1) * n_global // w


def make_shard(n_local: int) -> Shard:
    off, tot = coll.exclusive_offset(n_local)
    return Shard(off, int(n_local), tot)


# ------------------------------------------------------------------------------------------------
# shard <-> replicate
def shard_columns(cols, n_global: int):
    """Replicated columns -> this rank's contiguous slice (no communication)."""
    from ..frame import Column
    lo, hi = bounds(n_global)
    out = []
    for c in cols:
        if c.type == "string":
            out.append(Column(c.name, c.type, strings=c.strings[lo:hi].copy(), domain=c.domain))
        else:
            out.append(Column(c.name, c.type, c.data[lo:hi].clone(), c.domain))
    return out, Shard(lo, hi - lo, n_global)


def shard_frame(fr):
    """Replicated frame -> sharded frame with the same frame id semantics (a new frame object)."""
    if fr._shard is not None or not active():
        return fr
    from ..frame import H2OFrame
    cols, sh = shard_columns(list(fr._cols.values()), fr._nlocal)
    with shard_ctx(sh):
        out = H2OFrame._from_columns(cols)
    return out


def gather_column(c):
    from ..frame import Column
    if c.type == "string":
        parts = coll.all_gather_object(list(c.strings))
        return Column(c.name, c.type, strings=np.array([s for p in parts for s in p], dtype=object), domain=c.domain)
    t = c.data
    if t.is_cuda and coll.comm_device().type != "cuda":
        full = coll.all_gather_cat(t.cpu(), 0, force=True).to(t.device)
    else:
        full = coll.all_gather_cat(t, 0, force=True)
    return Column(c.name, c.type, full, c.domain)


def gather_frame(fr):
    """Sharded frame -> replicated frame holding every row on every rank (rank order)."""
    if fr is None or getattr(fr, "_shard", None) is None:
        return fr
    from ..frame import H2OFrame
    with shard_ctx(None):
        return H2OFrame._from_columns([gather_column(c) for c in fr._cols.values()])


def gather_tensor(t: torch.Tensor, dim: int = 0, bounded: bool = False) -> torch.Tensor:
    """Concatenate every rank's ``t``; ``bounded``: t is a per-rank summary whose size does not grow with
    the rows (distinct codes, a fixed-size sample)."""
    return coll.all_gather_cat(t.contiguous(), dim, force=True, bounded=bounded)


# ------------------------------------------------------------------------------------------------
# categorical domains: every rank must agree (ParseDataset's domain unification)
def unify_domain(codes: torch.Tensor, local_domain, sort_key=None) -> tuple:
    """Remap local level codes to the sorted union of all ranks' domains. Returns (codes, domain)."""
    if not active():
        return codes, list(local_domain)
    doms = coll.all_gather_object(list(local_domain))
    glob = sorted(set().union(*[set(d) for d in doms]), key=sort_key)
    if all(list(d) == glob for d in doms):
        return codes, glob
    lut = {s: i for i, s in enumerate(glob)}
    m = torch.tensor([lut[s] for s in local_domain] + [-1], dtype=torch.int32, device=codes.device)
    idx = torch.where(codes < 0, torch.full_like(codes, len(local_domain)), codes).long()
    return m[idx], glob


def global_unique(v: torch.Tensor) -> torch.Tensor:
    """Sorted unique values of a sharded numeric vector (NaN dropped)."""
    u = torch.unique(v[~torch.isnan(v)])
    if not active():
        return u
    return torch.unique(gather_tensor(u.cpu() if coll.comm_device().type == "cpu" else u).to(v.device))


# ------------------------------------------------------------------------------------------------
# reductions (MRTask map -> reduce)
def moments(v: torch.Tensor, sharded: bool) -> dict:
    """Exact global count / sum / min / max / centred second moment of a numeric vector (NaN skipped):
    per-rank partials combined with the parallel-variance merge (Chan et al.), as RollupStats does."""
    ok = ~torch.isnan(v)
    x = v[ok].double()
    n = float(x.numel())
    s = float(x.sum()) if n else 0.0
    mn = float(x.min()) if n else float("inf")
    mx = float(x.max()) if n else float("-inf")
    m2 = float(((x - s / n) ** 2).sum()) if n else 0.0
    nz = float((x == 0).sum())
    nas = float((~ok).sum())
    if sharded and active():
        parts = coll.all_gather_object((n, s, mn, mx, m2, nz, nas))
        N = sum(p[0] for p in parts)
        S = sum(p[1] for p in parts)
        mean = S / N if N else float("nan")
        M2 = sum(p[4] + (p[0] * (p[1] / p[0] - mean) ** 2 if p[0] else 0.0) for p in parts)
        return dict(n=N, sum=S, min=min(p[2] for p in parts), max=max(p[3] for p in parts), m2=M2,
                    zeros=sum(p[5] for p in parts), nas=sum(p[6] for p in parts), mean=mean)
    return dict(n=n, sum=s, min=mn, max=mx, m2=m2, zeros=nz, nas=nas, mean=s / n if n else float("nan"))


# ------------------------------------------------------------------------------------------------
# method wrappers
def _frames_in(args, kwargs):
    from ..frame import H2OFrame
    out = [a for a in args if isinstance(a, H2OFrame)]
    out += [v for v in kwargs.values() if isinstance(v, H2OFrame)]
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, (list, tuple)):
            out += [x for x in a if isinstance(x, H2OFrame)]
    return out


def _map_frames(args, kwargs, f):
    from ..frame import H2OFrame

    def one(a):
        if isinstance(a, H2OFrame):
            return f(a)
        if isinstance(a, list):
            return [f(x) if isinstance(x, H2OFrame) else x for x in a]
        if isinstance(a, tuple):
            return tuple(f(x) if isinstance(x, H2OFrame) else x for x in a)
        return a
    return [one(a) for a in args], {k: one(v) for k, v in kwargs.items()}


def local_method(fn):
    """Row-local method: runs on the shard; frames it builds carry the shard of ``self``. Replicated
    operand frames of the same global length are sliced to the shard; operands sharded differently
    (e.g. after different filters) fall back to the gathered path."""
    @functools.wraps(fn)
    def w(self, *args, **kwargs):
        others = _frames_in(args, kwargs)
        sh = self._shard
        if sh is None and not any(o._shard is not None for o in others):
            with _method(), shard_ctx(None):
                return fn(self, *args, **kwargs)
        if sh is None:
            sh = next(o._shard for o in others if o._shard is not None)
            if self.nrows == sh.n_global and self.nrows > 1:
                self = shard_frame(self)
            else:
                return _gathered(fn, self, args, kwargs)
        ok = True

        def fix(o):
            nonlocal ok
            if o._shard == sh:
                return o
            if o._shard is None and o.nrows == sh.n_global and sh.n_global > 1:
                return shard_frame(o)
            if o._shard is None and o.nrows == 1:
                return o                         # 1-row operand broadcasts
            ok = False
            return o
        args, kwargs = _map_frames(args, kwargs, fix)
        if not ok:
            return _gathered(fn, self, args, kwargs)
        with _method(), shard_ctx(sh):
            return fn(self, *args, **kwargs)
    w._dist_kind = "local"
    return w


def _gathered(fn, self, args, kwargs):
    g = gather_frame
    args, kwargs = _map_frames(args, kwargs, g)
    with _method(), shard_ctx(None), coll.replicated():
        return fn(g(self), *args, **kwargs)


def gathered_method(fn):
    """Global re-ordering: gather the shards, compute on every row, return a replicated result."""
    @functools.wraps(fn)
    def w(self, *args, **kwargs):
        if self._shard is None and not any(o._shard is not None for o in _frames_in(args, kwargs)):
            with _method(), shard_ctx(None):
                return fn(self, *args, **kwargs)
        return _gathered(fn, self, args, kwargs)
    w._dist_kind = "gather"
    return w


def plain_method(fn):
    """Method with its own collective logic (or none needed): only marks internal construction."""
    @functools.wraps(fn)
    def w(self, *args, **kwargs):
        with _method(), shard_ctx(None):
            return fn(self, *args, **kwargs)
    w._dist_kind = "plain"
    return w


LOCAL = {
    "_binop", "_unop", "_cmp", "ifelse", "isna", "asnumeric", "ascharacter", "_str_map", "nchar", "countmatches",
    "entropy", "_time", "year", "month", "day", "hour", "minute", "second", "week", "dayOfWeek", "as_date", "cbind",
    "cut", "relevel", "set_levels", "as_tensor", "model_matrix", "response_tensor", "weights_tensor",
    "__invert__", "__neg__", "__abs__", "log", "log10", "log2", "log1p", "exp", "expm1", "sqrt", "abs", "ceil", "floor",
    "trunc", "sign", "sin", "cos", "tan", "tanh", "round", "signif", "na_omit", "interaction_local",
}
# methods with their own collective / metadata logic, or which only touch column metadata
PLAIN = {
    "__init__", "_from_python", "_from_columns", "from_predictions", "from_tensor", "names", "columns", "col_names",
    "nrows", "nrow", "ncols", "ncol", "shape", "dim", "types", "dtypes", "type", "columns_by_type", "__len__", "_col",
    "_resolve", "set_names", "set_name", "rename", "__getitem__", "_rows", "__setitem__", "__delitem__", "drop", "pop",
    "__repr__", "show", "isfactor", "isnumeric", "isstring", "levels", "nlevels", "_num", "_reduce", "mean", "sum",
    "max", "min", "sd", "std", "var", "nacnt", "any", "all", "summary", "describe", "asfactor", "impute", "_impute_by", "scale",
    "split_frame", "runif", "kfold_column", "modulo_kfold_column", "head", "tail", "refresh", "key", "__iter__",
    "__contains__", "__hash__", "__eq__", "__ne__", "__lt__", "__le__", "__gt__", "__ge__", "__and__", "__or__",
    "__add__", "__radd__", "__sub__", "__rsub__", "__mul__", "__rmul__", "__truediv__", "__rtruediv__",
    "__floordiv__", "__mod__", "__pow__", "__rpow__", "_nlocal", "_shard", "is_sharded", "gather", "reshard",
    "as_data_frame", "get_frame_data", "flatten",
}


def install(cls):
    """Wrap every public method of ``cls`` (H2OFrame) by its distribution class; anything not listed
    as row-local or self-managed is treated as a global re-ordering (gathered)."""
    for name, v in list(vars(cls).items()):
        if isinstance(v, (property, staticmethod, classmethod)) or not callable(v):
            continue
        if name in PLAIN:
            if not name.startswith("__") or name in ("__getitem__", "__setitem__"):
                setattr(cls, name, plain_method(v))
            continue
        if name.startswith("__") and name not in LOCAL:
            continue
        setattr(cls, name, local_method(v) if name in LOCAL else gathered_method(v))
    return cls
