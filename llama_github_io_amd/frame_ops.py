"""Frame-level operations beyond the H2OFrame methods (reference: ``water/rapids/ast/prims/mungers/
AstGroup.java``, ``hex/Interaction.java``, ``hex/CreateFrame.java``, ``hex/SplitFrame.java``,
``water/util/FrameUtils.java`` MissingInserter, ``hex/tfidf/TfIdfPreprocessor.java``).

Group-by runs on device: the group key of every row is a dense integer id (``torch.unique`` over the
stacked key codes), and every aggregate is one ``index_add_`` / ``scatter_reduce_`` over that id.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .frame import Column, H2OFrame, engine_device
from .ops.segment import segment_sum

_NA_MODES = ("all", "ignore", "rm")


class GroupBy:
    """``h2o.group_by.GroupBy``: chain aggregates then ``get_frame()``."""

    def __init__(self, fr: H2OFrame, by):
        self.fr = fr
        self.by = fr._resolve(by if isinstance(by, (list, tuple)) else [by])
        keys = []
        for n in self.by:
            c = fr._col(n)
            v = c.as_float().to(engine_device())
            keys.append(torch.nan_to_num(v, nan=float("-inf")))
        K = torch.stack(keys, 1)
        uniq, inv = torch.unique(K, dim=0, return_inverse=True)
        self.uniq = uniq
        self.gid = inv
        self.G = uniq.shape[0]
        self.aggs = []

    def _add(self, op, col, na):
        cols = self.fr._resolve(col) if col is not None else [n for n in self.fr.names if n not in self.by]
        for c in cols:
            self.aggs.append((op, c, na))
        return self

    def count(self, na="all"): self.aggs.append(("nrow", None, na)); return self  # noqa: E702
    def sum(self, col=None, na="all"): return self._add("sum", col, na)
    def mean(self, col=None, na="all"): return self._add("mean", col, na)
    def min(self, col=None, na="all"): return self._add("min", col, na)
    def max(self, col=None, na="all"): return self._add("max", col, na)
    def sd(self, col=None, na="all"): return self._add("sdev", col, na)
    def var(self, col=None, na="all"): return self._add("var", col, na)
    def ss(self, col=None, na="all"): return self._add("sumSquares", col, na)
    def median(self, col=None, na="all"): return self._add("median", col, na)
    def mode(self, col=None, na="all"): return self._add("mode", col, na)

    def _agg(self, op, name, na):
        G, gid = self.G, self.gid
        dev = gid.device
        if op == "nrow":
            return segment_sum(gid, torch.ones_like(gid, dtype=torch.float64), G)
        v = self.fr._col(name).as_float().to(dev)
        nan = torch.isnan(v)
        ok = ~nan
        vz = torch.where(ok, v, torch.zeros_like(v))
        cnt = segment_sum(gid, ok.double(), G)
        anynan = segment_sum(gid, nan.double(), G) > 0
        if op == "sum":
            r = segment_sum(gid, vz, G)
        elif op == "sumSquares":
            r = segment_sum(gid, vz * vz, G)
        elif op in ("mean", "var", "sdev"):
            s = segment_sum(gid, vz, G)
            m = s / cnt
            if op == "mean":
                r = m
            else:
                d = torch.where(ok, v - m[gid], torch.zeros_like(v))
                ss = segment_sum(gid, d * d, G)
                r = ss / (cnt - 1)
                if op == "sdev":
                    r = r.sqrt()
        elif op in ("min", "max"):
            fill = float("inf") if op == "min" else float("-inf")
            r = torch.full((G,), fill, dtype=torch.float64, device=dev).scatter_reduce_(
                0, gid, torch.where(ok, v, torch.full_like(v, fill)), reduce="amin" if op == "min" else "amax")
        elif op == "median":
            r = torch.full((G,), float("nan"), dtype=torch.float64, device=dev)
            g_np, v_np = gid.cpu().numpy(), v.cpu().numpy()
            for g in range(G):
                x = v_np[(g_np == g) & ~np.isnan(v_np)]
                if x.size:
                    r[g] = float(np.median(x))
        elif op == "mode":
            r = torch.full((G,), float("nan"), dtype=torch.float64, device=dev)
            g_np, v_np = gid.cpu().numpy(), v.cpu().numpy()
            for g in range(G):
                x = v_np[(g_np == g) & ~np.isnan(v_np)]
                if x.size:
                    u, c = np.unique(x, return_counts=True)
                    r[g] = float(u[np.argmax(c)])
        else:
            raise ValueError(op)
        if na == "all" and op not in ("nrow",):
            r = torch.where(anynan, torch.full_like(r, float("nan")), r)
        return r

    def get_frame(self) -> H2OFrame:
        cols = []
        for j, n in enumerate(self.by):
            src = self.fr._col(n)
            v = self.uniq[:, j]
            v = torch.where(torch.isinf(v) & (v < 0), torch.full_like(v, float("nan")), v)
            if src.type == "enum":
                codes = torch.where(torch.isnan(v), torch.full_like(v, -1), v).to(torch.int32)
                cols.append(Column(n, "enum", codes, list(src.domain)))
            else:
                cols.append(Column(n, src.type if src.type != "string" else "real", v))
        if not self.aggs:
            self.count()
        for op, name, na in self.aggs:
            r = self._agg(op, name, na)
            cname = "nrow" if op == "nrow" else f"{op}_{name}"
            cols.append(Column(cname, "real", r))
        return H2OFrame._from_columns(cols)

    @property
    def frame(self):
        return self.get_frame()


# ------------------------------------------------------------------------------------------------
def interaction(fr: H2OFrame, factors, pairwise=False, max_factors=100, min_occurrence=1) -> H2OFrame:
    """``hex/Interaction.java``: categorical interaction columns ``a_b`` with levels ``la_lb``; levels
    are kept by frequency (top ``max_factors``, at least ``min_occurrence``), the rest -> "other"."""
    names = fr._resolve(factors)
    groups = [[a, b] for i, a in enumerate(names) for b in names[i + 1:]] if pairwise else [names]
    out = []
    for grp in groups:
        strs = None
        for n in grp:
            v = fr._col(n).to_numpy()
            s = np.array(["NA" if x is None or (isinstance(x, float) and math.isnan(x)) else str(x) for x in v], dtype=object)
            strs = s if strs is None else np.char.add(np.char.add(strs.astype(str), "_"), s.astype(str)).astype(object)
        u, c = np.unique(strs.astype(str), return_counts=True)
        order = np.argsort(-c, kind="stable")
        keep = [u[i] for i in order if c[i] >= min_occurrence][: int(max_factors)]
        keep_set = set(keep)
        lab = np.array([x if x in keep_set else "other" for x in strs.astype(str)], dtype=object)
        dom = sorted(set(lab.tolist()))
        lut = {s: i for i, s in enumerate(dom)}
        codes = torch.as_tensor(np.array([lut[s] for s in lab], dtype=np.int32), device=engine_device())
        out.append(Column("_".join(grp), "enum", codes, dom))
    return H2OFrame._from_columns(out)


# ------------------------------------------------------------------------------------------------
def create_frame(rows=10000, cols=10, randomize=True, value=0, real_range=100, categorical_fraction=0.2,
                 factors=100, integer_fraction=0.2, integer_range=100, binary_fraction=0.1, binary_ones_fraction=0.02,
                 time_fraction=0.0, string_fraction=0.0, missing_fraction=0.01, has_response=False,
                 response_factors=2, positive_response=False, seed=None, seed_for_column_types=None,
                 frame_id=None) -> H2OFrame:
    """``hex/CreateFrame.java``: random frame with the requested column-type mix, generated on device."""
    dev = engine_device()
    rng = np.random.default_rng(None if seed in (None, -1) else int(seed))
    trng = np.random.default_rng(None if seed_for_column_types in (None, -1) else int(seed_for_column_types)) \
        if seed_for_column_types not in (None, -1) else rng
    g = torch.Generator(device="cpu").manual_seed(int(rng.integers(1 << 62)))
    fracs = dict(cat=categorical_fraction, int=integer_fraction, bin=binary_fraction, time=time_fraction,
                 str=string_fraction)
    kinds = []
    for k, f in fracs.items():
        kinds += [k] * int(round(f * cols))
    kinds = (kinds + ["real"] * cols)[:cols]
    kinds = list(trng.permutation(kinds))
    out = []
    if has_response:
        if response_factors > 1:
            codes = torch.randint(0, response_factors, (rows,), generator=g).to(torch.int32)
            out.append(Column("response", "enum", codes.to(dev), [str(i) for i in range(response_factors)]))
        else:
            v = torch.rand(rows, generator=g, dtype=torch.float64) * real_range
            if not positive_response:
                v = v * 2 - real_range
            out.append(Column("response", "real", v.to(dev)))
    for j, k in enumerate(kinds):
        name = f"C{j + 1}"
        if not randomize:
            out.append(Column(name, "real", torch.full((rows,), float(value), dtype=torch.float64, device=dev)))
            continue
        if k == "cat":
            codes = torch.randint(0, factors, (rows,), generator=g).to(torch.int32)
            col = Column(name, "enum", codes, [f"c{j}.l{i}" for i in range(factors)])
        elif k == "int":
            col = Column(name, "int", torch.randint(-integer_range, integer_range + 1, (rows,), generator=g).double())
        elif k == "bin":
            col = Column(name, "int", (torch.rand(rows, generator=g) < binary_ones_fraction).double())
        elif k == "time":
            col = Column(name, "time", (torch.rand(rows, generator=g, dtype=torch.float64) * 1.6e12).floor())
        elif k == "str":
            col = Column(name, "string", strings=np.array([f"s{int(x)}" for x in torch.randint(0, 1 << 30, (rows,), generator=g)], dtype=object))
        else:
            col = Column(name, "real", (torch.rand(rows, generator=g, dtype=torch.float64) * 2 - 1) * real_range)
        if missing_fraction > 0:
            m = torch.rand(rows, generator=g) < missing_fraction
            if col.type == "enum":
                col.data[m] = -1
            elif col.type == "string":
                col.strings[m.numpy()] = None
            else:
                col.data[m] = float("nan")
        if col.data is not None:
            col.data = col.data.to(dev)
        out.append(col)
    return H2OFrame._from_columns(out, frame_id)


def insert_missing_values(fr: H2OFrame, fraction=0.1, seed=None) -> H2OFrame:
    """``MissingInserter``: set each cell to NA with probability ``fraction`` (in place, like H2O)."""
    g = torch.Generator(device="cpu").manual_seed(int(seed) if seed not in (None, -1) else np.random.randint(1 << 30))
    for n in fr.names:
        c = fr._col(n)
        m = torch.rand(fr.nrows, generator=g) < fraction
        if c.type == "enum":
            c.data[m.to(c.data.device)] = -1
        elif c.type == "string":
            c.strings[m.numpy()] = None
        else:
            c.data[m.to(c.data.device)] = float("nan")
    return fr


def tf_idf(fr: H2OFrame, document_id_col=0, text_col=1, preprocess=True, case_sensitive=True) -> H2OFrame:
    """``TfIdfPreprocessor`` + ``TermFrequency/InverseDocumentFrequency``: (doc, word, tf, idf, tf_idf)."""
    ids = fr._col(document_id_col).to_numpy()
    texts = fr._col(text_col).to_numpy()
    rows = []
    for d, t in zip(ids, texts):
        if t is None:
            continue
        s = str(t) if case_sensitive else str(t).lower()
        words = s.split() if preprocess else [s]
        for w in words:
            rows.append((d, w))
    import collections
    tf = collections.Counter(rows)
    ndocs = len(set(ids.tolist()))
    df = collections.Counter(w for (_, w) in tf.keys())
    docs, words, tfs, idfs, tfidf = [], [], [], [], []
    for (d, w), c in sorted(tf.items(), key=lambda kv: (str(kv[0][0]), kv[0][1])):
        idf = math.log((ndocs + 1) / (df[w] + 1))
        docs.append(d); words.append(w); tfs.append(c); idfs.append(idf); tfidf.append(c * idf)
    return H2OFrame({"DocID": docs, "Word": np.array(words, dtype=object), "TF": tfs, "IDF": idfs, "TF-IDF": tfidf},
                    column_types={"Word": "string"})
