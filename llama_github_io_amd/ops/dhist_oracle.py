"""NumPy oracle of H2O's per-node adaptive histograms (the reference algorithm behind ``histogram_type=AUTO``).

The engine's tree kernels histogram PRE-BINNED columns: every numeric column is cut once into global quantile bins
(QuantilesGlobal exactly, the other types as candidate lattices over up to ~1016 global edges). The reference instead
re-bins every column of every node over the node's OWN value range:

* the root histogram of column ``j`` has ``nbins_top_level`` (1024) uniform bins over ``[min_j, maxEx_j)`` of the whole
  column (``DHistogram.initialHist``, ``DHistogram.java:474-497``; ``maxEx = max + ulp(max)``, or ``max + 1`` for
  integer columns, ``find_maxEx`` :454);
* a child's histogram of column ``j`` has ``max(parent_nbins >> 1, nbins)`` uniform bins over the range of the values
  the PARENT's histogram actually saw (``find_min`` / ``find_maxEx`` of the parent, which covers both children),
  narrowed at the split point for the split column (``DTree.java:337-411``);
* integer columns whose range fits the bin count get unit bins (``DHistogram.java:226-233``);
* ``bin(x) = (int)((x - min) * step)`` with ``step = nbins / (maxEx - min)`` (``:257-291``), and the split value of bin
  ``b`` is ``binAt(b) = min + b / step`` (``:293-297``): rows with ``x < splat`` go left.

Split search follows ``DTree.findBestSplitPoint`` (``DTree.java:984-1330``): cumulative (w, wY, wYY) sweeps,
``min_rows``, the relative ``min_split_improvement`` test against the node's squared error, ties towards the middle
bin, equal-prediction rejection; the best column is the smallest SE (``bestCol``, ``:616-656``). Leaves are GBM's
Newton steps (``GBM.fitBestConstants``). NAs and categoricals are not modelled (the comparison datasets have none).

:func:`train_gbm` grows a whole GBM with these histograms (``hist="uniform_adaptive"``) or with fixed global
quantile bins (``hist="quantiles_global"``), so ``scripts/dhist_report.py`` can compare the reference's split
decisions and model quality against the engine's lattice approximation.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


def find_max_ex(max_in: float, is_int: bool) -> float:
    ulp = math.ulp(max_in)
    if is_int and ulp < 1:
        ulp = 1.0
    r = max_in + ulp
    return max_in if math.isinf(r) else r


@dataclass
class Hist:
    """One node's histogram of one column (DHistogram)."""
    nbins: int
    lo: float            # _min
    max_ex: float        # _maxEx
    step: float
    is_int: bool
    w: np.ndarray = field(default=None)
    wy: np.ndarray = field(default=None)
    wyy: np.ndarray = field(default=None)
    min2: float = math.inf     # observed inclusive min of the node's values
    max_in: float = -math.inf  # observed inclusive max

    @staticmethod
    def make(nbins: int, lo: float, max_ex: float, is_int: bool) -> "Hist | None":
        if not (lo < max_ex) or nbins < 1:
            return None
        xb = nbins
        if is_int and max_ex - lo <= xb:
            xb = int(max_ex) - int(lo)
            step = 1.0
        else:
            step = xb / (max_ex - lo)
            if step <= 0 or math.isinf(step) or math.isnan(step):
                return None
        return Hist(int(xb), float(lo), float(max_ex), float(step), bool(is_int))

    def bins_of(self, x: np.ndarray) -> np.ndarray:
        b = np.floor((x - self.lo) * self.step).astype(np.int64)
        return np.clip(b, 0, self.nbins - 1)     # (round-off can hit nbins; DHistogram.bin truncates)

    def fill(self, x: np.ndarray, r: np.ndarray):
        b = self.bins_of(x)
        self.w = np.bincount(b, minlength=self.nbins).astype(np.float64)
        self.wy = np.bincount(b, weights=r, minlength=self.nbins)
        self.wyy = np.bincount(b, weights=r * r, minlength=self.nbins)
        if x.size:
            self.min2 = float(x.min())
            self.max_in = float(x.max())

    def bin_at(self, b: int) -> float:
        return self.lo + b / self.step


def find_best_split(h: Hist, min_rows: float, msi: float):
    """(se, bin, nleft, nright, predl, predr) of DTree.findBestSplitPoint with no NAs, or None."""
    nb = h.nbins
    w, wy, wyy = h.w, h.wy, h.wyy
    wlo = np.concatenate([[0.0], np.cumsum(w)])
    wylo = np.concatenate([[0.0], np.cumsum(wy)])
    wyylo = np.concatenate([[0.0], np.cumsum(wyy)])
    tot = wlo[nb]
    if tot < 2 * min_rows:
        return None
    var = wyylo[nb] * tot - wylo[nb] * wylo[nb]
    if np.float32(var) == 0:
        return None
    whi = tot - wlo
    wyhi = wylo[nb] - wylo
    wyyhi = wyylo[nb] - wyylo
    se_before = max(0.0, wyyhi[0] - wyhi[0] * wyhi[0] / whi[0])
    best, best_se = 0, math.inf
    for b in range(1, nb):
        if w[b] == 0:
            continue
        if wlo[b] < min_rows:
            continue
        if whi[b] < min_rows:
            break
        selo = max(0.0, wyylo[b] - wylo[b] * wylo[b] / wlo[b])
        sehi = max(0.0, wyyhi[b] - wyhi[b] * wyhi[b] / whi[b])
        s = selo + sehi
        if s < best_se or (s == best_se and abs(b - (nb >> 1)) < abs(best - (nb >> 1))):
            best, best_se = b, s
    if best == 0:
        return None
    if not (best_se < se_before * (1 - msi)):
        return None
    nl, nr = wlo[best], whi[best]
    pl, pr = wylo[best], wyhi[best]
    if np.float32(pl / nl) == np.float32(pr / nr):
        return None
    if nl < min_rows or nr < min_rows:
        return None
    return best_se, best, nl, nr, pl, pr


@dataclass
class Node:
    rows: np.ndarray
    hists: list                # per column: Hist or None (the bins this node's split search uses)
    depth: int
    feat: int = -1
    splat: float = math.nan
    bin: int = -1
    left: "Node | None" = None
    right: "Node | None" = None
    value: float = 0.0


def _grow(X, r, hess, node: Node, D, min_rows, msi, nbins, hist_mode, qedges, splits_out):
    rows = node.rows
    F = X.shape[1]
    best = None
    for j in range(F):
        h = node.hists[j]
        if h is None:
            continue
        h.fill(X[rows, j], r[rows])
        if node.depth >= D:
            continue
        s = find_best_split(h, min_rows, msi)
        if s is not None and (best is None or s[0] < best[0]):
            best = (s[0], j, s[1])
    if node.depth >= D or best is None:
        node.value = float(r[rows].sum() / max(hess[rows].sum(), 1e-300)) if hess[rows].sum() > 0 else 0.0
        return
    _, j, b = best
    h = node.hists[j]
    splat = h.bin_at(b)
    node.feat, node.bin, node.splat = j, b, splat
    splits_out.append((node.depth, j, splat))
    xs = X[rows, j]
    lmask = xs < splat
    kids = []
    for way, sub in ((0, rows[lmask]), (1, rows[~lmask])):
        hs = []
        for c in range(F):
            ph = node.hists[c]
            if ph is None:
                hs.append(None)
                continue
            adj = max(ph.nbins >> 1, nbins)
            lo = ph.min2
            if ph.max_in == lo:
                hs.append(None)            # this column will not split again in this node
                continue
            mx = find_max_ex(ph.max_in, ph.is_int)
            if c == j:
                sp = math.ceil(splat) if ph.is_int else splat
                if way == 0:
                    mx = sp
                else:
                    lo = sp
            if lo >= mx:
                hs.append(None)
                continue
            if ph.is_int and not (lo + 1 < mx):
                hs.append(None)
                continue
            hs.append(Hist.make(adj, lo, mx, ph.is_int))
        kids.append(Node(sub, hs, node.depth + 1))
    node.left, node.right = kids
    for k in kids:
        _grow(X, r, hess, k, D, min_rows, msi, nbins, hist_mode, qedges, splits_out)


def _root_hists(X, nbins_top, hist_mode, q_nbins=255):
    F = X.shape[1]
    hs = []
    for j in range(F):
        x = X[:, j]
        lo, hi = float(x.min()), float(x.max())
        is_int = bool(np.all(np.floor(x) == x))
        if lo == hi:
            hs.append(None)
            continue
        if hist_mode == "quantiles_global":
            hs.append(QHist.make(x, q_nbins))
        else:
            hs.append(Hist.make(nbins_top, lo, find_max_ex(hi, is_int), is_int))
    return hs


class QHist(Hist):
    """Global quantile bins (QuantilesGlobal): bin = #edges <= x, split value = the edge."""

    @staticmethod
    def make(x, nb):
        qs = np.unique(np.quantile(x, np.linspace(0, 1, nb + 1)[1:-1]))
        h = QHist(len(qs) + 1, float(x.min()), float(x.max()), 1.0, False)
        h.edges = qs
        return h

    def bins_of(self, x):
        return np.searchsorted(self.edges, x, side="right")

    def bin_at(self, b):
        return float(self.edges[b - 1])


def _copy_q(ph):
    h = QHist(ph.nbins, ph.lo, ph.max_ex, 1.0, False)
    h.edges = ph.edges
    return h


def _predict(node: Node, X):
    out = np.zeros(X.shape[0])
    stack = [(node, np.arange(X.shape[0]))]
    while stack:
        n, idx = stack.pop()
        if n.left is None:
            out[idx] = n.value
            continue
        m = X[idx, n.feat] < n.splat
        stack.append((n.left, idx[m]))
        stack.append((n.right, idx[~m]))
    return out


def train_gbm(X, y, ntrees=50, max_depth=5, min_rows=10.0, learn_rate=0.1, nbins=20, nbins_top_level=1024,
              min_split_improvement=1e-5, distribution="bernoulli", hist="uniform_adaptive"):
    """GBM with the reference's histograms. Returns (f0, trees, per-tree split lists); trees are Node roots whose
    leaf values include the learning rate."""
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    N = X.shape[0]
    if distribution == "bernoulli":
        m = y.mean()
        f0 = math.log(m / (1 - m))
    else:
        f0 = float(y.mean())
    f = np.full(N, f0)
    trees, splits = [], []
    root_q = _root_hists(X, nbins_top_level, hist) if hist == "quantiles_global" else None
    for _ in range(ntrees):
        if distribution == "bernoulli":
            p = 1 / (1 + np.exp(-f))
            r = y - p
            hess = p * (1 - p)
        else:
            r = y - f
            hess = np.ones(N)
        if hist == "quantiles_global":
            hs = [None if h is None else _copy_q(h) for h in root_q]
        else:
            hs = _root_hists(X, nbins_top_level, hist)
        root = Node(np.arange(N), hs, 0)
        sp = []
        _grow_q = _grow if hist != "quantiles_global" else _grow_quantiles
        _grow_q(X, r, hess, root, max_depth, min_rows, min_split_improvement, nbins, hist, None, sp)
        _scale(root, learn_rate)
        f = f + _predict(root, X)
        trees.append(root)
        splits.append(sp)
    return f0, trees, splits


def _grow_quantiles(X, r, hess, node, D, min_rows, msi, nbins, hist_mode, qedges, splits_out):
    rows = node.rows
    best = None
    for j, h in enumerate(node.hists):
        if h is None:
            continue
        h.fill(X[rows, j], r[rows])
        if node.depth >= D:
            continue
        s = find_best_split(h, min_rows, msi)
        if s is not None and (best is None or s[0] < best[0]):
            best = (s[0], j, s[1])
    if node.depth >= D or best is None:
        node.value = float(r[rows].sum() / hess[rows].sum()) if hess[rows].sum() > 0 else 0.0
        return
    _, j, b = best
    splat = node.hists[j].bin_at(b)
    node.feat, node.bin, node.splat = j, b, splat
    splits_out.append((node.depth, j, splat))
    lmask = X[rows, j] < splat
    kids = [Node(sub, [None if h is None else _copy_q(h) for h in node.hists], node.depth + 1)
            for sub in (rows[lmask], rows[~lmask])]
    node.left, node.right = kids
    for k in kids:
        _grow_quantiles(X, r, hess, k, D, min_rows, msi, nbins, hist_mode, qedges, splits_out)


def _scale(node, lr):
    if node.left is None:
        node.value *= lr
        return
    _scale(node.left, lr)
    _scale(node.right, lr)


def predict(model, X):
    f0, trees, _ = model
    X = np.asarray(X, dtype=np.float64)
    f = np.full(X.shape[0], f0)
    for t in trees:
        f += _predict(t, X)
    return f
