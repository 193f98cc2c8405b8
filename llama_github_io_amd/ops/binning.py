"""Global feature binning for the histogram tree engine (H2O ``histogram_type = QuantilesGlobal``).

Reference: ``hex/tree/GlobalQuantilesCalc.java`` (global quantile split points) and
``hex/tree/DHistogram.java`` (bin(), NA bin). Each numeric column gets at most 255 data bins whose
edges are exact sample values: ``bin(x) = #{edges <= x}``, so a split "bins < b go left" is the
threshold rule ``x < edges[b-1]`` on raw values. Categorical columns use their level codes as bins
(levels beyond 254 are folded by frequency into one shared bin). NaN -> NA bin 255.

Wide numeric bins (``max_bins`` up to 1016, e.g. UniformAdaptive's ``nbins_top_level = 1024``,
``SharedTreeModel.java:57``): a feature with more than 254 edges e is binned as n = ceil(|e| / 254) adjacent
ENGINE columns, column k holding the byte bin of the edge subset e[k::n]. With fine bin t = #{e <= x} = 4h + l
(n = 4), column k's bin is #{e[k::4] <= x} = h + [l > k], and its split "bin < h'" is exactly the fine split
"t <= 4(h' - 1) + k": the n columns together offer every threshold of the fine edges, their histograms are
exact, and the uint8 engine (histograms, routing, leaf walk) runs unchanged. ``vmap`` maps engine columns to
the original features (split decoding, column sampling, constraints, importances).

Wide categoricals (``nbins_cats`` up to 1016 levels kept apart, H2O default 1024, ``SharedTreeModel.java:72``):
a categorical with L > 254 bins spans n = ceil(L / 254) engine columns; column k holds the levels of bins
[254k, 254k + L_k) as bins 0..L_k-1 and every other level in one "elsewhere" bin L_k (NA stays bin 255). No
level is folded. The n columns form a GROUP at a 4-aligned engine position, padded to 4 with constant columns
(``cat_groups``, ``pad``), so a row's group bytes are one aligned 32-bit word of its bins: the split search
merges the group's histograms into one histogram over all L levels and sorts ALL of them by mean response
(H2O's single sort, DTree.java:1004-1013), and the group decision (a bitset over the L bins) routes a row from
that word (the one column whose byte is not 'elsewhere' names the row's level). The byte histograms stay
exact. Decoding maps the bitset back through ``level_to_bin`` to a bitset over the original levels.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as nat
from .tree import MAX_DATA_BINS, NA_BIN

SUB_EDGES = MAX_DATA_BINS - 1            # edges one engine column holds (254)
WIDE_MAX_BINS = 4 * SUB_EDGES            # data bins of a wide numeric feature (1016 = 4 engine columns)


@dataclass
class Binning:
    F: int
    stride: int
    edges: list                     # per feature: float32 np.ndarray (numeric) or None (categorical)
    nbins: np.ndarray               # int32 [F] data bins per feature
    iscat: np.ndarray               # int32 [F]
    nlevels: np.ndarray             # int32 [F] categorical cardinality (0 numeric)
    level_to_bin: list = field(default_factory=list)  # per feature: int array (None = identity)
    vmap: np.ndarray | None = None  # int32 [F] engine column -> original feature (None: identity)
    n_low: int = 0                  # engine columns [0, n_low) = every feature's first column (narrow view), 0: none
    n_mid: int = 0                  # [0, n_mid): + the subsets halving the edge spacing (512-bin levels), 0: none
    cat_groups: list = field(default_factory=list)   # wide categoricals: (first engine column, real columns)
    pad: np.ndarray | None = None   # bool [F]: constant padding column of a wide-categorical group (bin 0)

    # every per-feature field above is per ENGINE column (F of them); see the module note on wide bins
    @property
    def F_orig(self) -> int:
        return self.F if self.vmap is None else int(self.vmap.max()) + 1 if len(self.vmap) else 0

    def orig(self, f: int) -> int:
        return f if self.vmap is None else int(self.vmap[f])

    def expand(self, a):
        """Per-original-feature array -> per engine column (None passes through)."""
        if a is None or self.vmap is None:
            return a
        if torch.is_tensor(a):
            return a[torch.as_tensor(self.vmap, device=a.device, dtype=torch.long)].contiguous()
        return np.asarray(a)[self.vmap]

    def to_state(self):
        return dict(F=self.F, stride=self.stride, edges=[None if e is None else e.tolist() for e in self.edges],
                    nbins=self.nbins.tolist(), iscat=self.iscat.tolist(), nlevels=self.nlevels.tolist(),
                    level_to_bin=[None if m is None else m.tolist() for m in self.level_to_bin],
                    vmap=None if self.vmap is None else self.vmap.tolist(), n_low=int(self.n_low),
                    n_mid=int(self.n_mid), cat_groups=[list(map(int, g)) for g in self.cat_groups],
                    pad=None if self.pad is None else self.pad.astype(int).tolist())

    @staticmethod
    def from_state(s):
        return Binning(s["F"], s["stride"], [None if e is None else np.asarray(e, dtype=np.float32) for e in s["edges"]],
                       np.asarray(s["nbins"], dtype=np.int32), np.asarray(s["iscat"], dtype=np.int32),
                       np.asarray(s["nlevels"], dtype=np.int32),
                       [None if m is None else np.asarray(m, dtype=np.int64) for m in s["level_to_bin"]],
                       None if s.get("vmap") is None else np.asarray(s["vmap"], dtype=np.int32),
                       int(s.get("n_low", 0)), int(s.get("n_mid", 0)),
                       [tuple(g) for g in s.get("cat_groups", [])],
                       None if s.get("pad") is None else np.asarray(s["pad"], dtype=bool))

    def gcat(self) -> np.ndarray | None:
        """int32 [F] for the engine: a wide-categorical group's first column = its number of real columns (1..4),
        its other columns (real and padding) = -1, every other column 0; None without groups."""
        if not self.cat_groups:
            return None
        g = np.zeros(self.F, dtype=np.int32)
        for c0, n in self.cat_groups:
            g[c0] = n
            g[c0 + 1:c0 + 4] = -1
        return g


def sample_rows(X: torch.Tensor, sample: int, seed: int, row0: int = 0, n_glob: int | None = None) -> torch.Tensor:
    """Bernoulli row sample for the quantile edges, decided per GLOBAL row index (counter-based hash,
    ``collectives.row_uniform``): identical on one process and on any row sharding, drawn on the
    device (no host permutation of N indices). Keeps ~``sample`` rows of ``n_glob``."""
    from ..parallel import collectives as coll
    F, N = X.shape
    n_glob = N if n_glob is None else int(n_glob)
    if n_glob <= sample:
        return X
    u = coll.row_uniform(int(seed), 0xB1A5, row0, N, X.device)
    return X[:, u < (sample / n_glob)]


def fit_binning_rows(X: torch.Tensor, iscat, nlevels=None, max_bins: int = MAX_DATA_BINS, sample: int = 1 << 20,
                     seed: int = 0, max_cat_bins: int = NA_BIN) -> "Binning":
    """:func:`fit_binning` over the rows of EVERY rank when the rows are sharded (exactly the
    single-process edges): each rank keeps the rows of the global-index sample it owns and only that
    sample (<= ``sample`` rows, not the frame) is exchanged."""
    from ..parallel import collectives as coll
    if not coll.is_dist():
        return fit_binning(X, iscat, nlevels, max_bins=max_bins, sample=sample, seed=seed, max_cat_bins=max_cat_bins)
    row0, n_glob = coll.exclusive_offset(X.shape[1])
    Xl = sample_rows(X, sample, seed, row0, n_glob)
    Xs = coll.all_gather_cat(Xl.contiguous(), dim=1, bounded=sample < (1 << 40))
    return fit_binning(Xs, iscat, nlevels, max_bins=max_bins, seed=seed, max_cat_bins=max_cat_bins, presampled=True)


def fit_binning(X: torch.Tensor, iscat, nlevels=None, max_bins: int = MAX_DATA_BINS, sample: int = 1 << 20,
                seed: int = 0, weights: torch.Tensor | None = None, max_cat_bins: int = NA_BIN,
                presampled: bool = False) -> Binning:
    """X: float32 [F, N] (column-major; NaN = missing; categorical columns hold level codes).
    Numeric edges are QuantilesGlobal cut points of a ~``sample``-row sample (all distinct values
    when there are at most ``max_bins``), computed on X's device: one batched sort of the sample,
    then per-feature distinct / quantile gathers; only the <=255 edges per feature reach the host.
    ``max_cat_bins`` (nbins_cats, at most 1016): categoricals with more levels keep their most
    frequent ``max_cat_bins - 1`` levels as bins and fold the rest into one shared bin; categoricals with
    more than 254 bins are WIDE categoricals (module note).
    ``presampled``: X already is the (gathered) sample. ``max_bins`` above 255 (at most 1016) bins numeric
    features with more distinct values into several engine columns (module note)."""
    cat_cap = int(min(max(2, max_cat_bins), WIDE_MAX_BINS))
    F, N = X.shape
    max_bins = int(min(max(2, max_bins), WIDE_MAX_BINS))
    iscat = np.asarray(iscat, dtype=np.int32)
    nlevels = np.zeros(F, dtype=np.int32) if nlevels is None else np.asarray(nlevels, dtype=np.int32)
    Xs = X if presampled else sample_rows(X, sample, seed)
    edges, nbins, l2b = [], np.zeros(F, dtype=np.int32), []
    num_cols = [f for f in range(F) if not iscat[f]]
    if num_cols:
        Xn = Xs[num_cols].float()
        Xn = torch.where(torch.isnan(Xn), torch.full_like(Xn, float("inf")), Xn)
        srt, _ = torch.sort(Xn, dim=1)
        M = srt.shape[1]
        # distinct-value counts of every feature in one pass (sorted rows: count value changes); finite counts,
        # distinct counts and the first value of every feature reach the host in ONE copy
        fin = torch.isfinite(srt)
        if M > 1:
            chg = (srt[:, 1:] != srt[:, :-1]) & fin[:, 1:]
            stats = torch.stack([fin.sum(1).double(), (chg.sum(1) + fin[:, 0].long()).double(), srt[:, 0].double()], 1)
        else:
            chg = None
            stats = torch.stack([fin.sum(1).double(), fin.sum(1).double(), srt[:, 0].double()], 1)
        stats = stats.cpu().numpy()
        nfin, ndist, first = stats[:, 0].astype(np.int64), stats[:, 1].astype(np.int64), stats[:, 2]
        # every numeric feature's edges in two batched gathers (one host copy each) instead of a gather + copy per
        # feature (MEASURED r5: the per-feature loop was ~60 host syncs, ~10 ms of a 100-tree GBM job)
        pre_edges = {}
        kq = [k for k in range(len(num_cols)) if nfin[k] > 0 and ndist[k] > max_bins]
        if kq:
            q = (np.arange(1, max_bins, dtype=np.int64)[None, :] * nfin[kq][:, None]) // max_bins
            vals = srt[torch.as_tensor(kq, device=srt.device)].gather(
                1, torch.as_tensor(q, device=srt.device)).float().cpu().numpy()
            for r, k in enumerate(kq):
                e = np.unique(vals[r])
                pre_edges[k] = np.ascontiguousarray(e[e > np.float32(first[k])], dtype=np.float32)
        kd = [k for k in range(len(num_cols)) if 0 < nfin[k] and ndist[k] <= max_bins and np.isfinite(first[k])]
        if kd and chg is not None:
            sub = chg[torch.as_tensor(kd, device=srt.device)]
            rc = torch.nonzero(sub)                                  # (row of kd, position - 1), row-major order
            vals = srt[torch.as_tensor(kd, device=srt.device)][rc[:, 0], rc[:, 1] + 1].float()
            both = torch.cat([rc[:, 0].float()[:, None], vals[:, None]], 1).cpu().numpy() if rc.numel() else \
                np.zeros((0, 2), dtype=np.float32)
            rows = both[:, 0].astype(np.int64)
            for r, k in enumerate(kd):
                pre_edges[k] = np.ascontiguousarray(both[rows == r, 1], dtype=np.float32)
        elif kd:
            for k in kd:
                pre_edges[k] = np.zeros(0, dtype=np.float32)
    for f in range(F):
        if iscat[f]:
            nl = int(nlevels[f]) if nlevels[f] > 0 else int(torch.nan_to_num(X[f], nan=-1).max().item()) + 1
            nlevels[f] = nl
            if nl <= cat_cap:
                l2b.append(None)
                nbins[f] = max(nl, 1)
            else:  # fold rare levels into the last bin
                codes = Xs[f][~torch.isnan(Xs[f])].long()      # frequencies of the (global) sample
                cnt = torch.bincount(codes, minlength=nl).cpu().numpy()
                order = np.argsort(-cnt, kind="stable")
                m = np.full(nl, cat_cap - 1, dtype=np.int64)
                m[order[: cat_cap - 1]] = np.arange(cat_cap - 1)
                l2b.append(m)
                nbins[f] = cat_cap
            edges.append(None)
            continue
        k = num_cols.index(f)
        n = int(nfin[k])
        l2b.append(None)
        if n == 0:
            edges.append(np.zeros(0, dtype=np.float32)); nbins[f] = 1
            continue
        if k in pre_edges:
            e = pre_edges[k]
        else:
            row = srt[k, :n]
            if int(ndist[k]) <= max_bins:
                e = torch.unique_consecutive(row)[1:]
            else:
                q = (torch.arange(1, max_bins, device=row.device, dtype=torch.int64) * n) // max_bins
                e = torch.unique_consecutive(row[q])
                e = e[e > row[0]]  # first bin must be non-empty
            e = e.float().cpu().numpy()
        edges.append(e)
        nbins[f] = e.size + 1
    vmap = None
    n_low = n_mid = 0
    wide_cat = [bool(iscat[f]) and nbins[f] > SUB_EDGES for f in range(F)]
    if any(e is not None and e.size > SUB_EDGES for e in edges) or any(wide_cat):
        # wide numeric features -> n adjacent engine columns with the interleaved edge subsets e[k::n];
        # wide categoricals -> n adjacent engine columns of (at most) 254 consecutive bins each
        # Layout in three tiers: every feature's FIRST column (edge subset e[0::n], ~254 quantile edges; all blocks
        # of a wide categorical), then the other subsets except the odd ones of 4-column features (with k = 2
        # these halve the edge spacing: e[0::4] + e[2::4] = e[0::2]), then those odd subsets. From the level on
        # where the adaptive bin count drops to 512 the tree searches only the first two tiers (n_mid columns),
        # from 256 only the first (n_low; ops/tree.narrow_cut): only their planes are histogrammed and moved.
        # H2O_HIST_FINE=1 keeps the former layout instead: the features of exactly 4 interleaved columns first,
        # each filling one aligned 4-byte row word (one fine-bin atomic per row and feature in the histogram kernel).
        fine_layout = os.environ.get("H2O_HIST_FINE") == "1"
        quad, rest, low, mid, high, groups = [], [], [], [], [], []
        for f in range(F):
            e = edges[f]
            if wide_cat[f]:
                # a group of n real columns padded to 4 (the group's bytes are one aligned row word)
                nb = int(nbins[f])
                lb = np.arange(nlevels[f], dtype=np.int64) if l2b[f] is None else l2b[f]
                n = -(-nb // SUB_EDGES)
                g = []
                for k in range(4):
                    if k < n:
                        b0, nk = k * SUB_EDGES, min(SUB_EDGES, nb - k * SUB_EDGES)
                        inb = (lb >= b0) & (lb < b0 + nk)
                        g.append((f, None, nk + 1, np.where(inb, lb - b0, nk), False))
                    else:
                        g.append((f, None, 1, np.zeros(max(int(nlevels[f]), 1), dtype=np.int64), True))
                groups.append((g, n))
                continue
            n = 1 if e is None or e.size <= SUB_EDGES else -(-e.size // SUB_EDGES)
            for k in range(n):
                ek = e if n == 1 else np.ascontiguousarray(e[k::n])
                c = (f, ek, (ek.size + 1) if e is not None else nbins[f], l2b[f])
                (quad if n == 4 else rest).append(c)
                (low if k == 0 else high if (n == 4 and k % 2) else mid).append(c)
        gcols = [c for g, _ in groups for c in g]
        cat_groups = []
        for i, (_, n) in enumerate(groups):
            cat_groups.append((4 * i, n))
        if fine_layout:
            cols = gcols + quad + rest
        else:
            cols = gcols + low + mid + high
            n_low = len(gcols) + len(low) if (mid or high) else 0
            n_mid = len(gcols) + len(low) + len(mid) if high else 0
        pad = np.asarray([len(c) > 4 and c[4] for c in cols], dtype=bool)
        cols = [c[:4] for c in cols]
        vmap = np.asarray([c[0] for c in cols], dtype=np.int32)
        edges = [c[1] for c in cols]
        nbins = np.asarray([c[2] for c in cols], dtype=np.int32)
        iscat, nlevels = iscat[vmap], nlevels[vmap]
        l2b = [c[3] for c in cols]
        F = len(cols)
    # rows of more than 12 features are padded to 16 B multiples so the partition kernel moves them
    # with 16-byte vector loads/stores (2 per 28-feature row instead of 7 dword pairs)
    # > 32 features: whole 32-byte planes (the device engine stores such bins PLANAR, one plane per
    # histogram feature tile — apply_binning(planar=True))
    stride = (F + 3) // 4 * 4 if F <= 12 else ((F + 15) // 16 * 16 if F <= 32 else (F + 31) // 32 * 32)
    if vmap is None:
        cat_groups, pad = [], None
    return Binning(F, stride, edges, nbins, iscat, nlevels, l2b, vmap, n_low, n_mid, cat_groups,
                   pad if pad is not None and pad.any() else None)


def _edge_table(b: Binning, device):
    maxe = max([1] + [0 if e is None else e.size for e in b.edges])
    tab = np.full((b.F, maxe), np.inf, dtype=np.float32)
    ned = np.zeros(b.F, dtype=np.int32)
    for f, e in enumerate(b.edges):
        if e is None:
            ned[f] = b.nbins[f] - 1
        else:
            tab[f, : e.size] = e
            ned[f] = e.size
    return torch.from_numpy(tab).to(device), torch.from_numpy(ned).to(device), maxe


def apply_binning(b: Binning, X: torch.Tensor, planar: bool = False) -> torch.Tensor:
    """X float32 [F, N] (original features) -> uint8 bins [N, stride] (row-major, one byte per ENGINE column) on
    X's device; with ``planar`` (device, stride a multiple of 32 and >= 64) the [stride / 32, N, 32] plane
    layout of the tree engine."""
    F, N = X.shape
    assert F == b.F_orig
    # source row of every engine column: its original feature, or (remapped categoricals: folded or
    # wide-categorical blocks) an extra row holding the column's own level -> bin codes
    src = [b.orig(f) for f in range(b.F)]
    maps = [(f, m) for f, m in enumerate(b.level_to_bin or []) if m is not None]
    if maps:
        Xc = torch.empty(F + len(maps), N, dtype=torch.float32, device=X.device)
        Xc[:F] = X
        for i, (f, m) in enumerate(maps):
            src[f] = F + i
            if b.pad is not None and b.pad[f]:       # group padding: bin 0 on every row (NA included)
                Xc[F + i] = 0.0
                continue
            col = X[b.orig(f)]
            mt = torch.as_tensor(m, device=X.device, dtype=torch.float32)
            codes = torch.nan_to_num(col, nan=0.0).long().clamp(0, m.size - 1)
            Xc[F + i] = torch.where(torch.isnan(col), col, mt[codes])
    else:
        Xc = X.contiguous().float()
    if X.is_cuda:
        tab, ned, maxe = _edge_table(b, X.device)
        iscat = torch.from_numpy(b.iscat.astype(np.int32)).to(X.device)
        planar = bool(planar) and b.stride >= 64 and b.stride % 32 == 0
        out = (torch.empty(b.stride // 32, N, 32, dtype=torch.uint8, device=X.device) if planar
               else torch.empty(N, b.stride, dtype=torch.uint8, device=X.device))
        xmap = (None if b.vmap is None and not maps
                else torch.as_tensor(np.asarray(src, dtype=np.int32), dtype=torch.int32, device=X.device))
        nat.call("h2o_bin_assign", Xc.data_ptr(), N, b.F, b.stride, tab.data_ptr(), maxe, ned.data_ptr(),
                 iscat.data_ptr(), out.data_ptr(), int(planar), 0 if xmap is None else xmap.data_ptr(),
                 nat.stream_ptr(X.device))
        return out
    out = torch.zeros(N, b.stride, dtype=torch.uint8)
    for f in range(b.F):
        col = Xc[src[f]]
        nan = torch.isnan(col)
        if b.iscat[f]:
            code = torch.nan_to_num(col, nan=-1).long()
            bad = nan | (code < 0) | (code >= max(int(b.nbins[f]), 1))
            bf = torch.where(bad, torch.full_like(code, NA_BIN), code)
        else:
            e = torch.from_numpy(b.edges[f])
            bf = torch.bucketize(torch.nan_to_num(col, nan=0.0), e, right=True)
            bf = torch.where(nan, torch.full_like(bf, NA_BIN), bf)
        out[:, f] = bf.to(torch.uint8)
    return out
