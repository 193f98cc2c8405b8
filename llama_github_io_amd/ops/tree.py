"""Histogram tree engine (device side) shared by GBM / DRF / XGBoost / IsolationForest / DT / Uplift.

Two interchangeable builders produce the same :class:`TreeLevels` result:

* :class:`GpuTreeBuilder` drives the HIP kernels of ``csrc/tree_kernels.hip`` (node-partitioned rows,
  LDS histograms, fused partition + smaller-child histogram, on-device split search and planning).
  A whole tree is a fixed sequence of launches on the current stream with no host synchronisation.
* :class:`RefTreeBuilder` is the PyTorch/NumPy reference of exactly the same algorithm (same split
  rules, same tie breaks, same leaf numbering); it runs on CPU tensors and is the numerics oracle.

Split semantics follow ``hex/tree/DTree.java:984`` (findBestSplitPoint): squared-error reduction on
(w, wY) histograms, NA bin with NA-left / NA-right / NA-vs-rest options, ``min_rows`` on weighted
counts, relative ``min_split_improvement`` against the node's squared error, categorical levels
sorted by mean response. Mode 1 is XGBoost's Newton gain G²/(H+λ) with L1 soft-threshold α and γ.
"""
from __future__ import annotations

import ctypes
import math
import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _native as nat
from ..parallel import collectives as coll

NBIN = 256
NA_BIN = 255
MAX_DATA_BINS = 255
FTILE = 32
AMAX_SHARDS = 64   # per-block |aux| maxima shards (csrc: AMAX_SHARDS)

NODE_DT = np.dtype([("start", "<i4"), ("len", "<i4"), ("build", "<i4"), ("parent", "<i4"), ("sib", "<i4"),
                    ("dir", "<i4"), ("p1", "<i4"), ("p2", "<i4")])
NBW = 32            # 32-bit words of a decision bitset: 1024 bins (a wide-categorical group's levels)
DEC_DT = np.dtype([("feat", "<i4"), ("bin", "<i4"), ("na_left", "<i4"), ("is_cat", "<i4"), ("bits", "<u4", (NBW,)),
                   ("gain", "<f8"), ("wl", "<f8"), ("wr", "<f8"), ("predl", "<f4"), ("predr", "<f4")])
CAND_BYTES = 184
_GRAPH_CACHE = 16          # captured per-tree graphs kept (one per launch-plan signature)
GROUP_CAT = 2       # Dec.is_cat of a wide-categorical group split: bin = the group's packed 'elsewhere' bytes
MODE_SE, MODE_NEWTON, MODE_RANDOM = 0, 1, 2
# histogram types as candidate lattices over the global bins (k_split_find HT_*)
HT_QUANTILES, HT_UNIFORM, HT_RANDOM, HT_ROBUST, HT_ROUND_ROBIN = 0, 1, 2, 3, 4
HIST_TYPES = {"auto": HT_UNIFORM, "uniformadaptive": HT_UNIFORM, "random": HT_RANDOM, "uniformrobust": HT_ROBUST,
              "roundrobin": HT_ROUND_ROBIN, "quantilesglobal": HT_QUANTILES}
_M64 = (1 << 64) - 1


def fine_columns(fgroup, iscat, F):
    """int32 [F]: 1 for the columns of the word-aligned (4m .. 4m+3) groups of exactly 4 engine columns of one
    numeric feature (wide numeric bins, ops/binning.py) — the histogram kernel adds one fine-bin atomic per row and
    group there — or None when there is no such group."""
    if fgroup is None:
        return None
    g = np.asarray(fgroup, dtype=np.int64)
    out = np.zeros(F, dtype=np.int32)
    for m in range(0, F - 3, 4):
        if (g[m] == g[m + 1] == g[m + 2] == g[m + 3] and (m == 0 or g[m - 1] != g[m]) and (m + 4 >= F or g[m + 4] != g[m])
                and not any(int(iscat[m + l]) for l in range(4))):
            out[m:m + 4] = 1
    return out if out.any() else None


def narrow_cut(p: "SplitParams", n_low: int, n_mid: int, F: int):
    """Columns each level searches under the NARROW views of wide numeric bins: ``(mid_from, lo_from)``, the first
    levels (or -1) from which only engine columns [0, n_mid) resp. [0, n_low) are searched (ops/binning.py three-tier
    layout). With an adaptive histogram type a level whose bin count max(nbins, nbins_top_level >> d) is at most
    512 needs no finer edge spacing than every other fine edge (the first two tiers), at most 256 than every fourth
    (the first tier, ~254 quantile edges); their histograms, searches and row moves then cost what a 2x / 1x
    255-bin QuantilesGlobal run does. H2O_TREE_NARROW=0: every level searches every column."""
    off = (-1, -1)
    if os.environ.get("H2O_TREE_NARROW", "1") == "0" or not p.adapt_nbins or p.edges is None:
        return off
    lo = mid = -1
    for d in range(64):
        nb = p.adapt_nb(d)
        if mid < 0 and 0 < n_mid < F and 0 < nb <= 512:
            mid = d
        if lo < 0 and 0 < n_low < F and 0 < nb <= 256:
            lo = d
    return mid, lo


def level_fcut(cut, n_low: int, n_mid: int, d: int) -> int:
    """Columns level ``d`` searches (0 = all) for ``cut = narrow_cut(...)``."""
    mid, lo = cut
    if lo >= 0 and d >= lo:
        return n_low
    if mid >= 0 and d >= mid:
        return n_mid
    return 0


def encode_groups(fgroup) -> np.ndarray | None:
    """int32 [F] for the device: the original feature in bits 0-29, bit 30 on every column but the feature's
    first (k_split_reduce's column-sampling leaders)."""
    if fgroup is None:
        return None
    g = np.asarray(fgroup, dtype=np.int64)
    seen, out = set(), np.empty(g.size, dtype=np.int32)
    for f, v in enumerate(g.tolist()):
        out[f] = v | (0 if v not in seen else 1 << 30)
        seen.add(v)
    return out


def splitmix64(x: int) -> int:
    x = (x + 0x9E3779B97F4A7C15) & _M64
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & _M64
    return x ^ (x >> 31)


@dataclass
class SplitParams:
    min_w: float = 10.0                  # min_rows (SE) / min_child_weight (Newton)
    min_split_improvement: float = 1e-5
    lam: float = 0.0
    alpha: float = 0.0
    gamma: float = 0.0
    mode: int = MODE_SE
    random_split: bool = False
    # UniformAdaptive (the H2O default histogram_type): per-level bin counts max(nbins, nbins_top_level >> d)
    # applied as a candidate lattice over the global bin edges ([F, 255] float32, inf padded)
    adapt_nbins: int = 0
    adapt_top: int = 0
    edges: object = None
    # lattice of the split points (HT_*): UniformAdaptive, Random, UniformRobust or RoundRobin
    hist_type: int = 1
    # [F, 2] float32 exact (min, max) of every engine column over ALL rows (the root histogram's range,
    # DHistogram.initialHist); with it the open-ended first / last bins map to the true extremes. None: edges only.
    vrange: object = None
    # the reference's node range (DTree.java:337-375): a node at depth >= 1 bins over the range its PARENT's
    # histogram observed, narrowed at the parent's split for the split feature; False: the node's own occupied range
    parent_range: bool = True

    def adapt_nb(self, level: int) -> int:
        if not self.adapt_nbins or self.edges is None:
            return 0
        return max(int(self.adapt_nbins), int(self.adapt_top) >> int(level))


@dataclass
class TreeLevels:
    """Host copy of one built tree: per level decision records and child links.

    child >= 0 is the index of the child in the next level; child < 0 encodes leaf id ``-1 - child``.
    A terminal node (dec.feat < 0) has child_l == child_r == its own leaf.
    """
    decs: list
    child_l: list
    child_r: list
    n_leaves: int
    leaf_values: np.ndarray | None = None
    root_weight: float = 0.0


# ================================================================================================
# reference split search (NumPy, float64) — mirrors k_split_find / k_split_reduce exactly
def _E(mode, p: SplitParams, w, y):
    if mode == MODE_NEWTON:
        g = y
        if p.alpha > 0:
            g = np.where(g > p.alpha, g - p.alpha, np.where(g < -p.alpha, g + p.alpha, 0.0))
        return g * g / (w + p.lam)
    with np.errstate(divide="ignore", invalid="ignore"):
        return np.where(w > 0, y * y / np.where(w > 0, w, 1.0), 0.0)


def _leafv(mode, p, w, y):
    if mode == MODE_NEWTON:
        return y / (w + p.lam)
    return y / w if w > 0 else 0.0


def _bin_lo(p: SplitParams, f, b):
    """Lower value bound of data bin b of engine column f (bin 0: the column's true minimum when known)."""
    if b > 0:
        return float(np.float32(p.edges[f][b - 1]))
    return float(np.float32(p.vrange[f][0])) if p.vrange is not None else float(np.float32(p.edges[f][0]))


def _bin_hi(p: SplitParams, f, b, nb):
    """Upper (exclusive) value bound of data bin b (the last data bin: the column's true maximum when known)."""
    if b < nb - 1:
        return float(np.float32(p.edges[f][b]))
    return float(np.float32(p.vrange[f][1])) if p.vrange is not None else float(np.float32(p.edges[f][nb - 2]))


def _lattice(p: SplitParams, level, node, f, nb, w, sw, W, seed, off, vr=None):
    """Allowed thresholds t = 1 .. nb-1 of the histogram type's split points (None = every threshold);
    mirrors the lattice block of k_split_find (UniformAdaptive / Random / UniformRobust / RoundRobin).
    ``vr`` = (lo, hi): the node's value range (the parent's observed range narrowed at its split, see
    :meth:`RefTreeBuilder.build`); None: the node's own occupied range."""
    anb = p.adapt_nb(level)
    lt = p.hist_type if (anb > 1 and not off) else HT_QUANTILES
    if lt == HT_ROUND_ROBIN:
        r = splitmix64((seed ^ 0xDECAF ^ (level << 48) ^ (node << 20) ^ f) & _M64) & 3
        lt = HT_QUANTILES if r == 3 else (HT_RANDOM if r == 2 else HT_UNIFORM)
    if lt == HT_QUANTILES:
        return None
    occ = np.nonzero(w[:nb] > 0)[0]
    if not (occ.size and occ[-1] > occ[0]):
        return None
    a_lo, a_hi = int(occ[0]), int(occ[-1])
    e = np.asarray(p.edges[f], dtype=np.float32).astype(np.float64)
    if vr is not None:
        lo, hi = float(vr[0]), float(vr[1])
    else:
        if lt != HT_RANDOM and not a_hi - a_lo + 1 > anb:
            return None
        lo = float(e[a_lo - 1 if a_lo > 0 else 0])
        hi = float(e[a_hi if a_hi <= nb - 2 else nb - 2])
    if not hi > lo:
        return None
    sc = anb / (hi - lo)

    def cnt(x):
        return int(min(max(np.floor((x - lo) * sc), 0), anb - 1))

    mark = np.zeros(max(nb, 1), dtype=bool)        # mark[t]: threshold t is kept
    ee = e[:nb - 1]

    def put(x):
        i = int(np.searchsorted(ee, x, side="left"))   # first i with edge[i] >= x
        if i < nb - 1:
            mark[i + 1] = True
    if lt == HT_ROBUST:
        cell = np.array([0 if t == a_lo else cnt(e[t - 1]) for t in range(a_lo, a_hi + 1)])
        cw = np.zeros(anb)
        for c in np.unique(cell):
            ts = np.nonzero(cell == c)[0] + a_lo
            cw[c] = sw[ts[-1]] - (sw[ts[0] - 1] if ts[0] > 0 else 0.0)
        K = int((cw > 0).sum())
        budget = anb - K - 2
        if K <= 0.2 * anb and budget > 0 and K > 0:
            nz = [c for c in range(anb) if cw[c] > 0]
            order = sorted(nz, key=lambda c: (-cw[c], c))
            left = budget
            step = (hi - lo) / anb
            for c in order:
                q = int(np.ceil(budget * cw[c] / W))
                nnew = max(0, min(q, left))
                left -= min(q, left) if left > 0 else 0
                c0 = lo + step * float(c)
                sub = step / float(1 + nnew)
                for j in range(nnew + 1):
                    put(c0 + sub * float(j))
            put(lo)
            put(hi)
        else:
            lt = HT_UNIFORM
    if lt == HT_UNIFORM:
        c = np.clip(np.floor((e[:nb - 1] - lo) * sc), 0, anb - 1)     # cnt(e[t - 1]), t = 1 .. nb-1
        return c > np.concatenate([[0.0], c[:-1]])
    if lt == HT_RANDOM:
        for k in range(1, anb):
            h = splitmix64((seed ^ 0xC0FFEE ^ (level << 48) ^ (node << 20) ^ (f << 10) ^ k) & _M64)
            put(lo + (hi - lo) * (float(h >> 11) * 2.0 ** -53))
    return mark[1:nb]


def group_pack(nbins_f, f, n) -> int:
    """Dec.bin of a group split: byte k = the 'elsewhere' bin of the group's k-th real column (0: padding)."""
    v = sum(int(nbins_f[f + k] - 1) << (8 * k) for k in range(n))
    return v - (1 << 32) if v >= 1 << 31 else v          # as the int32 the record holds


def _invalid_cand():
    return dict(expl=-1.0e300, gain=0.0, wl=0.0, wr=0.0, bin=0, na_left=0, valid=False, is_cat=0,
                bits=np.zeros(NBW, dtype=np.uint32), predl=0.0, predr=0.0)


def split_find_ref(h, nayy, wyy, nbins_f, iscat_f, mono_f, p: SplitParams, level: int, node: int, seed: int,
                   vranges=None, gcat=None):
    """h: float64 [F, 256, 2]. Returns list of per-feature candidate dicts. ``vranges``: [F, 2] value ranges of
    the node (reference node ranges, :meth:`RefTreeBuilder.build`) or None. ``gcat`` (Binning.gcat): a
    wide-categorical group's first column searches ONE histogram over all the group's levels (global bin 254k + b
    of real column k), its other columns offer nothing."""
    F = h.shape[0]
    out = []
    for f in range(F):
        grp = 0 if gcat is None else int(gcat[f])
        if grp < 0:
            out.append(_invalid_cand())
            continue
        nb = int(nbins_f[f])
        cat = bool(iscat_f[f])
        mono = int(mono_f[f]) if mono_f is not None else 0
        M = 256 if grp == 0 else 1024
        w = np.zeros(M); wy = np.zeros(M)
        if grp == 0:
            lim = min(nb, NA_BIN)
            w[:lim] = h[f, :lim, 0]; wy[:lim] = h[f, :lim, 1]
        else:                          # the group's levels, 'elsewhere' bins dropped
            for k in range(grp):
                nk = int(nbins_f[f + k]) - 1
                w[254 * k:254 * k + nk] = h[f + k, :nk, 0]; wy[254 * k:254 * k + nk] = h[f + k, :nk, 1]
                nb = 254 * k + nk
            cat = True
        wNA, wyNA = h[f, NA_BIN, 0], h[f, NA_BIN, 1]
        idx = np.arange(M)
        if cat:
            key = np.where(idx < nb, np.where(w > 0, wy / np.where(w > 0, w, 1), -1.0e308), 1.0e308)
            idx = np.lexsort((idx, key))  # sort by key then index
            w = w[idx]; wy = wy[idx]
        sw = np.cumsum(w); swy = np.cumsum(wy)
        W, WY = sw[M - 1], swy[M - 1]
        Wall, WYall = W + wNA, WY + wyNA
        random_mode = p.random_split
        rand_b = -1
        if random_mode:
            occ = np.nonzero(w[:nb] > 0)[0]
            if occ.size and occ[-1] > occ[0]:
                lo, hi = int(occ[0]), int(occ[-1])
                hsh = splitmix64((seed ^ (level << 48) ^ (node << 20) ^ f) & _M64)
                rand_b = lo + 1 + int(hsh % (hi - lo))
        allowed = _lattice(p, level, node, f, nb, w, sw, W, seed, cat or random_mode,
                           None if vranges is None else vranges[f])
        best_e, best_code = -1.0e300, -1
        cands = []
        if wNA >= p.min_w and W > 0 and not random_mode:
            cands.append((float(_E(p.mode, p, W, WY) + _E(p.mode, p, wNA, wyNA)), 0))
        if random_mode:
            ts = [rand_b] if 1 <= rand_b < nb else []
        else:
            ts = None
        if ts is None and nb > 1:
            # every threshold t = 1 .. nb-1 at once (same float64 operations as the per-t rule below)
            t = np.arange(1, nb)
            m = (sw[t] - sw[t - 1]) != 0.0
            if allowed is not None:
                m &= allowed
            wlo, wylo = sw[t - 1], swy[t - 1]
            whi, wyhi = W - wlo, WY - wylo

            def lv(a, b):
                if p.mode == MODE_NEWTON:
                    return b / (a + p.lam)
                with np.errstate(divide="ignore", invalid="ignore"):
                    return np.where(a > 0, b / np.where(a > 0, a, 1.0), 0.0)

            def mono_ok(a1, b1, a2, b2):
                return np.ones_like(a1, dtype=bool) if mono == 0 else mono * lv(a1, b1) <= mono * lv(a2, b2)
            if wNA == 0.0:
                ok = m & (wlo >= p.min_w) & (whi >= p.min_w) & mono_ok(wlo, wylo, whi, wyhi)
                ev = _E(p.mode, p, wlo, wylo) + _E(p.mode, p, whi, wyhi)
                code = t * 2 + (wlo > whi)
            else:
                ok1 = m & (wlo + wNA >= p.min_w) & (whi >= p.min_w) & mono_ok(wlo + wNA, wylo + wyNA, whi, wyhi)
                e1 = _E(p.mode, p, wlo + wNA, wylo + wyNA) + _E(p.mode, p, whi, wyhi)
                ok2 = m & (wlo >= p.min_w) & (whi + wNA >= p.min_w) & mono_ok(wlo, wylo, whi + wNA, wyhi + wyNA)
                e2 = _E(p.mode, p, wlo, wylo) + _E(p.mode, p, whi + wNA, wyhi + wyNA)
                right = ok2 & (~ok1 | (e2 > e1))
                ok = ok1 | ok2
                ev = np.where(right, e2, e1)
                code = t * 2 + np.where(right, 0, 1)
            if ok.any():
                ev, code = ev[ok], code[ok]
                be = float(ev.max())
                cands.append((be, int(code[ev == be].min())))
        for t in (ts or []):
            wlo, wylo = sw[t - 1], swy[t - 1]
            whi, wyhi = W - wlo, WY - wylo
            my_e, my_c = -1.0e300, -1
            if wNA == 0.0:
                if wlo >= p.min_w and whi >= p.min_w:
                    ok = mono == 0 or mono * _leafv(p.mode, p, wlo, wylo) <= mono * _leafv(p.mode, p, whi, wyhi)
                    if ok:
                        my_e = float(_E(p.mode, p, wlo, wylo) + _E(p.mode, p, whi, wyhi)); my_c = t * 2 + (1 if wlo > whi else 0)
            else:
                if wlo + wNA >= p.min_w and whi >= p.min_w:
                    e = float(_E(p.mode, p, wlo + wNA, wylo + wyNA) + _E(p.mode, p, whi, wyhi))
                    ok = mono == 0 or mono * _leafv(p.mode, p, wlo + wNA, wylo + wyNA) <= mono * _leafv(p.mode, p, whi, wyhi)
                    if ok and e > my_e:
                        my_e, my_c = e, t * 2 + 1
                if wlo >= p.min_w and whi + wNA >= p.min_w:
                    e = float(_E(p.mode, p, wlo, wylo) + _E(p.mode, p, whi + wNA, wyhi + wyNA))
                    ok = mono == 0 or mono * _leafv(p.mode, p, wlo, wylo) <= mono * _leafv(p.mode, p, whi + wNA, wyhi + wyNA)
                    if ok and e > my_e:
                        my_e, my_c = e, t * 2
            if my_c >= 0:
                cands.append((my_e, my_c))
        for e, c in cands:
            if best_code < 0 or e > best_e or (e == best_e and c < best_code):
                best_e, best_code = e, c
        b, nal = (best_code >> 1, best_code & 1) if best_code > 0 else (0, 0)
        bits = np.zeros(NBW, dtype=np.uint32)
        if cat and best_code > 0:
            for t in range(nb):
                cidx = idx[t]
                empty = (sw[t] - (sw[t - 1] if t > 0 else 0.0)) == 0.0
                left = (nal != 0) if empty else (t < b)
                if left:
                    bits[cidx >> 5] |= np.uint32(1 << (cidx & 31))
        wl = wr = yl = yr = 0.0
        if best_code == 0:
            wl, yl, wr, yr = W, WY, wNA, wyNA
        elif best_code > 0:
            wl, yl = sw[b - 1], swy[b - 1]
            wr, yr = W - wl, WY - yl
            if nal:
                wl += wNA; yl += wyNA
            else:
                wr += wNA; yr += wyNA
        Epar = float(_E(p.mode, p, Wall, WYall))
        gain = best_e - Epar
        valid = False
        if best_code >= 0 and Wall >= 2.0 * p.min_w:
            if p.mode == MODE_SE:
                var = wyy * Wall - WYall * WYall
                seBefore = (wyy - Epar) if wNA >= p.min_w else ((wyy - nayy[f]) - float(_E(p.mode, p, W, WY)))
                seAfter = wyy - best_e
                pl, pr = np.float32(yl / wl) if wl else np.float32(np.nan), np.float32(yr / wr) if wr else np.float32(np.nan)
                valid = (np.float32(var) != 0) and (seAfter < seBefore * (1.0 - p.min_split_improvement)) and \
                    (pl != pr) and wl >= p.min_w and wr >= p.min_w
                if random_mode:
                    valid = wl > 0 and wr > 0
            elif p.mode == MODE_NEWTON:
                valid = (0.5 * gain - p.gamma) > 1e-6 and wl >= p.min_w and wr >= p.min_w
                gain = 0.5 * gain - p.gamma
            else:
                valid = wl > 0 and wr > 0
        if cat and best_code == 0:
            bits[:] = 0xFFFFFFFF
        cbin = NA_BIN if best_code == 0 else b
        if grp > 0:
            cbin = group_pack(nbins_f, f, grp)
        out.append(dict(expl=best_e, gain=gain, wl=wl, wr=wr, bin=cbin,
                        na_left=0 if best_code == 0 else nal, valid=bool(valid), is_cat=GROUP_CAT if grp else int(cat),
                        bits=bits, predl=_leafv(p.mode, p, wl, yl), predr=_leafv(p.mode, p, wr, yr)))
    return out


def split_reduce_ref(cands, feat_ok, k_cols, seed, level, node, node_ok=None, fgroup=None):
    """k_split_reduce: best usable column; with ``fgroup`` (engine column -> original feature) the column
    sample draws original features, whose engine columns share one key and rank (the feature's first column
    counts it)."""
    F = len(cands)
    gid = list(range(F)) if fgroup is None else [int(g) for g in fgroup]
    lead = [gid[f] not in gid[:f] for f in range(F)] if fgroup is not None else [True] * F
    base = splitmix64((seed ^ ((level + 1) << 40) ^ node) & _M64)
    ok = [bool(feat_ok[f]) and (node_ok is None or bool(node_ok[f])) for f in range(F)]
    n_ok = sum(1 for f in range(F) if ok[f] and lead[f])
    sample = 0 < k_cols < n_ok
    allowed = ok[:]
    if sample:
        keys = [splitmix64((base + gid[f]) & _M64) for f in range(F)]
        for f in range(F):
            if not ok[f]:
                continue
            rank = sum(1 for g in range(F) if ok[g] and lead[g] and
                       (keys[g] < keys[f] or (keys[g] == keys[f] and gid[g] < gid[f])))
            allowed[f] = rank < k_cols
    be, bf = -1.0e300, -1
    for f in range(F):
        c = cands[f]
        if allowed[f] and c["valid"] and (bf < 0 or c["expl"] > be):
            be, bf = c["expl"], f
    d = np.zeros(1, dtype=DEC_DT)[0]
    d["feat"] = bf
    if bf >= 0:
        c = cands[bf]
        d["bin"], d["na_left"], d["is_cat"], d["bits"] = c["bin"], c["na_left"], c["is_cat"], c["bits"]
        d["gain"], d["wl"], d["wr"], d["predl"], d["predr"] = c["gain"], c["wl"], c["wr"], c["predl"], c["predr"]
    return d


def _level_k(k_cols, d: int) -> int:
    """Column sample size at depth ``d``: an int for every level, or a per-level list
    (DTree.actual_mtries with col_sample_rate_change_per_level)."""
    if isinstance(k_cols, (list, tuple)):
        return int(k_cols[min(d, len(k_cols) - 1)]) if k_cols else 0
    return int(k_cols)


def group_level_np(pack: int, b4: np.ndarray) -> np.ndarray:
    """Global bin (254k + byte) of every row of a wide-categorical group from its 4 group bytes [n, 4]; -1 = NA."""
    b4 = np.asarray(b4, dtype=np.int64)
    lvl = np.full(b4.shape[0], -1, dtype=np.int64)
    na = b4[:, 0] == NA_BIN
    for k in range(4):
        ek = ((int(pack) & 0xFFFFFFFF) >> (8 * k)) & 255
        if ek == 0:
            continue
        hit = (lvl < 0) & ~na & (b4[:, k] != ek)
        lvl[hit] = 254 * k + b4[hit, k]
    return lvl


def dec_go_left_np(d, b: np.ndarray) -> np.ndarray:
    """``b``: the split column's bins [n] — or, for a group split (is_cat == GROUP_CAT), the group's 4 bytes [n, 4]."""
    if d["feat"] < 0:
        return np.ones(b.shape[0], dtype=bool)
    if int(d["is_cat"]) == GROUP_CAT:
        lvl = group_level_np(int(d["bin"]), b)
        bits = d["bits"]
        lc = np.maximum(lvl, 0)
        gl = ((bits[lc >> 5] >> (lc & 31).astype(np.uint32)) & 1).astype(bool)
        return np.where(lvl < 0, bool(d["na_left"]), gl)
    na = b == NA_BIN
    if d["is_cat"]:
        bits = d["bits"]
        gl = ((bits[b >> 5] >> (b & 31).astype(np.uint32)) & 1).astype(bool)
    else:
        gl = b < d["bin"]
    return np.where(na, bool(d["na_left"]), gl)


# ================================================================================================
class RefTreeBuilder:
    """CPU reference builder (same algorithm, float64 histograms, index lists instead of partitions)."""

    def __init__(self, bins: torch.Tensor, F: int, nbins_f, iscat_f, mono_f, max_depth: int, params: SplitParams,
                 node_cap: int = 1 << 15):
        self.bins = bins.cpu().numpy() if isinstance(bins, torch.Tensor) else np.asarray(bins)
        self.F = F
        self.nbins_f = np.asarray(nbins_f)
        self.iscat_f = np.asarray(iscat_f)
        self.mono_f = None if mono_f is None else np.asarray(mono_f)
        self.D = max_depth
        self.p = params
        self.node_cap = node_cap
        self.N = self.bins.shape[0]
        self.ic_map = None
        self.n_low = self.n_mid = 0
        self.gcat = None

    def set_interaction_constraints(self, ic_map, root_ok):
        """``ic_map`` [F, F] (row f: features allowed to interact with f), ``root_ok`` [F]."""
        self.ic_map = np.asarray(ic_map, dtype=np.uint8)
        self.ic_root = np.asarray(root_ok, dtype=np.uint8)

    def set_feature_groups(self, fgroup, n_low: int = 0, n_mid: int = 0):
        """Engine column -> original feature (wide numeric features span several columns): column sampling
        draws original features. ``n_low`` / ``n_mid``: leading columns of the narrow views (:func:`narrow_cut`)."""
        self.fgroup = None if fgroup is None else np.asarray(fgroup, dtype=np.int64)
        self.n_low, self.n_mid = int(n_low), int(n_mid)

    def set_cat_groups(self, gcat):
        """Wide-categorical groups (Binning.gcat): one search over all of a group's levels (H2O's single sort)."""
        self.gcat = None if gcat is None else np.asarray(gcat, dtype=np.int32)

    def _split_bytes(self, d, rows):
        f = int(d["feat"])
        if int(d["is_cat"]) == GROUP_CAT:
            return self.bins[rows, f:f + 4].astype(np.int64)
        return self.bins[rows, f].astype(np.int64)

    def _hist(self, rows, aux):
        F = self.F
        h = np.zeros((F, 256, 2))
        a = aux[rows, 0].astype(np.float64); b = aux[rows, 1].astype(np.float64)
        a32 = aux[rows, 0]; b32 = aux[rows, 1]
        yy = np.where(a32 > 0, (b32 * b32 / np.where(a32 > 0, a32, 1)).astype(np.float32), 0).astype(np.float64)
        nayy = np.zeros(F)
        for f0 in range(0, F, 16):          # 16 features per bincount (same per-bin summation order)
            f1 = min(F, f0 + 16)
            bf = self.bins[rows, f0:f1].astype(np.int64)
            key = (bf + 256 * np.arange(f1 - f0)[None, :]).T.reshape(-1)
            n = 256 * (f1 - f0)
            h[f0:f1, :, 0] = np.bincount(key, weights=np.tile(a, f1 - f0), minlength=n).reshape(f1 - f0, 256)
            h[f0:f1, :, 1] = np.bincount(key, weights=np.tile(b, f1 - f0), minlength=n).reshape(f1 - f0, 256)
            for j in range(f1 - f0):
                nayy[f0 + j] = yy[bf[:, j] == NA_BIN].sum()
        return h, nayy, yy.sum()

    def _ranges_on(self) -> bool:
        p = self.p
        return (bool(p.parent_range) and bool(p.adapt_nbins) and p.edges is not None and p.vrange is not None
                and p.hist_type != HT_QUANTILES)

    def _occupied(self, h):
        """[F, 2] int: first / last occupied data bin of every column of a node histogram (-1: none)."""
        F = self.F
        occ = np.full((F, 2), -1, dtype=np.int64)
        for f in range(F):
            nb = min(int(self.nbins_f[f]), NA_BIN)
            nz = np.nonzero(h[f, :nb, 0] > 0)[0]
            if nz.size:
                occ[f] = (nz[0], nz[-1])
        return occ

    def _value_ranges(self, occ, split=None, side=0):
        """[F, 2] value ranges of a node: the parent's observed ranges ``occ`` (bins -> values; the open-ended
        first / last bins -> the column's true extremes), and for the parent's numeric split ``split`` = (column,
        bin) the narrowing of every column of the same feature at the split value (DTree.java:360-375: the left
        side's exclusive max / the right side's min)."""
        p, F = self.p, self.F
        vr = np.full((F, 2), np.nan)
        for f in range(F):
            if occ[f, 0] < 0 or self.iscat_f[f]:
                continue
            nb = int(self.nbins_f[f])
            vr[f] = (_bin_lo(p, f, int(occ[f, 0])), _bin_hi(p, f, int(occ[f, 1]), nb))
        if split is not None:
            sf, b = split
            v = float(np.float32(p.edges[sf][b - 1]))
            grp = getattr(self, "fgroup", None)
            for f in range(F):
                same = f == sf if grp is None else grp[f] == grp[sf]
                if same and not np.isnan(vr[f, 0]):
                    if side == 0:
                        vr[f, 1] = min(vr[f, 1], v)
                    else:
                        vr[f, 0] = max(vr[f, 0], v)
        return vr

    def build(self, aux_static: torch.Tensor, feat_ok=None, k_cols: int = 0, seed: int = 0, leaf_fn=None):
        aux = aux_static.detach().cpu().numpy().astype(np.float32)
        ranges = self._ranges_on()
        F, D, p = self.F, self.D, self.p
        feat_ok = np.ones(F, dtype=np.int32) if feat_ok is None else np.asarray(feat_ok)
        leaf_of_row = np.full(self.N, -1, dtype=np.int64)
        cut = narrow_cut(p, self.n_low, self.n_mid, F)
        leafsum = []
        level_rows = [np.arange(self.N)]
        level_ok = [None if self.ic_map is None else self.ic_root]
        level_vr = [None]                 # per node: [F, 2] value ranges (None at the root: its own, set below)
        decs, cls, crs = [], [], []
        n_leaves = 0
        for d in range(D):
            cap_next = min(1 << (d + 1), self.node_cap) if d + 1 < D else 1
            n = len(level_rows)
            dl = np.zeros(n, dtype=DEC_DT)
            level_occ = []
            for i, rows in enumerate(level_rows):
                h, nayy, wyy = self._hist(rows, aux)
                if coll.is_dist():  # row-sharded: every rank sees the global node histogram
                    flat = torch.from_numpy(np.concatenate([h.ravel(), nayy, [wyy]]))
                    coll.all_reduce_(flat)
                    flat = flat.numpy()
                    h = flat[: h.size].reshape(h.shape)
                    nayy = flat[h.size: h.size + F]
                    wyy = float(flat[-1])
                vr = None
                if ranges:
                    level_occ.append(self._occupied(h))
                    vr = level_vr[i] if level_vr[i] is not None else self._value_ranges(level_occ[i])
                cands = split_find_ref(h, nayy, wyy, self.nbins_f, self.iscat_f, self.mono_f, p, d, i, seed, vr,
                                       self.gcat)
                fc = level_fcut(cut, self.n_low, self.n_mid, d)
                if fc:                          # narrow level: the columns past fc are not searched
                    for f in range(fc, F):
                        cands[f]["valid"] = False
                dl[i] = split_reduce_ref(cands, feat_ok, _level_k(k_cols, d), seed, d, i, level_ok[i],
                                         getattr(self, "fgroup", None))
            cl = np.zeros(n, dtype=np.int64); cr = np.zeros(n, dtype=np.int64)
            nxt, nxt_ok, nxt_vr = [], [], []
            act = 0
            for i, rows in enumerate(level_rows):
                dd = dl[i]
                if dd["feat"] < 0:
                    lid = n_leaves; n_leaves += 1
                    cl[i] = cr[i] = -1 - lid
                    leaf_of_row[rows] = lid
                    leafsum.append((aux[rows, 2].astype(np.float64).sum(), aux[rows, 3].astype(np.float64).sum()))
                    continue
                gl = dec_go_left_np(dd, self._split_bytes(dd, rows))
                lrows, rrows = rows[gl], rows[~gl]
                for side, crow, wside, arr in ((0, lrows, dd["wl"], cl), (1, rrows, dd["wr"], cr)):
                    active = d + 1 < D and wside >= 2.0 * p.min_w and act < cap_next
                    if d + 1 < D and wside >= 2.0 * p.min_w:
                        act += 1
                    if active:
                        arr[i] = len(nxt); nxt.append(crow)
                        nxt_ok.append(None if self.ic_map is None else level_ok[i] & self.ic_map[dd["feat"]])
                        if ranges:
                            num = not dd["is_cat"] and int(dd["bin"]) != NA_BIN
                            nxt_vr.append(self._value_ranges(level_occ[i], (int(dd["feat"]), int(dd["bin"]))
                                                             if num else None, side))
                    else:
                        lid = n_leaves; n_leaves += 1
                        arr[i] = -1 - lid
                        leaf_of_row[crow] = lid
                        leafsum.append((aux[crow, 2].astype(np.float64).sum(), aux[crow, 3].astype(np.float64).sum()))
            decs.append(dl); cls.append(cl); crs.append(cr)
            level_rows = nxt
            level_ok = nxt_ok
            level_vr = nxt_vr if ranges else [None] * len(nxt)
            if not nxt:
                break
        res = TreeLevels(decs, cls, crs, n_leaves)
        res.root_weight = float(aux[:, 0].astype(np.float64).sum())
        self.leafsum = torch.tensor(np.array(leafsum, dtype=np.float64).reshape(-1, 2))
        if coll.is_dist():
            coll.all_reduce_(self.leafsum)
            res.root_weight = coll.all_reduce_scalar(res.root_weight)
        self.leaf_of_row = torch.from_numpy(leaf_of_row.astype(np.int32))
        if leaf_fn is not None:
            res.leaf_values = leaf_fn(self.leafsum).to(torch.float32).cpu().numpy()
        if not hasattr(self, "history"):
            self.history = []
        self.history.append(res)
        return len(self.history) - 1

    def pop_levels(self, ready_only: bool = False) -> list:
        """Built trees in build order (the reference builder is synchronous: all are ready)."""
        out = list(getattr(self, "history", []))
        self.history = []
        return out


# ================================================================================================
_MAXL = 65
_SNAP_KERNEL = os.environ.get("H2O_SNAP_KERNEL", "1") != "0"
_vp, _ci, _cd = ctypes.c_void_p, ctypes.c_int, ctypes.c_double


class _TreePlan(ctypes.Structure):
    """Mirror of ``TreePlan`` in ``csrc/tree_kernels.hip`` (native per-tree launch sequence)."""
    _fields_ = ([("N", ctypes.c_longlong)] +
                [(n, _ci) for n in ("stride", "F", "D", "slot", "used", "pf32", "grid", "leaf_cap", "mode",
                                    "random_split", "unit")] +
                [(n, _cd) for n in ("min_w", "msi", "lam", "alpha", "gamma")] +
                [(n, _vp) for n in ("master", "partials", "hist0", "hist1", "hbuild", "cand", "scratch", "nbins_f",
                                    "iscat_f", "mono_f", "qs", "leafsum", "leaf_of_row", "counters", "rootw",
                                    "leafval", "leafq", "lvptrs")] +
                [(n, _vp * 2) for n in ("bb", "by", "bw")] +
                [(n, _vp * _MAXL) for n in ("nodes", "meta", "tp", "bp", "dec", "cl", "cr", "nl", "cur")] +
                [("caps", _ci * _MAXL), ("tiles_cap", _ci * _MAXL)] +
                [(n, _vp) for n in ("aux", "amax_bits", "feat_ok")] +
                [(n, _ci) for n in ("compute_amax", "k_cols", "packed", "leaf_native", "log_link", "hist_type")] +
                [("seed", ctypes.c_ulonglong)] + [(n, _cd) for n in ("scale", "kclamp", "mx")] +
                [("kc_level", _ci * _MAXL), ("pad2", _ci)] +
                [("edges", _vp), ("nb_level", _ci * _MAXL), ("pad3", _ci)] +
                [("ic_map", _vp), ("ic", _vp * _MAXL)] +
                [(n, _ci) for n in ("sliced", "fs0", "fsn", "sslot")] + [("cand_local", _vp), ("hrecv", _vp)] +
                [("leaf_lam", _cd), ("leaf_l1", _cd)] + [("planar", _ci), ("no_na", _ci)] +
                [("fgroup", _vp)] + [("coll_fn", _vp), ("coll_ctx", _vp)] +
                [(n, _ci) for n in ("W", "cf32", "cand_fs", "dist")] + [(n, _vp) for n in ("hsend", "cand_all", "lsx")] +
                [("fine_f", _vp)] + [(n, _ci) for n in ("lo_F", "lo_from", "mid_F", "mid_from")] + [("lvl2", _vp), ("fdir", _vp)] +
                [("num_plane", _ci), ("pad4", _ci)] +
                [(n, _vp) for n in ("fine16", "f16col", "f16n")] + [("f16_planes", _ci), ("pad5", _ci)] +
                [("vrange", _vp), ("range_on", _ci), ("pad6", _ci)] + [("gcat", _vp)])


class _Arena:
    """One device allocation holding every small per-level array (copied to host in one shot)."""

    def __init__(self):
        self.off = 0
        self.items = []

    def add(self, name, nbytes):
        self.items.append((name, self.off, nbytes))
        self.off += (nbytes + 255) // 256 * 256
        return name


class GpuTreeBuilder:
    """Drives the HIP tree kernels. ``bins`` is a CUDA uint8 tensor [N, stride] (stride % 4 == 0).

    Row statistics arrive as four planes (``aux`` [4, N] with ``soa=True``, or the [N, 4] row-major form of
    the CPU reference, transposed here): w, wY (histograms), gamma numerator / denominator (leaf sums).
    The routed row payload is the bins plus wY (plus w unless ``unit``: every row weight is exactly 1); the
    leaf of every row and the leaf sums come from one pass over the ORIGINAL row order after the last level
    (k_leaf_assign), so rows carry no index and stop moving once they reach a leaf."""

    def __init__(self, bins: torch.Tensor, F: int, nbins_f, iscat_f, mono_f, max_depth: int, params: SplitParams,
                 node_cap: int = 1 << 14, grid: int = 256):
        assert bins.is_cuda and bins.dtype == torch.uint8 and bins.dim() in (2, 3)
        # > 32 features: PLANAR bins [stride / 32, N, 32] (apply_binning(planar=True)); a row-major [N, stride]
        # input with whole 32-byte planes is converted once (H2O_BINS_ROWMAJOR=1 keeps row-major: A/B runs)
        if bins.dim() == 2 and bins.shape[1] >= 64 and bins.shape[1] % 32 == 0 and \
                os.environ.get("H2O_BINS_ROWMAJOR") != "1":
            bins = bins.view(bins.shape[0], bins.shape[1] // 32, 32).permute(1, 0, 2).contiguous()
        self.planar = bins.dim() == 3
        if self.planar:
            assert bins.shape[2] == 32 and bins.shape[0] >= 2
        self.lib = nat.hip()
        sz = np.zeros(16, dtype=np.int32)
        self.lib.h2o_tree_sizes(sz.ctypes.data)
        assert sz[0] == NODE_DT.itemsize and sz[1] == DEC_DT.itemsize and sz[2] == CAND_BYTES, sz
        assert sz[7] == AMAX_SHARDS, sz
        self.TILE = int(sz[3])
        dev = bins.device
        self.dev = dev
        if self.planar:
            self.N, self.stride = bins.shape[1], bins.shape[0] * 32
        else:
            self.N, self.stride = bins.shape
        assert self.stride % 4 == 0
        self.F = F
        self.D = D = max(1, int(max_depth))
        if D >= _MAXL - 1:
            raise ValueError(f"max_depth {D} exceeds the native tree plan ({_MAXL - 2})")
        self.p = params
        self.grid = int(os.environ.get("H2O_HIST_GRID", grid))
        grid = self.grid
        # fp32 per-block partial histograms (half the flush + reduce bytes; the reduce sums in fp64)
        # MEASURED (scripts/gpu_small_shard_sweep.sh): 0.511 -> 0.492 ms/tree at 1.375M rows and 0.718 -> 0.707
        # at 2.75M (the per-rank shards of an 8/4-GPU HIGGS run); r5, after the vectorized flush, also at 11M:
        # 1.262-1.268 -> 1.244-1.253 ms/tree, same trees (scripts/gpu_r5_c13.sh). Small test shards keep fp64.
        self.pf32 = int(os.environ.get("H2O_PARTIAL_F32", "1" if self.N >= 1_000_000 else "0"))
        self.master = bins
        N, T = self.N, self.TILE
        self.caps = [min(1 << d, node_cap) for d in range(D)] + [1]
        capmax = max(self.caps)
        self.used = F * 2 * NBIN + F + 1      # doubles of a node histogram slot actually written
        self.slot = self.used + (self.used & 1)
        self.hist = [torch.empty(capmax * self.slot, dtype=torch.float64, device=dev) for _ in range(2)]
        # compact histograms of the BUILT children of a level, slot = parent index (<= caps[d] slots):
        # the only histogram bytes a row-sharded run all-reduces per level
        self.hbuild = torch.empty(max(self.caps[:D]) * self.slot, dtype=torch.float64, device=dev)
        # per-block partial histograms of one level (k_hist_build -> k_hist_reduce): G + nodes slots
        # (packed histograms fit two blocks per CU; H2O_HIST_BPC=2 launches hist_bpc * grid blocks)
        # measured: 2 is 3-14 % slower; again with the barrier-free filtered pass (round 3): 11M 1.34 -> 1.40,
        # 1.375M 0.423 -> 0.474 ms/tree (the doubled partial slots cost more than the extra waves gain)
        self.hist_bpc = int(os.environ.get("H2O_HIST_BPC", "1"))
        # (zeroed: narrow levels leave the partial entries of columns they do not build untouched)
        self.partials = torch.zeros((self.hist_bpc * grid + capmax) * self.slot, dtype=torch.float64, device=dev)
        self.tiles_cap = [(N + T - 1) // T + c for c in self.caps]
        self.cand = torch.empty(capmax * F * CAND_BYTES, dtype=torch.uint8, device=dev)
        self.scratch = torch.empty(2 * capmax + 16, dtype=torch.int32, device=dev)
        self.leaf_cap = min(N + 1, 2 * sum(self.caps) + 2)
        self.leafsum = torch.zeros(self.leaf_cap, 2, dtype=torch.float64, device=dev)
        # fixed-point leaf sums, LEAFQ_STRIPES copies (blocks spread their flush atomics over them)
        self.leafq = torch.zeros(int(sz[8]) * self.leaf_cap * 2, dtype=torch.int64, device=dev)
        self.leaf_of_row = torch.empty(N, dtype=torch.int32, device=dev)
        self.nbins_f = torch.as_tensor(np.asarray(nbins_f, dtype=np.int32), device=dev)
        self.iscat_f = torch.as_tensor(np.asarray(iscat_f, dtype=np.int32), device=dev)
        self.iscat_np = np.asarray(iscat_f, dtype=np.int32)
        self.fine_f = None
        self.n_low = self.n_mid = 0
        self.mono_f = None if mono_f is None else torch.as_tensor(np.asarray(mono_f, dtype=np.int32), device=dev)
        self.feat_ok_all = torch.ones(F, dtype=torch.int32, device=dev)
        self.qs = torch.zeros(16, dtype=torch.float64, device=dev)  # fixed-point scales (k_qscale)
        self.amax_bits = torch.zeros(4 * AMAX_SHARDS, dtype=torch.int32, device=dev)
        self._soa = None                       # [4, N] staging of row-major aux input
        # ping-pong row payload buffers: bins + wY (+ w for weighted rows, allocated on first use)
        self.bufs = [dict(bins=torch.empty(N * self.stride, dtype=torch.uint8, device=dev),
                          y=torch.empty(N, dtype=torch.float32, device=dev), w=None) for _ in range(2)]
        # small per-level arrays in one arena
        ar = _Arena()
        for d in range(D + 1):
            c = self.caps[d]
            ar.add(f"nodes{d}", c * NODE_DT.itemsize)
            ar.add(f"meta{d}", 16)                 # [n_nodes, n_tiles, n_build_tiles, pad]
            ar.add(f"tp{d}", (c + 1) * 4)
            ar.add(f"bp{d}", (c + 1) * 4)          # tile prefix over build (histogrammed) nodes only
            ar.add(f"dec{d}", c * DEC_DT.itemsize)
            ar.add(f"cl{d}", c * 4)
            ar.add(f"cr{d}", c * 4)
            ar.add(f"nl{d}", c * 4)                # even levels: rows going left (filled by the odd-level histogram)
            ar.add(f"cur{d}", c * 16)              # odd levels: region cursors {front, back, start, end}
        ar.add("counters", 16)
        ar.add("rootw", 8)
        ar.add("leafval", self.leaf_cap * 4)
        self.arena = torch.zeros(ar.off, dtype=torch.uint8, device=dev)
        self.av = {}
        self._off = {}
        for name, off, nb in ar.items:
            self.av[name] = self.arena[off:off + nb]
            self._off[name] = (off, nb)
        # level-0 constants
        n_tiles0 = (N + T - 1) // T
        root = np.zeros(1, dtype=NODE_DT)
        root[0] = (0, N, 1, -1, -1, 0, 0, 0)
        self.av["nodes0"].copy_(torch.from_numpy(root.view(np.uint8)))
        self.av["meta0"].copy_(torch.from_numpy(np.array([1, n_tiles0, n_tiles0, 0], dtype=np.int32).view(np.uint8)))
        self.av["tp0"][:8].copy_(torch.from_numpy(np.array([0, n_tiles0], dtype=np.int32).view(np.uint8)))
        self.av["bp0"][:8].copy_(torch.from_numpy(np.array([0, n_tiles0], dtype=np.int32).view(np.uint8)))
        self.history = []       # (pinned host snapshot, copy-done event) per built tree, in build order
        # snapshot buffers allocated up front: a pinned allocation (hipHostMalloc) inside the tree loop stalls the
        # host for milliseconds and serialises with the device (MEASURED r5: one 7.4 ms build at 1.375M rows)
        npre = int(os.environ.get("H2O_TREE_SNAP_POOL", "8")) if dev.type == "cuda" else 0
        self._pinned_pool = [torch.empty(self.arena.numel(), dtype=torch.uint8, pin_memory=True) for _ in range(npre)]
        self._event_pool = [torch.cuda.Event() for _ in range(npre)]
        self._decoded = []      # trees decoded early by a bounded-lookahead wait (_snapshot), handed out first
        self._snap_wait = npre > 0 and os.environ.get("H2O_TREE_SNAP_WAIT", "1") == "1"
        # raw device pointers resolved once: the per-tree launch sequence is ~45 ctypes calls and at small
        # shards (1.375M rows/GPU) the host loop, not the GPU, set the pace (82 % busy, rocprofv3 trace)
        self._pt = {name: t.data_ptr() for name, t in self.av.items()}
        # per-level (dec, cl, cr, cap) records for the leaf traversal (k_leaf_assign)
        self.lvptrs = torch.tensor([[self._pt[f"dec{d}"], self._pt[f"cl{d}"], self._pt[f"cr{d}"], self.caps[d]]
                                    for d in range(D)],
                                   dtype=torch.int64).reshape(-1).to(dev)
        self.ic_map = None
        self._hp = [h.data_ptr() for h in self.hist]
        self._init_comm(capmax)

    def _init_comm(self, capmax: int):
        """Row-sharded histogram exchange (reference: ScoreBuildHistogram2 + MRTask reduce), run by the native
        driver ``h2o_tree_dist``: one host call per tree enqueues every kernel and collective on the stream.

        ``H2O_TREE_COMM=ar`` (default): each level's built-node histograms are ALL-REDUCED, every rank searches
        every feature of the same global histograms — one collective per level (the exchange is latency-bound:
        a depth-6 HIGGS tree moves 32 histogram slots, 3.7 MB in fp64, in 6 level collectives).
        ``rs``: feature-sliced — the histograms are packed by feature slice (k_hist_pack) and REDUCE-SCATTERED, so
        every rank holds the global histograms of F/W features only and searches that slice; the per-(node,
        feature) candidates are ALL-GATHERED (a few KB, read in place rank-major) — two collectives per level,
        1/W of the split search each. Both end with one all-reduce of the leaf sums (+ the root weight).
        Wire dtype ``H2O_TREE_COMM_DTYPE``: ``f64`` (default; decisions equal the single-process ones, exact
        ties included) or ``f32`` (half the bytes; a tie between two equal-gain splits may break differently).

        Transport: RCCL from C++ when the process group runs ``nccl`` (:class:`parallel.rccl.NativeComm`), else
        the same driver with host-staged callbacks (:class:`parallel.rccl.HostTransport`, gloo).
        ``H2O_TREE_COMM_FORCE=ar|rs`` runs the row-sharded driver at world size 1 (a 1-rank RCCL communicator):
        the 1-GPU rehearsal of the multi-GPU path."""
        force = os.environ.get("H2O_TREE_COMM_FORCE", "")
        self.dist_mode = coll.is_dist() or force in ("rs", "ar")
        self.W = coll.world() if coll.is_dist() else 1
        mode = force if force in ("rs", "ar") else os.environ.get("H2O_TREE_COMM", "ar")
        self.sliced = self.dist_mode and mode == "rs"
        self.cf32 = int(self.dist_mode and os.environ.get("H2O_TREE_COMM_DTYPE", "f64") == "f32")
        self.fs = self.fs0 = self.fsn = 0
        self.sslot = self.slot
        self.transport = None
        if not self.dist_mode:
            return
        W, F, dev = self.W, self.F, self.dev
        wire = torch.float32 if self.cf32 else torch.float64
        self.hsend = self.cand_local = self.cand_all = self.lsx = None
        if self.sliced:
            self.fs = Fs = (F + W - 1) // W
            self.fs0 = min(F, coll.rank() * Fs)
            self.fsn = max(0, min(F, self.fs0 + Fs) - self.fs0)
            self.sslot = Fs * 2 * NBIN + Fs + 1
            self.hsend = torch.empty(W * capmax * self.sslot, dtype=wire, device=dev)
            self.cand_local = torch.zeros(capmax * Fs * CAND_BYTES, dtype=torch.uint8, device=dev)
            self.cand_all = torch.zeros(W * capmax * Fs * CAND_BYTES, dtype=torch.uint8, device=dev)
            # leaf sums + the root weight (written by the owner of feature 0) in one all-reduce
            self.lsx = torch.zeros(self.leaf_cap * 2 + 1, dtype=torch.float64, device=dev)
        else:
            self.sslot = self.used            # exchanged slots hold the used values of a slot
        self.hrecv = torch.empty(capmax * self.sslot, dtype=wire, device=dev)
        from ..parallel import rccl
        comm = rccl.native_comm(force=bool(force))
        if comm is not None:
            self.transport = comm
        else:
            bufs = [self.hist[0], self.hbuild, self.leafsum, self.hsend, self.hrecv, self.cand_local,
                    self.cand_all, self.lsx]
            self.transport = rccl.HostTransport(bufs)

    def comm_per_tree(self) -> tuple:
        """(collectives, bytes handed to them) of one row-sharded tree of full depth (the driver's sequence is
        fixed: levels past the last split run on empty node lists)."""
        D, W = self.D, self.W
        if not self.dist_mode:
            return 0, 0
        es = 4 if self.cf32 else 8
        slots = [1] + self.caps[:D - 1]
        if self.sliced:
            rs = sum(W * n * self.sslot * es for n in slots)
            ag = sum(self.caps[d] * self.fs * CAND_BYTES for d in range(D))
            return len(slots) + D + 1, rs + ag + (self.leaf_cap * 2 + 1) * 8
        return len(slots) + 1, sum(n * self.sslot * es for n in slots) + self.leaf_cap * 2 * 8

    def _p(self, name):
        return self._pt[name]

    def set_interaction_constraints(self, ic_map, root_ok):
        """Per-node allowed features (GlobalInteractionConstraints): ``ic_map`` [F, F] uint8, row f = the
        features allowed to interact with f; ``root_ok`` [F]. Level masks [caps[d], F] live on the device and
        are propagated by k_ic_next after each plan."""
        F, dev = self.F, self.dev
        self.ic_map = torch.as_tensor(np.asarray(ic_map, dtype=np.uint8), device=dev).contiguous()
        self.ic_lv = [torch.zeros(self.caps[d] * F, dtype=torch.uint8, device=dev) for d in range(self.D + 1)]
        self.ic_lv[0][:F].copy_(torch.as_tensor(np.asarray(root_ok, dtype=np.uint8), device=dev))
        if getattr(self, "_plan", None) is not None:
            self._set_plan_ic(self._plan)

    def set_feature_groups(self, fgroup, n_low: int = 0, n_mid: int = 0):
        """Engine column -> original feature (k_split_reduce column sampling by original feature); ``n_low`` /
        ``n_mid``: leading columns of the narrow views (:func:`narrow_cut`)."""
        enc = encode_groups(fgroup)
        self.fgroup = None if enc is None else torch.as_tensor(enc, device=self.dev).contiguous()
        self._fgroup_np = None if fgroup is None else np.asarray(fgroup, dtype=np.int64)
        self._fine16 = None
        self.fine_f = fine_columns(fgroup, self.iscat_np, self.F)
        if self.fine_f is not None:
            self.fine_f = torch.as_tensor(self.fine_f, device=self.dev).contiguous()
        self.n_low, self.n_mid = int(n_low), int(n_mid)
        if getattr(self, "_plan", None) is not None:
            self._plan.fgroup = 0 if self.fgroup is None else self.fgroup.data_ptr()
            self._plan.fine_f = 0 if self.fine_f is None else self.fine_f.data_ptr()
            self._set_plan_narrow(self._plan)
            self._set_plan_fine16(self._plan)

    def set_cat_groups(self, gcat):
        """Wide-categorical groups (Binning.gcat, see RefTreeBuilder.set_cat_groups): k_split_find's group path."""
        if gcat is not None and self.sliced:
            raise ValueError("wide-categorical groups need the all-reduce histogram exchange (H2O_TREE_COMM=ar): a "
                             "feature slice could cut a group")
        self.gcat_np = None if gcat is None else np.asarray(gcat, dtype=np.int32)
        self.gcat = None if gcat is None else torch.as_tensor(self.gcat_np, device=self.dev).contiguous()
        if getattr(self, "_plan", None) is not None:
            self._plan.gcat = 0 if self.gcat is None else self.gcat.data_ptr()

    def _set_plan_narrow(self, P):
        mid, lo = narrow_cut(self.p, self.n_low, self.n_mid, self.F)
        P.lo_F, P.lo_from = (self.n_low, lo) if lo >= 0 else (0, 0)
        P.mid_F, P.mid_from = (self.n_mid, mid) if mid >= 0 else (0, 0)
        # every row's level-2 position from the root route (the leaf walk starts there; narrow planar runs only)
        # and the root split's side of every row (level 1 reads these bytes instead of the split column's plane)
        # H2O_ROW_DIR_PLANAR=1: planar runs of >= 2 planes (e.g. XGBoost 100M x 50) also get the root split's side as
        # bytes for level 1. MEASURED r5 (scripts/gpu_r5_c30.sh): 17.48-17.75 vs 17.53 ms/tree — the second plane's
        # read of the split column hits the caches; off by default
        wide = self.planar and self.F > 32 and os.environ.get("H2O_ROW_DIR_PLANAR", "0") == "1"
        if (lo >= 0 and self.planar) or wide:
            if getattr(self, "_fdir", None) is None:
                self._fdir = torch.empty(self.N, dtype=torch.uint8, device=self.dev)
            if lo >= 0 and getattr(self, "_lvl2", None) is None:
                self._lvl2 = torch.empty(self.N, dtype=torch.uint8, device=self.dev)
        on = lo >= 0 and self.planar
        P.lvl2 = self._lvl2.data_ptr() if on else 0
        P.fdir = self._fdir.data_ptr() if (on or wide) else 0

    def _fine16_map(self):
        """Slot maps of the root pass from 16-bit fine planes (k_hist_root16), or None when it does not apply: the
        wide-bin layout (several engine columns per numeric feature holding the interleaved edge subsets e[k::n]),
        planar bins, at most 4 columns per feature and 64 features, no wide categorical. Returns (cslot [planes*32],
        fcol [slots][4], fn [slots], nslot); slots are the original features in first-column order, a feature's
        columns ordered by subset k (= by first edge)."""
        if os.environ.get("H2O_HIST_ROOT16", "1") == "0" or not self.planar or self.dev.type != "cuda":
            return None
        fg = getattr(self, "_fgroup_np", None)
        if fg is None or not (self.n_low or self.n_mid) or self.p.edges is None:
            return None
        F = self.F
        edges = np.asarray(self.p.edges, dtype=np.float32)
        order, cols = [], {}
        for c in range(F):
            g = int(fg[c])
            if g not in cols:
                cols[g] = []
                order.append(g)
            cols[g].append(c)
        nslot = len(order)
        if nslot > 64:
            return None
        ns = (nslot + 15) // 16 * 16
        cslot = np.full(self.master.shape[0] * 32, -1, dtype=np.int32)
        fcol = np.full((ns, 4), -1, dtype=np.int32)
        fn = np.zeros(ns, dtype=np.int32)
        for s_, g in enumerate(order):
            cs = cols[g]
            if len(cs) > 4 or (len(cs) > 1 and any(int(self.iscat_np[c]) for c in cs)):
                return None
            cs = sorted(cs, key=lambda c: float(edges[c, 0]))      # subset k holds edge k first
            fcol[s_, :len(cs)] = cs
            fn[s_] = len(cs)
            cslot[cs] = s_
        return cslot, fcol, fn, nslot

    def _set_plan_fine16(self, P):
        P.fine16 = P.f16col = P.f16n = 0
        P.f16_planes = 0
        m = self._fine16_map()
        if m is None:
            return
        cslot, fcol, fn, nslot = m
        dev = self.dev
        if getattr(self, "_fine16", None) is None:
            planes16 = (nslot + 15) // 16
            self._f16_cslot = torch.as_tensor(cslot, device=dev)
            self._f16col = torch.as_tensor(fcol.reshape(-1), device=dev)
            self._f16n = torch.as_tensor(fn, device=dev)
            self._fine16 = torch.empty(planes16 * self.N * 16, dtype=torch.int16, device=dev)
            nat.call("h2o_fine16_build", self.master.data_ptr(), int(self.master.shape[0]), self.N,
                     self._f16_cslot.data_ptr(), nslot, self._fine16.data_ptr(), nat.stream_ptr(dev))
            self._f16_planes = planes16
        P.fine16, P.f16col, P.f16n = self._fine16.data_ptr(), self._f16col.data_ptr(), self._f16n.data_ptr()
        P.f16_planes = self._f16_planes

    def _set_plan_ic(self, P):
        if self.ic_map is None:
            P.ic_map = 0
            return
        P.ic_map = self.ic_map.data_ptr()
        for d in range(self.D + 1):
            P.ic[d] = self.ic_lv[d].data_ptr()

    def _make_plan(self):
        """Static part of the native launch plan (pointers / shapes fixed for the builder's lifetime)."""
        assert self.lib.h2o_tree_plan_size() == ctypes.sizeof(_TreePlan), "TreePlan layout mismatch"
        P = _TreePlan()
        p = self.p
        P.N, P.stride, P.F, P.D, P.slot, P.used, P.pf32 = self.N, self.stride, self.F, self.D, self.slot, self.used, self.pf32
        P.leaf_cap, P.mode, P.random_split = self.leaf_cap, int(p.mode), int(p.random_split)
        P.min_w, P.msi, P.lam, P.alpha, P.gamma = p.min_w, p.min_split_improvement, p.lam, p.alpha, p.gamma
        P.master, P.partials = self.master.data_ptr(), self.partials.data_ptr()
        P.hist0, P.hist1, P.hbuild = self._hp[0], self._hp[1], self.hbuild.data_ptr()
        P.cand, P.scratch = self.cand.data_ptr(), self.scratch.data_ptr()
        P.nbins_f, P.iscat_f = self.nbins_f.data_ptr(), self.iscat_f.data_ptr()
        P.mono_f = 0 if self.mono_f is None else self.mono_f.data_ptr()
        P.qs, P.leafsum, P.leaf_of_row = self.qs.data_ptr(), self.leafsum.data_ptr(), self.leaf_of_row.data_ptr()
        P.leafq, P.lvptrs = self.leafq.data_ptr(), self.lvptrs.data_ptr()
        P.counters, P.rootw, P.leafval = self._p("counters"), self._p("rootw"), self._p("leafval")
        for i in range(2):
            P.bb[i], P.by[i] = self.bufs[i]["bins"].data_ptr(), self.bufs[i]["y"].data_ptr()
            P.bw[i] = 0
        for d in range(self.D + 1):
            for n in ("nodes", "meta", "tp", "bp", "dec", "cl", "cr", "nl", "cur"):
                getattr(P, n)[d] = self._p(f"{n}{d}")
            P.caps[d], P.tiles_cap[d] = self.caps[d], self.tiles_cap[d]
        P.edges = self._edges_ptr()
        for d in range(_MAXL):
            P.nb_level[d] = p.adapt_nb(d) if P.edges else 0
        P.hist_type = int(p.hist_type)
        # the reference's node ranges (SplitParams.parent_range): exact column extremes on the device
        if P.edges and p.vrange is not None and p.parent_range and p.hist_type != HT_QUANTILES:
            self._vrange_dev = torch.as_tensor(np.asarray(p.vrange, dtype=np.float32).reshape(-1),
                                               device=self.dev).contiguous()
            P.vrange, P.range_on = self._vrange_dev.data_ptr(), 1
        else:
            P.vrange, P.range_on = 0, 0
        self._set_plan_ic(P)
        fg = getattr(self, "fgroup", None)
        P.fgroup = 0 if fg is None else fg.data_ptr()
        gc = getattr(self, "gcat", None)
        P.gcat = 0 if gc is None else gc.data_ptr()
        P.fine_f = 0 if self.fine_f is None else self.fine_f.data_ptr()     # used only under H2O_HIST_FINE=1
        self._set_plan_narrow(P)
        self._set_plan_fine16(P)
        P.sliced, P.fs0, P.fsn, P.sslot = int(self.sliced), self.fs0, self.fsn, self.sslot
        P.planar = int(self.planar)
        P.no_na = int(self._no_na())
        P.cand_local = self.cand_local.data_ptr() if self.sliced else 0
        P.hrecv = self.hrecv.data_ptr() if self.dist_mode else 0
        P.W, P.cf32, P.cand_fs, P.dist = self.W, self.cf32, self.fs, int(self.dist_mode)
        if self.sliced:
            P.hsend, P.cand_all, P.lsx = self.hsend.data_ptr(), self.cand_all.data_ptr(), self.lsx.data_ptr()
        if self.transport is not None:
            P.coll_fn, P.coll_ctx = self.transport.fn, self.transport.ctx
        return P

    def _no_na(self) -> bool:
        """True when no feature byte of the bins is the NA bin: the histogram loop then skips its per-word NA
        test (rows are only permuted between levels, so the property holds for every level's buffer)."""
        b, F = self.master, self.F
        if b.numel() == 0:
            return True
        hit = torch.zeros((), dtype=torch.bool, device=b.device)
        step = 1 << 24
        if self.planar:
            for pl in range(b.shape[0]):
                nf = min(32, F - 32 * pl)
                if nf <= 0:
                    break
                for r0 in range(0, b.shape[1], step):
                    hit |= (b[pl, r0:r0 + step, :nf] == NA_BIN).any()
        else:
            for r0 in range(0, b.shape[0], step):
                hit |= (b[r0:r0 + step, :F] == NA_BIN).any()
        return not bool(hit)

    def _edges_ptr(self):
        if self.p.edges is None or not self.p.adapt_nbins:
            return 0
        if getattr(self, "_edges_dev", None) is None:
            self._edges_dev = torch.as_tensor(np.asarray(self.p.edges, dtype=np.float32), device=self.master.device).contiguous()
        return self._edges_dev.data_ptr()

    def _planes(self, aux: torch.Tensor, soa: bool) -> torch.Tensor:
        """[4, N] float32 planes of the row statistics (row-major [N, 4] input is transposed once)."""
        if soa:
            assert aux.shape == (4, self.N) and aux.dtype == torch.float32 and aux.is_contiguous()
            return aux
        assert aux.shape == (self.N, 4) and aux.dtype == torch.float32
        if self._soa is None:
            self._soa = torch.empty(4, self.N, dtype=torch.float32, device=self.dev)
        self._soa.copy_(aux.t())
        return self._soa

    def build(self, aux_static: torch.Tensor, feat_ok: torch.Tensor | None = None, k_cols: int = 0, seed: int = 0,
              leaf_fn=None, amax_bits: torch.Tensor | None = None, packed: bool | int = False, leaf_native=None,
              soa: bool = False, unit: bool = False, num_plane: int = 2):
        """Launch one tree (one host call single-process; one per collective segment row-sharded).
        ``leaf_fn(leafsum[L,2] f64) -> leaf values f32`` runs on device before the arena snapshot, so values
        travel to the host with the structure (no extra sync); ``leaf_native = (log_link, scale, kclamp,
        max_abs)`` instead computes closed-form Newton leaf values in one HIP launch (k_leaf_values).
        ``amax_bits`` (int32[4*AMAX_SHARDS], max |plane| as float bits) may be produced by a fused prepare
        kernel; otherwise it is computed here. ``packed`` (caller guarantees w is a 0/1 or small integer row
        weight) switches the LDS histograms to one packed count|wY atomic per (row, feature), ``packed=2`` (float
        weights, XGBoost hessians) to the 32/32 fixed-point hessian|wY word (FPACK, k_qscale scales); ``unit``
        (every w is exactly 1) drops w from the row payload altogether."""
        if not hasattr(self, "_plan"):
            self._plan = self._make_plan()
        planes = self._planes(aux_static, soa)
        lib, P = self.lib, self._plan
        s = nat.stream_ptr(self.dev)
        P.aux = planes.data_ptr()
        P.unit = int(bool(unit))
        P.num_plane = int(num_plane) if soa else 2
        if not unit:
            for i in range(2):
                if self.bufs[i]["w"] is None:
                    self.bufs[i]["w"] = torch.empty(self.N, dtype=torch.float32, device=self.dev)
                P.bw[i] = self.bufs[i]["w"].data_ptr()
        P.compute_amax = int(amax_bits is None)
        P.amax_bits = (self.amax_bits if amax_bits is None else amax_bits).data_ptr()
        P.feat_ok = (self.feat_ok_all if feat_ok is None else feat_ok).data_ptr()
        P.k_cols, P.packed, P.seed = _level_k(k_cols, 0), (2 if packed == 2 else int(bool(packed))), int(seed) & _M64
        for d in range(_MAXL):
            P.kc_level[d] = _level_k(k_cols, d) if isinstance(k_cols, (list, tuple)) else 0
        P.grid = self.grid * (self.hist_bpc if packed else 1)
        P.leaf_native = int(leaf_native is not None)
        if leaf_native is not None:
            lg, scale, kclamp, mx = leaf_native[:4]
            lam, l1 = (tuple(leaf_native[4:6]) + (0.0, 0.0))[:2]
            P.log_link, P.scale, P.kclamp, P.mx = int(lg), float(scale), float(kclamp), float(mx)
            P.leaf_lam, P.leaf_l1 = float(lam), float(l1)
        ref = ctypes.byref(P)
        if not self.dist_mode:
            if self._graph_replay(P, k_cols):
                pass
            else:
                nat.check(lib.h2o_tree_all(ref, s), "tree_all")
        else:
            rc = lib.h2o_tree_dist(ref, s)
            err = getattr(self.transport, "error", None)
            if err is not None:
                self.transport.error = None
                raise RuntimeError(f"tree collective failed: {err}") from err
            nat.check(rc, "tree_dist")
            if isinstance(self.transport, _native_comm_cls()):   # (host transport counts its own calls)
                coll.add_stats(*self.comm_per_tree())
        if leaf_native is None and leaf_fn is not None:
            vals = leaf_fn(self.leafsum)
            self.av["leafval"].view(torch.float32)[: vals.numel()].copy_(vals.to(torch.float32))
        return self._snapshot()

    # ---- hipGraph replay of the per-tree launch sequence (single process)
    def _seed_used(self, P, k_cols) -> bool:
        """Does any kernel of the tree read the seed? (column sampling, random splits, Random / RoundRobin lattices)"""
        ht = int(self.p.hist_type)
        return (bool(P.k_cols) or any(int(v) for v in P.kc_level) or bool(P.random_split)
                or (bool(P.edges) and ht in (HT_RANDOM, HT_ROUND_ROBIN)))

    def _graph_replay(self, P, k_cols) -> bool:
        """The whole tree as ONE hipGraph launch: the native sequence (h2o_tree_all, ~30 kernels) is captured once
        into a torch.cuda.CUDAGraph and replayed for every tree whose launch plan is byte-identical (kernel arguments
        are baked in at capture: the plan struct is the signature; the seed only when a kernel reads it). Up to 16 plans
        keep their graphs (the K classes of a multinomial model share one); a plan that changes every tree (e.g. learn_rate_annealing in the
        leaf values) stops the capture after 16 new signatures without a replay.
        ``H2O_TREE_GRAPH=0``: direct launches."""
        if self.dev.type != "cuda" or os.environ.get("H2O_TREE_GRAPH", "1") == "0" or self.__dict__.get("_graph_off"):
            return False
        seed = P.seed
        if not self._seed_used(P, k_cols):
            P.seed = 0
        sig = bytes(P)
        P.seed = seed
        # one graph per plan signature (plans that alternate between trees keep theirs): up to _GRAPH_CACHE of them;
        # a run of new signatures with no replay in between (the plan changes every tree) turns capture off
        cache = self.__dict__.setdefault("_graphs", {})
        g = cache.get(sig)
        if g is None:
            misses = self.__dict__.get("_graph_misses", 0) + 1
            self._graph_misses = misses
            if misses > _GRAPH_CACHE:
                self._graph_off = True
                cache.clear()
                return False
            g = torch.cuda.CUDAGraph()
            try:
                with torch.cuda.graph(g, capture_error_mode="thread_local"):
                    rc = self.lib.h2o_tree_all(ctypes.byref(P), nat.stream_ptr(self.dev))
            except Exception:          # noqa: BLE001 - capture refused by the runtime: launch directly from now on
                self._graph_off = True
                cache.clear()
                return False
            nat.check(rc, "tree_all (capture)")
            if len(cache) >= _GRAPH_CACHE:
                cache.pop(next(iter(cache)))
            cache[sig] = g
        else:
            self._graph_misses = 0
        g.replay()
        return True

    def _snapshot(self):
        # the tree's structure travels to pinned host memory asynchronously: the host decodes finished
        # trees (pop_levels(ready_only=True)) while the GPU builds the next ones. MEASURED: moving the
        # device-to-host copy to a side stream (device staging ring + stream events) made the host block
        # in the launches (820 us/tree host, 1.09 vs 0.575 ms/tree at 1.375M rows): kept on the compute stream
        if not self._pinned_pool and self.history and self._snap_wait:
            # bounded lookahead: the host is a whole pool of trees ahead of the GPU. Wait for the OLDEST tree
            # (the GPU still has the rest of the pool queued, so it does not idle) and decode it now, instead of
            # a pinned allocation (hipHostMalloc serialises with the device: a GPU gap per tree once the host runs
            # ahead — profiles/r6_final_tree_timeline_1375000.md). H2O_TREE_SNAP_WAIT=0: allocate as before.
            self._decoded.extend(self._pop(1))
        host = self._pinned_pool.pop() if self._pinned_pool else torch.empty(self.arena.numel(), dtype=torch.uint8,
                                                                               pin_memory=True)
        dptr = self._snap_dev_ptr(host) if self.dev.type == "cuda" and _SNAP_KERNEL else 0
        if dptr:
            # the snapshot kernel stores into the mapped pinned buffer (no runtime device-to-host copy)
            nat.call("h2o_snap_copy", self.arena.data_ptr(), dptr, self.arena.numel(), nat.stream_ptr(self.dev))
        else:
            host.copy_(self.arena, non_blocking=True)
        ev = self._event_pool.pop() if self._event_pool else torch.cuda.Event()
        ev.record()
        self.history.append((host, ev))
        return len(self.history) - 1

    def _snap_dev_ptr(self, host: torch.Tensor) -> int:
        """Device address of a pinned snapshot buffer (0: not device-mapped -> runtime copy), cached per buffer."""
        cache = self.__dict__.setdefault("_dev_ptrs", {})
        hp = host.data_ptr()
        if hp not in cache:
            out = ctypes.c_ulonglong(0)
            rc = nat.hip().h2o_host_dev_ptr(ctypes.c_void_p(hp), ctypes.byref(out))
            cache[hp] = int(out.value) if rc == 0 and host.is_pinned() and out.value % 16 == 0 else 0
        return cache[hp]

    def leaf_values_view(self) -> torch.Tensor:
        """Device float32 leaf values of the last built tree (valid until the next build writes them)."""
        return self.av["leafval"].view(torch.float32)

    def pop_levels(self, ready_only: bool = False) -> list:
        """Decode built trees in build order: all of them, or (``ready_only``) the prefix whose snapshot
        copies have completed — never blocks in that mode."""
        out, self._decoded = self._decoded, []
        return out + self._pop(None, ready_only)

    def _pop(self, limit, ready_only: bool = False) -> list:
        out = []
        while self.history and (limit is None or len(out) < limit):
            host, ev = self.history[0]
            if ready_only and not ev.query():
                break
            ev.synchronize()
            self.history.pop(0)
            hn = host.numpy()
            o = self._off["rootw"][0]
            out.append(self._decode(hn, float(hn[o:o + 8].view(np.float64)[0])))
            self._pinned_pool.append(host)
            self._event_pool.append(ev)
        return out

    def _decode(self, host: np.ndarray, root_weight: float) -> TreeLevels:
        off = self._off

        def arr(name, dt):
            o, nb = off[name]
            return host[o:o + nb].view(dt)
        decs, cls, crs = [], [], []
        for d in range(self.D):
            n = int(arr(f"meta{d}", np.int32)[0])
            if d == 0:
                n = 1
            if n <= 0:
                break
            decs.append(arr(f"dec{d}", DEC_DT)[:n].copy())
            cls.append(arr(f"cl{d}", np.int32)[:n].astype(np.int64))
            crs.append(arr(f"cr{d}", np.int32)[:n].astype(np.int64))
        n_leaves = int(arr("counters", np.int32)[0])
        vals = arr("leafval", np.float32)[:n_leaves].copy()
        return TreeLevels(decs, cls, crs, n_leaves, vals, root_weight)


def _native_comm_cls():
    from ..parallel.rccl import NativeComm
    return NativeComm


# ================================================================================================
def make_builder(bins: torch.Tensor, F, nbins_f, iscat_f, mono_f, max_depth, params, node_cap=1 << 14):
    if bins.is_cuda:
        return GpuTreeBuilder(bins, F, nbins_f, iscat_f, mono_f, max_depth, params, node_cap=node_cap)
    return RefTreeBuilder(bins, F, nbins_f, iscat_f, mono_f, max_depth, params, node_cap=node_cap)


# ================================================================================================
# best-first ("lossguide") growth
def best_first_prune(tl: TreeLevels, max_leaves: int, by_depth: bool = False):
    """Cut a level-wise tree down to the one XGBoost's lossguide policy grows (reference:
    ``h2o-extensions/xgboost`` ``grow_policy=lossguide`` / ``max_leaves`` -> xgboost ``updater_hist``
    driven by a loss-change priority queue).

    Best-first growth expands, among the current leaves, the one whose split has the largest loss
    change, until ``max_leaves`` leaves exist or nothing can split. Every split it considers is the
    split the level-wise engine already found for that node (the node's rows do not depend on growth
    order), so the best-first tree is a top part of the level-wise tree of the same depth: expand by
    recorded gain from the root, stop at ``max_leaves``, and every node left unexpanded becomes a
    leaf holding the sums of the original leaves below it.

    ``by_depth`` is xgboost's depthwise policy under a leaf limit: nodes expand shallowest first, in
    creation order within a depth.

    Returns ``(pruned TreeLevels without leaf values, map old leaf id -> new leaf id)``.
    """
    import heapq
    decs, cl, cr = tl.decs, tl.child_l, tl.child_r
    can = lambda d, i: d < len(decs) and int(decs[d]["feat"][i]) >= 0
    expanded = set()
    key = (lambda d, i: float(d)) if by_depth else (lambda d, i: -float(decs[d]["gain"][i]))
    heap = [(key(0, 0), 0, 0, 0)] if decs and can(0, 0) else []
    leaves, seq = 1, 1
    while heap and (max_leaves <= 0 or leaves < max_leaves):
        _, _, d, i = heapq.heappop(heap)
        expanded.add((d, i))
        leaves += 1
        for c in (int(cl[d][i]), int(cr[d][i])):
            if c >= 0 and can(d + 1, c):
                heapq.heappush(heap, (key(d + 1, c), seq, d + 1, c))
                seq += 1
    leaf_map = np.zeros(max(int(tl.n_leaves), 1), dtype=np.int64)

    def sub_leaves(d, i):
        out, stack = [], [(d, i)]
        while stack:
            a, b = stack.pop()
            for c in {int(cl[a][b]), int(cr[a][b])}:
                if c < 0:
                    out.append(-1 - c)
                else:
                    stack.append((a + 1, c))
        return out

    ndecs, ncl, ncr = [], [], []
    n_new = 0
    level = [0] if decs else []
    d = 0
    while level:
        dd = decs[d][level].copy()
        lcl = np.zeros(len(level), dtype=np.int64)
        lcr = np.zeros(len(level), dtype=np.int64)
        nxt = []
        for j, i in enumerate(level):
            if (d, i) in expanded:
                for c, arr in ((int(cl[d][i]), lcl), (int(cr[d][i]), lcr)):
                    if c >= 0:
                        arr[j] = len(nxt)
                        nxt.append(c)
                    else:
                        leaf_map[-1 - c] = n_new
                        arr[j] = -1 - n_new
                        n_new += 1
            else:
                for lf in sub_leaves(d, i):
                    leaf_map[lf] = n_new
                dd["feat"][j] = -1
                dd["gain"][j] = 0.0
                lcl[j] = lcr[j] = -1 - n_new
                n_new += 1
        ndecs.append(dd)
        ncl.append(lcl)
        ncr.append(lcr)
        level = nxt
        d += 1
    return TreeLevels(ndecs, ncl, ncr, max(n_new, 1), None, tl.root_weight), leaf_map


class BestFirstBuilder:
    """Builder wrapper that grows each tree level-wise on the GPU, then prunes it best-first to
    ``max_leaves`` leaves (:func:`best_first_prune`) and remaps the rows' leaf ids and the leaf sums
    on the device. The wrapper waits for each tree's structure (one sync per tree)."""

    def __init__(self, inner, max_leaves: int, by_depth: bool = False):
        self.inner, self.max_leaves, self.by_depth = inner, int(max_leaves), bool(by_depth)
        self.done = []
        self.leaf_of_row = None
        self.leafsum = None

    def __getattr__(self, name):
        return getattr(self.inner, name)

    def build(self, aux_static, feat_ok=None, k_cols=0, seed=0, leaf_fn=None, **kw):
        kw.pop("leaf_native", None)
        self.inner.build(aux_static, feat_ok, k_cols, seed=seed, leaf_fn=None, **kw)
        tl = self.inner.pop_levels()[-1]
        pruned, lmap = best_first_prune(tl, self.max_leaves, self.by_depth)
        dev = self.inner.leaf_of_row.device
        m = torch.from_numpy(lmap).to(dev)
        self.leaf_of_row = m[self.inner.leaf_of_row.long()].to(torch.int32)
        ls = self.inner.leafsum[: tl.n_leaves].to(dev)
        self.leafsum = torch.zeros(pruned.n_leaves, ls.shape[1], dtype=ls.dtype, device=dev).index_add_(0, m[: ls.shape[0]], ls)
        if leaf_fn is not None:
            pruned.leaf_values = leaf_fn(self.leafsum).to(torch.float32).cpu().numpy()
        self.done.append(pruned)
        return len(self.done) - 1

    def pop_levels(self, ready_only: bool = False) -> list:
        out, self.done = self.done, []
        return out
