"""Exact order statistics of a row-sharded column without gathering rows.

Reference: ``hex/quantile/Quantile.java`` — H2O finds exact quantiles of a distributed column by
iterative histogram refinement (each pass histograms the rows inside the current candidate range,
reduces the histogram over the cluster and narrows the range to the bin holding the target rank).

Here the refinement runs on an order-preserving int64 image of the float64 values: every pass splits
each candidate key range into at most 2^11 + 1 buckets by an arithmetic shift, so no pass can overflow
and the 64 key bits are exhausted after <= 6 passes, when the range is one key = one exact value. A
pass is one read of the local shard plus ONE all-reduce of the bucket weights, whatever the number of
rows. Rows may be split into groups (e.g. tree leaves), each with its own target: all groups refine in
the same passes (one bincount over group-offset buckets).

Weighted ranks follow ``weighted_quantiles``: the answer for target T is the smallest value whose
cumulative weight reaches T (rows of weight w count w times); rows of weight <= 0 are ignored.
"""
from __future__ import annotations

import math

import torch

from . import collectives as coll

_SHIFT_BITS = 11
_FLIP = 0x7FFFFFFFFFFFFFFF
_BIG = (1 << 63) - 1


def order_keys(v: torch.Tensor) -> torch.Tensor:
    """Order-preserving int64 keys of float64 values (NaN-free input; -0.0 is folded onto +0.0)."""
    bits = (v.double() + 0.0).contiguous().view(torch.int64)
    return torch.where(bits >= 0, bits, bits ^ _FLIP)


def key_value(k: int) -> float:
    """Inverse of :func:`order_keys` for one key."""
    b = k if k >= 0 else k ^ _FLIP
    return float(torch.tensor([b], dtype=torch.int64).view(torch.float64)[0])


def _reduce(t: torch.Tensor, op=None) -> torch.Tensor:
    if not coll.is_dist():
        return t
    dev = coll.comm_device()
    h = t.to(dev)
    coll.all_reduce_(h, op)
    return h.to(t.device)


def group_order_statistics(v: torch.Tensor, group: torch.Tensor | None, G: int, targets, w=None) -> list:
    """``targets[g]`` (cumulative weight, or None) of group g -> the value at that target among the rows
    of group g over ALL ranks (every rank passes its shard; works in one process too). NaN for groups
    with no row (or a None target). Returns python floats, identical on every rank."""
    import torch.distributed as dist
    dev = v.device
    keys = order_keys(v)
    ww = torch.ones(keys.numel(), dtype=torch.float64, device=dev) if w is None else w.double()
    grp = torch.zeros(keys.numel(), dtype=torch.long, device=dev) if group is None else group.long()
    pos = ww > 0
    keys, ww, grp = keys[pos], ww[pos], grp[pos]
    kmin = torch.full((G,), _BIG, dtype=torch.int64, device=dev).scatter_reduce(0, grp, keys, "amin")
    kmax = torch.full((G,), -_BIG, dtype=torch.int64, device=dev).scatter_reduce(0, grp, keys, "amax")
    mm = _reduce(torch.cat([kmin, -kmax]), dist.ReduceOp.MIN).cpu().tolist()
    lo, hi = mm[:G], [-x for x in mm[G:]]
    T = [None if t is None else float(t) for t in targets]
    done = [T[g] is None or lo[g] > hi[g] for g in range(G)]
    below = [0.0] * G
    while not all(done):
        s_l, off_l, nb_l, base_l = [0] * G, [0] * G, [0] * G, [0] * G
        total = 0
        for g in range(G):
            if done[g]:
                continue
            s = max(0, (hi[g] - lo[g]).bit_length() - _SHIFT_BITS)
            s_l[g], off_l[g] = s, lo[g] >> s
            nb_l[g] = (hi[g] >> s) - off_l[g] + 1
            base_l[g] = total
            total += nb_l[g]
        act = torch.tensor([not d for d in done], device=dev)
        lo_t = torch.tensor([min(x, _BIG) for x in lo], dtype=torch.int64, device=dev)
        hi_t = torch.tensor([max(x, -_BIG) for x in hi], dtype=torch.int64, device=dev)
        s_t = torch.tensor(s_l, dtype=torch.int64, device=dev)
        o_t = torch.tensor(off_l, dtype=torch.int64, device=dev)
        b_t = torch.tensor(base_l, dtype=torch.int64, device=dev)
        m = act[grp] & (keys >= lo_t[grp]) & (keys <= hi_t[grp])
        gm = grp[m]
        b = b_t[gm] + torch.bitwise_right_shift(keys[m], s_t[gm]) - o_t[gm]
        h = torch.bincount(b, weights=ww[m], minlength=total)[:total].to(torch.float64)
        hc = _reduce(h).cpu()
        for g in range(G):
            if done[g]:
                continue
            c = torch.cumsum(hc[base_l[g]:base_l[g] + nb_l[g]], 0) + below[g]
            j = int(torch.searchsorted(c, torch.tensor([T[g]], dtype=torch.float64)).clamp(max=nb_l[g] - 1))
            if j > 0:
                below[g] = float(c[j - 1])
            s = s_l[g]
            blo, bhi = (off_l[g] + j) << s, ((off_l[g] + j + 1) << s) - 1
            lo[g], hi[g] = max(lo[g], blo), min(hi[g], bhi)
            if s == 0 or lo[g] == hi[g]:
                hi[g] = lo[g]
                done[g] = True
    return [math.nan if (T[g] is None or lo[g] > hi[g]) else key_value(lo[g]) for g in range(G)]


def order_statistics(v: torch.Tensor, targets, w: torch.Tensor | None = None) -> list:
    """Values at cumulative-weight targets (1-based: target T = the first value whose cumulative weight
    reaches T; unweighted rank r is target r + 1) of the column ``v`` (NaN-free) split over the ranks.

    Any number of targets share the passes: targets that fall into the same bucket share its refined
    range, distinct ranges are disjoint, so every row lands in at most one active range (a searchsorted
    over the sorted range starts) and a pass is still one bincount + one all-reduce."""
    import torch.distributed as dist
    dev = v.device
    keys = order_keys(v)
    ww = torch.ones(keys.numel(), dtype=torch.float64, device=dev) if w is None else w.double()
    pos = ww > 0
    keys, ww = keys[pos], ww[pos]
    mm = torch.tensor([keys.min().item() if keys.numel() else _BIG, -(keys.max().item() if keys.numel() else -_BIG)],
                      dtype=torch.int64, device=dev)
    kmin, kmax = (int(x) for x in _reduce(mm, dist.ReduceOp.MIN).cpu().tolist())
    kmax = -kmax
    T = [float(t) for t in targets]
    out = [math.nan] * len(T)
    if kmin > kmax or not T:
        return out
    ranges = [dict(lo=kmin, hi=kmax, below=0.0, tg=list(range(len(T))))]
    while ranges:
        ranges.sort(key=lambda r: r["lo"])
        total = 0
        for r in ranges:
            r["s"] = max(0, (r["hi"] - r["lo"]).bit_length() - _SHIFT_BITS)
            r["off"] = r["lo"] >> r["s"]
            r["nb"] = (r["hi"] >> r["s"]) - r["off"] + 1
            r["base"] = total
            total += r["nb"]
        st = torch.tensor([r["lo"] for r in ranges], dtype=torch.int64, device=dev)
        en = torch.tensor([r["hi"] for r in ranges], dtype=torch.int64, device=dev)
        sh = torch.tensor([r["s"] for r in ranges], dtype=torch.int64, device=dev)
        of = torch.tensor([r["off"] for r in ranges], dtype=torch.int64, device=dev)
        ba = torch.tensor([r["base"] for r in ranges], dtype=torch.int64, device=dev)
        ri = torch.searchsorted(st, keys, right=True) - 1
        rc = ri.clamp(min=0)
        m = (ri >= 0) & (keys <= en[rc])
        rm = rc[m]
        b = ba[rm] + torch.bitwise_right_shift(keys[m], sh[rm]) - of[rm]
        h = torch.bincount(b, weights=ww[m], minlength=total)[:total].to(torch.float64)
        hc = _reduce(h).cpu()
        nxt = {}
        for r in ranges:
            c = torch.cumsum(hc[r["base"]:r["base"] + r["nb"]], 0) + r["below"]
            js = torch.searchsorted(c, torch.tensor([T[i] for i in r["tg"]], dtype=torch.float64)).clamp(max=r["nb"] - 1)
            for i, j in zip(r["tg"], js.tolist()):
                s_ = r["s"]
                blo, bhi = (r["off"] + j) << s_, ((r["off"] + j + 1) << s_) - 1
                lo, hi = max(r["lo"], blo), min(r["hi"], bhi)
                if s_ == 0 or lo == hi:
                    out[i] = key_value(lo)
                    continue
                key = (lo, hi)
                if key not in nxt:
                    nxt[key] = dict(lo=lo, hi=hi, below=float(c[j - 1]) if j > 0 else r["below"], tg=[])
                nxt[key]["tg"].append(i)
        ranges = list(nxt.values())
    return out


def global_quantile(v: torch.Tensor, alpha) -> float:
    """Quantile (linear interpolation at alpha * (n - 1), as torch.quantile) or, with alpha None, the lower
    median (as torch.median) of a row-sharded column; NaN if any value is NaN. Exact, no row gather."""
    v = v.double()
    st = torch.tensor([float(v.numel()), float(torch.isnan(v).sum())], dtype=torch.float64)
    if coll.is_dist():
        st = coll.all_reduce_(st.to(coll.comm_device())).cpu()
    n, nnan = int(st[0]), int(st[1])
    if n == 0 or nnan:
        return float("nan")
    if alpha is None:
        return order_statistics(v, [(n - 1) // 2 + 1])[0]
    pos = alpha * (n - 1)
    lo, hi = math.floor(pos), math.ceil(pos)
    a, b = order_statistics(v, [lo + 1, hi + 1])
    return a + (pos - lo) * (b - a)
