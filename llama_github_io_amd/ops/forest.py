"""Compressed trees and forest scoring (reference: ``hex/tree/CompressedTree.java``,
``hex/genmodel/algos/tree/SharedTreeMojoModel.java`` scoreTree).

A :class:`Tree` is a flat node table (root = 0): ``feat`` (-1 = leaf), raw-value threshold ``thr``
(numeric: ``x < thr`` goes left), ``na_left``, categorical level bitsets, children, leaf ``value``,
``cover`` (weighted rows, used by TreeSHAP) and split ``gain`` (variable importance).
:class:`Forest` concatenates trees (with their class index) and scores raw features either with the
HIP kernel ``k_predict`` (CUDA tensors) or a vectorised PyTorch traversal (CPU).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

from . import _native as nat
from .tree import NA_BIN, TreeLevels


@dataclass
class Tree:
    feat: np.ndarray
    thr: np.ndarray
    bin: np.ndarray
    na_left: np.ndarray
    is_cat: np.ndarray
    cat_bits: list          # per node: None or np.uint32 array over LEVELS
    cat_nbits: np.ndarray
    left: np.ndarray
    right: np.ndarray
    value: np.ndarray
    cover: np.ndarray
    gain: np.ndarray

    @property
    def n_nodes(self):
        return len(self.feat)

    def depth(self) -> int:
        d = np.zeros(self.n_nodes, dtype=np.int64)
        for i in range(self.n_nodes):
            if self.feat[i] >= 0:
                d[self.left[i]] = d[i] + 1
                d[self.right[i]] = d[i] + 1
        return int(d.max()) if self.n_nodes else 0

    def n_leaves(self) -> int:
        return int((self.feat < 0).sum())

    def to_state(self):
        return {k: (v.tolist() if isinstance(v, np.ndarray) else [None if b is None else b.tolist() for b in v])
                for k, v in self.__dict__.items()}

    @staticmethod
    def from_state(s):
        kw = {}
        for k, v in s.items():
            if k == "cat_bits":
                kw[k] = [None if b is None else np.asarray(b, dtype=np.uint32) for b in v]
            else:
                kw[k] = np.asarray(v)
        kw["thr"] = kw["thr"].astype(np.float32)
        kw["value"] = kw["value"].astype(np.float32)
        return Tree(**kw)


def levels_to_tree(tl: TreeLevels, binning, leaf_values=None) -> Tree:
    """Flatten level-wise decisions into a node array (root 0, children appended in visit order).
    Hot on the host during training (one call per tree, overlapped with GPU work): per-level columns
    are pulled out of the structured records once, the node loop touches only Python scalars."""
    vals = (tl.leaf_values if leaf_values is None else leaf_values)
    vals = [] if vals is None else np.asarray(vals, dtype=np.float64).tolist()
    nv = len(vals)
    feat, thr, bins, nal, iscat, bits, nbits, left, right, value, cover, gain = ([] for _ in range(12))

    def new(c):
        feat.append(-1); thr.append(0.0); bins.append(0); nal.append(0); iscat.append(0); bits.append(None)
        nbits.append(0); left.append(-1); right.append(-1); value.append(0.0); cover.append(c); gain.append(0.0)
        return len(feat) - 1

    ids = [new(tl.root_weight)]
    for d, decs in enumerate(tl.decs):
        fz, bz, nz, cz = decs["feat"].tolist(), decs["bin"].tolist(), decs["na_left"].tolist(), decs["is_cat"].tolist()
        gz, wlz, wrz = decs["gain"].tolist(), decs["wl"].tolist(), decs["wr"].tolist()
        clz, crz = np.asarray(tl.child_l[d]).tolist(), np.asarray(tl.child_r[d]).tolist()
        nxt = {}
        for i in range(len(fz)):
            g = ids[i]
            f, cl, cr = fz[i], clz[i], crz[i]
            if f < 0:
                value[g] = vals[-1 - cl] if cl < 0 and -1 - cl < nv else 0.0
                continue
            # engine column -> original feature (wide numeric features span several engine columns)
            feat[g], bins[g], nal[g], iscat[g], gain[g] = binning.orig(f), bz[i], nz[i], cz[i], gz[i]
            if cz[i]:
                nl = int(binning.nlevels[f])
                bits_b = decs["bits"][i]
                lv = np.arange(nl)
                if cz[i] == 2:
                    # wide-categorical group split: the bitset is over the group's global bins 254k + b (level_to_bin
                    # of real column k names the levels it holds; the others' bytes say 'elsewhere' = nbins - 1)
                    bl = np.full(nl, -1, dtype=np.int64)
                    for k in range(4):
                        if f + k >= binning.F or binning.orig(f + k) != binning.orig(f) or \
                                (binning.pad is not None and binning.pad[f + k]):
                            break
                        mk = np.asarray(binning.level_to_bin[f + k], dtype=np.int64)
                        hold = mk[lv] < int(binning.nbins[f + k]) - 1
                        bl[hold] = 254 * k + mk[lv][hold]
                    inleft = np.zeros(nl, dtype=bool)
                    ok = bl >= 0
                    inleft[ok] = ((bits_b[bl[ok] >> 5] >> (bl[ok] & 31).astype(np.uint32)) & 1).astype(bool)
                    iscat[g] = 1
                else:
                    m = binning.level_to_bin[f] if binning.level_to_bin else None
                    bl = lv if m is None else m[lv]
                    inleft = ((bits_b[bl >> 5] >> (bl & 31).astype(np.uint32)) & 1).astype(bool)
                words = np.zeros((nl + 31) // 32, dtype=np.uint32)
                lvl = np.nonzero(inleft)[0]
                np.bitwise_or.at(words, lvl >> 5, (np.uint32(1) << (lvl & 31).astype(np.uint32)))
                bits[g], nbits[g], thr[g] = words, nl, 0.0
            else:
                b = bz[i]
                e = binning.edges[f]
                thr[g] = float("inf") if b >= NA_BIN or b - 1 >= len(e) else float(e[b - 1])
            for c, w, arr in ((cl, wlz[i], left), (cr, wrz[i], right)):
                k = new(w)
                arr[g] = k
                if c >= 0:
                    nxt[c] = k
                else:
                    value[k] = vals[-1 - c] if -1 - c < nv else 0.0
        ids = [nxt[c] for c in sorted(nxt)]
    return Tree(feat=np.asarray(feat, dtype=np.int32), thr=np.asarray(thr, dtype=np.float32),
                bin=np.asarray(bins, dtype=np.int32), na_left=np.asarray(nal, dtype=np.int8),
                is_cat=np.asarray(iscat, dtype=np.int8), cat_bits=bits,
                cat_nbits=np.asarray(nbits, dtype=np.int32), left=np.asarray(left, dtype=np.int32),
                right=np.asarray(right, dtype=np.int32), value=np.asarray(value, dtype=np.float32),
                cover=np.asarray(cover, dtype=np.float64), gain=np.asarray(gain, dtype=np.float64))


class Forest:
    """Trees + class assignment, with cached flat device arrays for scoring."""

    def __init__(self, trees=None, tree_class=None, n_classes_out: int = 1):
        self._trees = list(trees or [])
        self._pending = []          # (TreeLevels, binning) decoded on first access of ``trees``
        self.tree_class = list(tree_class or [0] * len(self._trees))
        self.K = n_classes_out
        self._flat = {}

    @property
    def trees(self):
        """Node tables of every tree. Trees added with :meth:`add_levels` are decoded from their level
        records here, on first use (scoring, MOJO, summaries), so the training loop never waits on the
        host-side flattening of the last trees it built."""
        if self._pending:
            pend, self._pending = self._pending, []
            self._trees.extend(levels_to_tree(tl, b) for tl, b in pend)
        return self._trees

    @trees.setter
    def trees(self, v):
        self._trees = list(v)
        self._pending = []

    def add(self, tree: Tree, cls: int = 0):
        if self._pending:
            self.trees    # keep insertion order
        self._trees.append(tree)
        self.tree_class.append(cls)
        self._flat.clear()

    def add_levels(self, tl, binning, cls: int = 0):
        self._pending.append((tl, binning))
        self.tree_class.append(cls)
        self._flat.clear()

    def depth_leaves(self) -> list:
        """(depth, leaf count) of every tree; trees still pending as level records are read from those records
        (no host-side flattening: the model summary of a 100-tree GBM spent ~21 ms decoding every tree)."""
        out = [(t.depth(), t.n_leaves()) for t in self._trees]
        for tl, _ in self._pending:
            d = 0
            for i, dec in enumerate(tl.decs):
                if len(dec) and bool((np.asarray(dec["feat"]) >= 0).any()):
                    d = i + 1
            out.append((d, int(tl.n_leaves)))
        return out

    def __len__(self):
        return len(self._trees) + len(self._pending)

    def flatten(self, t0=0, t1=None):
        t1 = len(self.trees) if t1 is None else t1
        feat, thr, left, right, nal, coff, cnb, val, roots, cls = [], [], [], [], [], [], [], [], [], []
        bits = []
        base = 0
        for ti in range(t0, t1):
            t = self.trees[ti]
            n = t.n_nodes
            feat.append(t.feat); thr.append(t.thr)
            left.append(np.where(t.left >= 0, t.left + base, -1)); right.append(np.where(t.right >= 0, t.right + base, -1))
            nal.append(t.na_left.astype(np.int32)); val.append(t.value)
            co = np.full(n, -1, dtype=np.int32)
            for i in range(n):
                if t.feat[i] >= 0 and t.is_cat[i]:
                    co[i] = sum(len(b) for b in bits)
                    bits.append(t.cat_bits[i])
            coff.append(co); cnb.append(t.cat_nbits)
            roots.append(base); cls.append(self.tree_class[ti])
            base += n
        cat = lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt)
        return dict(feat=cat(feat, np.int32), thr=cat(thr, np.float32), left=cat(left, np.int32),
                    right=cat(right, np.int32), na_left=cat(nal, np.int32), cat_off=cat(coff, np.int32),
                    cat_bits=(np.concatenate(bits).astype(np.uint32) if bits else np.zeros(1, np.uint32)),
                    cat_nbits=cat(cnb, np.int32), value=cat(val, np.float32),
                    roots=np.asarray(roots, dtype=np.int32), cls=np.asarray(cls, dtype=np.int32))

    def _device_flat(self, device, t0, t1):
        key = (str(device), t0, t1)
        if key not in self._flat:
            fl = self.flatten(t0, t1)
            self._flat[key] = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in fl.items()}
        return self._flat[key]

    def predict_raw(self, X: torch.Tensor, t0: int = 0, t1: int | None = None, out: torch.Tensor | None = None,
                    return_leaves: bool = False):
        """X: float32 [F, N] column-major. Returns [N, K] sums of leaf values (no link, no init_f)."""
        t1 = len(self.trees) if t1 is None else t1
        F, N = X.shape
        if out is None:
            out = torch.zeros(N, self.K, dtype=torch.float32, device=X.device)
        nt = t1 - t0
        leaves = torch.empty(N, max(nt, 1), dtype=torch.int32, device=X.device) if return_leaves else None
        if nt <= 0 or N == 0:
            return (out, leaves) if return_leaves else out
        fl = self._device_flat(X.device, t0, t1)
        Xc = X.contiguous().float()
        if X.is_cuda:
            nat.call("h2o_predict", Xc.data_ptr(), N, self.K, fl["feat"].data_ptr(), fl["thr"].data_ptr(),
                     fl["left"].data_ptr(), fl["right"].data_ptr(), fl["na_left"].data_ptr(), fl["cat_off"].data_ptr(),
                     fl["cat_bits"].data_ptr(), fl["cat_nbits"].data_ptr(), fl["value"].data_ptr(),
                     fl["roots"].data_ptr(), fl["cls"].data_ptr(), nt, out.data_ptr(),
                     0 if leaves is None else leaves.data_ptr(), nat.stream_ptr(X.device))
        else:
            self._predict_torch(Xc, fl, nt, out, leaves)
        return (out, leaves) if return_leaves else out

    @staticmethod
    def _predict_torch(X, fl, nt, out, leaves):
        N = X.shape[1]
        ar = torch.arange(N)
        feat, thr, left, right = fl["feat"].long(), fl["thr"], fl["left"].long(), fl["right"].long()
        nal, coff, cnb, bits, val = fl["na_left"].bool(), fl["cat_off"].long(), fl["cat_nbits"].long(), fl["cat_bits"].long(), fl["value"]
        for t in range(nt):
            node = torch.full((N,), int(fl["roots"][t]), dtype=torch.long)
            for _ in range(10_000):
                f = feat[node]
                act = f >= 0
                if not bool(act.any()):
                    break
                fi = f.clamp(min=0)
                x = X[fi, ar]
                isnan = torch.isnan(x)
                co = coff[node]
                iscat = co >= 0
                code = torch.nan_to_num(x, nan=-1).long()
                inrange = (code >= 0) & (code < cnb[node])
                word = bits[(co.clamp(min=0) + (code.clamp(min=0) >> 5)).clamp(max=bits.numel() - 1)]
                catleft = ((word >> (code.clamp(min=0) & 31)) & 1).bool()
                catgo = torch.where(inrange, catleft, nal[node])
                numgo = x < thr[node]
                go = torch.where(isnan, nal[node], torch.where(iscat, catgo, numgo))
                nxt = torch.where(go, left[node], right[node])
                node = torch.where(act, nxt, node)
            out[:, int(fl["cls"][t])] += val[node]
            if leaves is not None:
                leaves[:, t] = node.int()
