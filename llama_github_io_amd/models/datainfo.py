"""Design-matrix expansion for numeric learners (reference: ``hex/DataInfo.java``).

Tree learners consume the raw ``[F, N]`` float32 matrix (categoricals as codes). GLM, DeepLearning,
KMeans, PCA, GLRM, PSVM, ... need H2O's expanded layout: categoricals first as one-hot blocks
(``useAllFactorLevels`` keeps the first level, otherwise it is the reference level dropped), then
numerics optionally standardised; missing numerics are mean-imputed (``MeanImputation``) and a
missing categorical maps to the most frequent level (or an extra NA level when
``missing_bucket``). Coefficient names follow H2O: ``col.level`` for one-hot entries.

The expansion is a device gather: one-hot blocks are written with a single ``scatter_`` per
categorical column into a zeroed ``[N, P]`` tensor, numerics with one fused ``(x - mu) * inv_sd``.
"""
from __future__ import annotations

import numpy as np
import torch

from .base import DataInfo
from ..ops.segment import segment_sum


def _hip_ok(X) -> bool:
    """The HIP Expander kernels take a contiguous fp32 [F, N] device matrix."""
    if not (X.is_cuda and X.dtype == torch.float32 and X.is_contiguous()):
        return False
    from ..ops import _native as nat
    nat.register_hip_signatures({
        "h2o_num_stats": [nat.c_void_p, nat.c_ll, nat.c_void_p, nat.c_int, nat.c_void_p, nat.c_void_p, nat.c_void_p],
        "h2o_num_transform": [nat.c_void_p, nat.c_ll, nat.c_void_p, nat.c_int, nat.c_void_p, nat.c_void_p, nat.c_void_p,
                              nat.c_void_p, nat.c_int, nat.c_int, nat.c_int, nat.ctypes.c_float, nat.c_int,
                              nat.c_void_p],
    })
    return True


class Expander:
    def __init__(self, info: DataInfo, standardize=True, use_all_factor_levels=False, missing="MeanImputation",
                 missing_bucket=False, center_only=False, plug_values=None):
        self.info = info
        self.plug_values = plug_values   # missing_values_handling="PlugValues": {column: value or level}
        self.standardize = bool(standardize)
        self.center_only = bool(center_only)
        self.use_all = bool(use_all_factor_levels)
        self.missing = missing
        self.missing_bucket = bool(missing_bucket)
        iscat = np.asarray(info.iscat)
        self.cats = [j for j in range(info.F) if iscat[j]]
        self.nums = [j for j in range(info.F) if not iscat[j]]
        self.fitted = False

    # ---- fit statistics on the training matrix X [F, N]
    def fit(self, X: torch.Tensor, w: torch.Tensor | None = None, reduce=None):
        dev = X.device
        N = X.shape[1]
        w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
        self.cat_offsets, self.cat_sizes, self.cat_modes = [], [], []
        names = []
        off = 0
        for j in self.cats:
            dom = self.info.domains[j] or []
            L = len(dom)
            codes = X[j]
            ok = ~torch.isnan(codes)
            cnt = segment_sum(codes[ok].long().clamp(0, max(L - 1, 0)), w[ok], max(L, 1))
            if reduce is not None:
                cnt = reduce(cnt)
            self.cat_modes.append(int(torch.argmax(cnt)) if L else 0)
            start = 0 if self.use_all else 1
            size = L - start + (1 if self.missing_bucket else 0)
            self.cat_offsets.append(off)
            self.cat_sizes.append(size)
            nm = self.info.x[j]
            names += [f"{nm}.{dom[k]}" for k in range(start, L)]
            if self.missing_bucket:
                names.append(f"{nm}.missing(NA)")
            off += size
        self.num_off = off
        k = len(self.nums)
        sw = torch.zeros(k, dtype=torch.float64, device=dev)
        s1 = torch.zeros(k, dtype=torch.float64, device=dev)
        s2 = torch.zeros(k, dtype=torch.float64, device=dev)
        CH = 32   # feature chunks keep the fp64 temporaries small on wide frames (e.g. 784 x 10M)
        if k and _hip_ok(X):
            # one HIP pass over the numeric rows: fp64 Σw, Σwx, Σwx² per feature (k_num_stats)
            from ..ops import _native as nat
            rows = torch.as_tensor(self.nums, dtype=torch.int32, device=dev)
            st = torch.zeros(k, 3, dtype=torch.float64, device=dev)
            wf = w.float().contiguous()
            # unit row weights are not re-read once per feature (784 x the weight column on a 784-wide frame)
            unit = N > 0 and bool((wf == 1).all())
            nat.call("h2o_num_stats", X.data_ptr(), N, rows.data_ptr(), k, 0 if unit else wf.data_ptr(), st.data_ptr(),
                     nat.stream_ptr(dev))
            sw, s1, s2 = st[:, 0].clone(), st[:, 1].clone(), st[:, 2].clone()
            CH = 0
        for a in range(0, k if CH else 0, CH or 1):
            Xn = X[self.nums[a:a + CH]].double()
            ok = ~torch.isnan(Xn)
            Xz = torch.where(ok, Xn, torch.zeros_like(Xn))
            sw[a:a + CH] = (ok.double() * w).sum(1)
            s1[a:a + CH] = (Xz * w).sum(1)
            s2[a:a + CH] = (Xz * Xz * w).sum(1)
            del Xn, ok, Xz
        if reduce is not None:
            packed = reduce(torch.cat([sw, s1, s2]))
            sw, s1, s2 = packed[:k], packed[k:2 * k], packed[2 * k:]
        mu = s1 / sw.clamp(min=1e-300)
        var = (s2 - sw * mu * mu) / (sw - 1).clamp(min=1e-300)
        sd = var.clamp(min=0).sqrt()
        self.num_mean = mu
        self.num_fill = None
        if str(self.missing).lower().replace("_", "") == "plugvalues":
            pv = self._plug_dict()
            fill = mu.clone()
            for i, j in enumerate(self.nums):
                nm = self.info.x[j]
                if nm in pv:
                    fill[i] = float(pv[nm])
            self.num_fill = fill
            for i, j in enumerate(self.cats):
                nm = self.info.x[j]
                if nm in pv:
                    dom = list(self.info.domains[j] or [])
                    v = str(pv[nm])
                    if v not in dom:
                        raise ValueError(f"plug_values: level {v!r} is not in the domain of {nm}")
                    self.cat_modes[i] = dom.index(v)
        self.num_sd = torch.where(sd > 0, sd, torch.ones_like(sd))
        self.num_sd_raw = sd
        names += [self.info.x[j] for j in self.nums]
        self.names = names
        self.P = off + len(self.nums)
        self.fitted = True
        return self

    @property
    def ncats_expanded(self):
        return self.num_off

    def set_cat_hash(self, n_slots: int, seed: int):
        """Hash the one-hot categorical columns into ``n_slots`` count columns (DeepLearning
        ``max_categorical_features``, Neurons.Input.setInput hash trick): one-hot column ``c`` adds 1 to
        slot ``|murmur2(big-endian int c, seed) % n_slots|``; numeric columns follow the slots."""
        nc = self.num_off
        if n_slots >= nc:
            return self
        self.cat_hash = dict(n=int(n_slots), seed=int(seed), idx=[abs(_jmod(_murmur2_int(c, seed), n_slots))
                                                                  for c in range(nc)])
        self.names = [f"hashed_cat_{i}" for i in range(n_slots)] + self.names[nc:]
        return self

    def transform(self, X: torch.Tensor, dtype=torch.float32, extra=None) -> torch.Tensor:
        """[F, N] raw -> [N, P] design matrix; ``extra`` (a constant, e.g. GLM's intercept column 1 / 0) appends
        column P = extra, written in place ([N, P + 1], no concatenation copy of the design)."""
        h = getattr(self, "cat_hash", None)
        if extra is not None and not h:
            return self._transform(X, dtype, extra)
        Z = self._transform(X, dtype)
        if extra is not None:
            Z = self._hash_cats(Z, h)
            return torch.cat([Z, torch.full((Z.shape[0], 1), float(extra), dtype=Z.dtype, device=Z.device)], 1)
        return self._hash_cats(Z, h)

    def _hash_cats(self, Z, h):
        if h:
            nc = self.num_off
            idx = torch.as_tensor(h["idx"], dtype=torch.long, device=Z.device)
            Zc = torch.zeros(Z.shape[0], h["n"], dtype=Z.dtype, device=Z.device).index_add_(1, idx, Z[:, :nc])
            Z = torch.cat([Zc, Z[:, nc:]], 1)
        return Z

    def _transform(self, X: torch.Tensor, dtype=torch.float32, extra=None) -> torch.Tensor:
        N = X.shape[1]
        dev = X.device
        ncol = self.P + (0 if extra is None else 1)
        dense = (not self.cats and self.nums and self.num_off == 0 and len(self.nums) == self.P and _hip_ok(X)
                 and dtype in (torch.float32, torch.bfloat16))
        # every column written below (all-numeric HIP transform): no zero fill of the [N, P] design
        Z = (torch.empty if dense else torch.zeros)(N, ncol, dtype=dtype, device=dev)
        # whole rows of <= 64 numeric columns: k_num_transform writes the constant extra column too (one contiguous
        # store span per block instead of a strided fill)
        kx = dense and extra is not None and self.P <= 64
        if extra is not None and not kx:
            Z[:, self.P] = float(extra)
        start = 0 if self.use_all else 1
        for i, j in enumerate(self.cats):
            codes = X[j]
            L = self.cat_sizes[i] + start - (1 if self.missing_bucket else 0)
            na = torch.isnan(codes)
            c = torch.where(na, torch.full_like(codes, -2.0), codes).long()
            if self.missing_bucket:
                c = torch.where(na, torch.full_like(c, L), c)
            else:
                c = torch.where(na, torch.full_like(c, self.cat_modes[i]), c)
            c = torch.where((c >= L + (1 if self.missing_bucket else 0)) | (c < 0), torch.full_like(c, -1), c)  # unseen
            col = c - start
            valid = col >= 0
            idx = (self.cat_offsets[i] + col.clamp(min=0))
            rows = torch.nonzero(valid, as_tuple=True)[0]
            Z[rows, idx[rows]] = 1
        CH = 32
        fill_all = getattr(self, "num_fill", None)
        if self.nums and _hip_ok(X) and dtype in (torch.float32, torch.bfloat16):
            # one tiled HIP pass (k_num_transform): NaN fill, centring / scaling, transpose into Z
            from ..ops import _native as nat
            k = len(self.nums)
            rows = torch.as_tensor(self.nums, dtype=torch.int32, device=dev)
            mu = self.num_mean.to(dev).float()
            fill = (mu if fill_all is None else fill_all.to(dev).float()).contiguous()
            sub = mu if (self.standardize or self.center_only) else torch.zeros_like(mu)
            mul = (1.0 / self.num_sd.to(dev).float()) if self.standardize else torch.ones_like(mu)
            nat.call("h2o_num_transform", X.data_ptr(), N, rows.data_ptr(), k, fill.data_ptr(), sub.contiguous().data_ptr(),
                     mul.contiguous().data_ptr(), Z.data_ptr(), ncol, self.num_off, int(dtype == torch.bfloat16),
                     float(extra) if kx else 0.0, int(kx), nat.stream_ptr(dev))
            return Z
        for a in range(0, len(self.nums), CH):
            Xn = X[self.nums[a:a + CH]].to(dtype=torch.float64)
            mu = self.num_mean[a:a + CH, None]
            fill = mu if fill_all is None else fill_all[a:a + CH, None].to(mu.device)
            Xn = torch.where(torch.isnan(Xn), fill.expand_as(Xn), Xn)
            if self.standardize:
                Xn = (Xn - mu) / self.num_sd[a:a + CH, None]
            elif self.center_only:
                Xn = Xn - mu
            Z[:, self.num_off + a:self.num_off + a + Xn.shape[0]] = Xn.T.to(dtype)
            del Xn
        return Z

    def _plug_dict(self):
        pv = self.plug_values
        if pv is None:
            raise ValueError("missing_values_handling='PlugValues' needs plug_values")
        if hasattr(pv, "as_data_frame"):
            pv = pv.as_data_frame()
        if hasattr(pv, "iloc"):
            return {str(c): pv[c].iloc[0] for c in pv.columns}
        return dict(pv)

    def row_mask_complete(self, X: torch.Tensor) -> torch.Tensor:
        """Rows with no NA (for ``missing_values_handling='Skip'``)."""
        return ~torch.isnan(X).any(0)

    # ---- coefficient (de)standardisation helpers for linear models
    def destandardize(self, beta: torch.Tensor, intercept: float):
        """beta on standardized numerics -> beta on raw scale (+ intercept shift)."""
        b = beta.clone().double()
        ic = float(intercept)
        if self.nums and self.standardize:
            k = self.num_off
            b[k:] = beta[k:].double() / self.num_sd
            ic = ic - float((b[k:] * self.num_mean).sum())
        return b, ic

    def to_state(self):
        nf = getattr(self, "num_fill", None)
        return dict(standardize=self.standardize, use_all=self.use_all, missing=self.missing,
                    missing_bucket=self.missing_bucket, center_only=self.center_only,
                    num_fill=None if nf is None else nf.cpu().tolist(),
                    cat_offsets=self.cat_offsets, cat_sizes=self.cat_sizes, cat_modes=self.cat_modes,
                    num_off=self.num_off, num_mean=self.num_mean.cpu().tolist(), num_sd=self.num_sd.cpu().tolist(),
                    num_sd_raw=self.num_sd_raw.cpu().tolist(), names=self.names, P=self.P,
                    cat_hash=getattr(self, "cat_hash", None))

    @staticmethod
    def from_state(info, s, device=None):
        e = Expander(info, s["standardize"], s["use_all"], s["missing"], s["missing_bucket"], s.get("center_only", False))
        for k in ("cat_offsets", "cat_sizes", "cat_modes", "num_off", "names", "P"):
            setattr(e, k, s[k])
        dev = device or torch.device("cpu")
        e.num_mean = torch.tensor(s["num_mean"], dtype=torch.float64, device=dev)
        e.num_sd = torch.tensor(s["num_sd"], dtype=torch.float64, device=dev)
        e.num_sd_raw = torch.tensor(s["num_sd_raw"], dtype=torch.float64, device=dev)
        e.num_fill = None if s.get("num_fill") is None else torch.tensor(s["num_fill"], dtype=torch.float64, device=dev)
        e.cat_hash = s.get("cat_hash")
        e.fitted = True
        return e

    def to(self, device):
        self.num_mean = self.num_mean.to(device)
        self.num_sd = self.num_sd.to(device)
        self.num_sd_raw = self.num_sd_raw.to(device)
        if getattr(self, "num_fill", None) is not None:
            self.num_fill = self.num_fill.to(device)
        return self


def _i32(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v >= 1 << 31 else v


def _jmod(a: int, b: int) -> int:
    """Java int remainder (sign of the dividend)."""
    r = abs(a) % b
    return -r if a < 0 else r


def _murmur2_int(c: int, seed: int) -> int:
    """MurmurHash2 (32 bit) of the 4 big-endian bytes of ``c`` with a 32-bit ``seed``, as a signed Java int."""
    m = 0x5BD1E995
    k = int.from_bytes(int(c & 0xFFFFFFFF).to_bytes(4, "big"), "little")
    h = (_i32(seed) ^ 4) & 0xFFFFFFFF
    k = (k * m) & 0xFFFFFFFF
    k ^= k >> 24
    k = (k * m) & 0xFFFFFFFF
    h = (h * m) & 0xFFFFFFFF
    h ^= k
    h ^= h >> 13
    h = (h * m) & 0xFFFFFFFF
    h ^= h >> 15
    return _i32(h)
