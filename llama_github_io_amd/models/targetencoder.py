"""Target Encoder (reference: ``h2o-extensions/target-encoder/src/main/java/ai/h2o/targetencoding/
TargetEncoder.java``, ``TargetEncoderModel.java``, ``TargetEncoderHelper.java``).

Per categorical column (and optional column groups via ``columns_to_encode``) the level statistics
(numerator = Σy, denominator = count; one numerator per class for multinomial) are device
``index_add_`` reductions. Encoded value = blended posterior
λ·num/den + (1-λ)·prior with λ = 1/(1+exp((k-n)/f)) when ``blending`` (k = inflection_point,
f = smoothing), plain posterior otherwise; unseen/NA levels get the prior. Leakage handling for
training data: ``none``, ``leave_one_out`` (subtract the row's own target) and ``k_fold`` (out-of-
fold statistics via ``fold_column``); optional uniform ``noise``. Output columns ``<col>_te``.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .base import DataInfo, Model, make_key
from ..ops.segment import segment_sum
from ..parallel import collectives as coll


def _merge(t: torch.Tensor) -> torch.Tensor:
    """Level statistics of a row-sharded frame: the sum over every rank's rows (MRTask reduce)."""
    if not coll.is_dist():
        return t
    return coll.all_reduce_(t.contiguous().to(coll.comm_device())).to(t.device)

TE_DEFAULTS = dict(blending=False, inflection_point=10.0, smoothing=20.0, data_leakage_handling="none", noise=0.01,
                   seed=-1, columns_to_encode=None, keep_original_categorical_columns=True, fold_column=None)


class TargetEncoderModel(Model):
    algo = "targetencoder"

    def _encode_col(self, codes, st, K, loo_y=None, fold=None, noise=0.0, gen=None, row0=0, stream=0):
        num, den = st["num"], st["den"]           # [L, K'] and [L]
        prior = st["prior"]                        # [K']
        dev = codes.device
        num = torch.as_tensor(num, dtype=torch.float64, device=dev)
        den = torch.as_tensor(den, dtype=torch.float64, device=dev)
        prior = torch.as_tensor(prior, dtype=torch.float64, device=dev)
        L = den.numel()
        na = torch.isnan(codes) | (codes >= L) | (codes < 0)
        c = torch.where(na, torch.zeros_like(codes), codes).long()
        n = den[c]
        s = num[c]
        if loo_y is not None:
            n = n - 1
            s = s - loo_y
        if fold is not None:
            n = n - st["fold_den"][fold, c]
            s = s - st["fold_num"][fold, c]
        post = s / n.clamp(min=1e-300)[:, None]
        if self.params.get("blending"):
            k, f = float(self.params["inflection_point"]), float(self.params["smoothing"])
            lam = 1.0 / (1.0 + torch.exp((k - n) / f))
            enc = lam[:, None] * post + (1 - lam[:, None]) * prior[None, :]
        else:
            enc = post
        enc = torch.where((n <= 0)[:, None] | na[:, None], prior[None, :].expand_as(enc), enc)
        if noise > 0:
            # counter-based per (global row, output column) uniforms: the same noise however rows are split
            cols = [coll.row_uniform(int(gen.initial_seed()), stream * 64 + k, row0, enc.shape[0], dev)
                    for k in range(enc.shape[1])]
            enc = enc + (torch.stack(cols, 1) * 2 - 1) * noise
        return enc

    def transform(self, frame, as_training=False, noise=None, blending=None, inflection_point=None, smoothing=None):
        from ..frame import Column, H2OFrame
        saved = dict(self.params)
        for k, v in (("blending", blending), ("inflection_point", inflection_point), ("smoothing", smoothing)):
            if v is not None:
                self.params[k] = v
        try:
            dev = self.device
            nz = float(self.params.get("noise", 0.0)) if noise is None else float(noise)
            gen = torch.Generator().manual_seed(int(self.params.get("seed") or 0) & 0x7FFFFFFF)
            leak = str(self.params.get("data_leakage_handling", "none")).lower().replace("_", "")
            y = None
            if as_training and leak == "leaveoneout":
                y = self._targets(frame, dev)
            fold = None
            if as_training and leak == "kfold":
                fold = frame._col(self.params["fold_column"]).as_float().to(dev).long()
            cols = [frame._col(n) for n in frame.names if self.params.get("keep_original_categorical_columns", True)
                    or n not in self.output["encoded_columns"]]
            sh = getattr(frame, "_shard", None)
            row0 = sh.offset if sh is not None else 0
            for ci, name in enumerate(self.output["encoded_columns"]):
                if name not in frame.names:
                    continue
                st = self.stats[name]
                codes = _codes(frame._col(name), st["domain"], dev)
                enc = self._encode_col(codes, st, self.K, y, fold, nz if as_training else 0.0, gen, row0, ci)
                if enc.shape[1] == 1:
                    cols.append(Column(f"{name}_te", "real", enc[:, 0]))
                else:
                    for k in range(enc.shape[1]):
                        cols.append(Column(f"{name}_{self.info.response_domain[k + 1]}_te", "real", enc[:, k]))
            return H2OFrame._from_columns([Column(c.name, c.type, c.data, c.domain, c.strings) for c in cols])
        finally:
            self.params.clear()
            self.params.update(saved)

    def _targets(self, frame, dev):
        from ..frame import _remap_codes
        c = frame._col(self.info.response)
        if self.info.response_domain is not None:
            yv = _remap_codes(c, self.info.response_domain, dev).double()
            if self.K == 1:
                return (yv == 1).double()[:, None]
            return torch.nn.functional.one_hot(yv.long(), len(self.info.response_domain))[:, 1:].double()
        return c.as_float().to(dev)[:, None]

    def predict(self, frame):
        return self.transform(frame)

    def _predict_tensor(self, X, offset=None):
        raise NotImplementedError("use transform()")

    def to_state(self):
        s = super().to_state()
        s["stats"] = {k: {kk: (np.asarray(vv.cpu() if torch.is_tensor(vv) else vv).tolist() if kk != "domain" else vv)
                          for kk, vv in v.items()} for k, v in self.stats.items()}
        s["K"] = self.K
        return s

    def _restore(self, s):
        super()._restore(s)
        self.K = s["K"]
        self.stats = {}
        for k, v in s["stats"].items():
            d = dict(v)
            for kk in ("fold_num", "fold_den"):
                if kk in d:
                    d[kk] = torch.tensor(d[kk], dtype=torch.float64)
            self.stats[k] = d


def _codes(col, domain, dev):
    from ..frame import _remap_codes
    return _remap_codes(col, domain, dev).double()


class TargetEncoderTrainer:
    def __init__(self, params):
        p = dict(TE_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        t0 = time.time()
        dev = X.device
        p = self.p
        cats = [j for j in range(info.F) if info.iscat[j]]
        if p.get("columns_to_encode"):
            want = [c if isinstance(c, str) else c[0] for c in p["columns_to_encode"]]
            cats = [j for j in cats if info.x[j] in want]
        if info.response_domain is not None:
            K = len(info.response_domain)
            Y = (y == 1).double()[:, None] if K == 2 else torch.nn.functional.one_hot(torch.nan_to_num(y).long(), K)[:, 1:].double()
        else:
            K = 1
            Y = y.double()[:, None]
        ok = ~torch.isnan(y)
        Y = torch.where(ok[:, None], Y, torch.zeros_like(Y))
        wt = ok.double()
        ps = _merge(torch.cat([(Y * wt[:, None]).sum(0), wt.sum().reshape(1)]))
        prior = ps[:-1] / ps[-1]
        fold = None
        if str(p["data_leakage_handling"]).lower().replace("_", "") == "kfold":
            fc = p.get("fold_column") or info.fold       # the builder hands the fold column over in DataInfo
            if not fc or fc not in info.x:
                raise ValueError("k_fold leakage handling needs fold_column")
            p["fold_column"] = fc
            fold = torch.nan_to_num(X[info.x.index(fc)]).long()
            cats = [j for j in cats if info.x[j] != fc]
            fmax = float(fold.max()) if fold.numel() else 0.0
            if coll.is_dist():
                import torch.distributed as dist
                fmax = coll.all_reduce_scalar(fmax, op=dist.ReduceOp.MAX)
            nf = int(fmax) + 1
        stats = {}
        for j in cats:
            L = len(info.domains[j])
            code = X[j]
            okc = ~torch.isnan(code) & ok
            c = torch.nan_to_num(code).long().clamp(0, max(L - 1, 0))
            num = _merge(segment_sum(c[okc], Y[okc], L))
            den = _merge(segment_sum(c[okc], torch.ones_like(c[okc], dtype=torch.float64), L))
            st = dict(num=num, den=den, prior=prior, domain=list(info.domains[j]))
            if fold is not None:
                fi = fold[okc] * L + c[okc]
                st["fold_num"] = _merge(segment_sum(fi, Y[okc], nf * L)).view(nf, L, -1)
                st["fold_den"] = _merge(segment_sum(fi, torch.ones_like(fi, dtype=torch.float64), nf * L)).view(nf, L)
            stats[info.x[j]] = st
        model = TargetEncoderModel(model_key or make_key("te"), p, info)
        model.device = dev
        model.stats = stats
        model.K = Y.shape[1]
        model.output["encoded_columns"] = list(stats)
        model.output["prior"] = prior.cpu().tolist()
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
