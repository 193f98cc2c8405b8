"""PCA and SVD (reference: ``hex/pca/PCA.java`` (GramSVD / Power / Randomized / GLRM methods,
``transform`` DEMEAN/STANDARDIZE/NORMALIZE/DESCALE/NONE, importance table), ``hex/svd/SVD.java``).

GramSVD: the P×P Gram of the transformed design matrix is one MFMA Gram kernel call (all-reduced
across ranks), eigen-decomposed in fp64 — P is small, N is huge, so the kernel does all the O(NP²)
work. Power and Randomized (subspace iteration with a Gaussian sketch, Halko et al.) run as
device GEMMs on the [N, P] matrix. Scores (``predict``) are ``Z @ V[:, :k]``; SVD also outputs
``u`` (``Z V / d``) as a frame and the singular values ``d``.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from ..ops.gram import gram
from ..parallel import collectives as coll
from .base import DataInfo, Model, make_key
from .datainfo import Expander

PCA_DEFAULTS = dict(k=1, transform="NONE", pca_method="GramSVD", pca_impl="MTJ_EVD_SYMMMATRIX", max_iterations=1000,
                    use_all_factor_levels=False, compute_metrics=True, impute_missing=False, seed=-1)
SVD_DEFAULTS = dict(nv=1, transform="NONE", svd_method="GramSVD", max_iterations=1000, use_all_factor_levels=True,
                    keep_u=True, u_name=None, seed=-1)


def _expander(info, transform, use_all, X, w):
    t = str(transform).upper()
    ex = Expander(info, standardize=t in ("STANDARDIZE", "NORMALIZE", "DESCALE"), use_all_factor_levels=use_all,
                  center_only=(t == "DEMEAN"))
    ex.fit(X, w, reduce=coll.all_reduce_ if coll.is_dist() else None)
    if t == "DESCALE":          # scale only, no centering
        ex.descale_only = True
    return ex


def _transform(ex, X):
    Z = ex.transform(X)
    if getattr(ex, "descale_only", False) and ex.nums:
        k = ex.num_off
        Z[:, k:] = Z[:, k:] + (ex.num_mean / ex.num_sd).float()[None, :]
    return Z


def _eig_top(G, k):
    evals, evecs = torch.linalg.eigh(G)
    order = torch.argsort(evals, descending=True)[:k]
    return evals[order].clamp(min=0), evecs[:, order]


def _power(Z, k, iters, gen):
    """Deflated power iteration per component (PCA.java Power method) on the (all-reduced) Gram."""
    P = Z.shape[1]
    V = torch.zeros(P, k, dtype=torch.float64, device=Z.device)
    d = torch.zeros(k, dtype=torch.float64, device=Z.device)
    Zd = Z.double()
    G = coll.all_reduce_(Zd.T @ Zd) if coll.is_dist() else Zd.T @ Zd
    for j in range(k):
        v = torch.randn(P, dtype=torch.float64, generator=gen).to(Z.device)
        v /= v.norm()
        for _ in range(iters):
            u = G @ v
            if j:
                u -= V[:, :j] @ (V[:, :j].T @ u)
            nv = u / u.norm().clamp(min=1e-300)
            if float((nv - v).abs().max()) < 1e-10:
                v = nv
                break
            v = nv
        V[:, j] = v
        d[j] = float(v @ (G @ v))
    return d, V


def _randomized(Z, k, iters, gen):
    N, P = Z.shape
    Zd = Z.double()
    q = min(P, k + 10)
    Om = torch.randn(P, q, dtype=torch.float64, generator=gen).to(Z.device)
    Y = Zd @ Om
    for _ in range(min(iters, 5)):
        Q, _ = torch.linalg.qr(Y)
        Y = Zd @ (Zd.T @ Q)
    Q, _ = torch.linalg.qr(Y)
    B = Q.T @ Zd
    _, s, Vt = torch.linalg.svd(B, full_matrices=False)
    return (s[:k] ** 2), Vt[:k].T


def _randomized_sharded(Z, k, iters, gen):
    """``_randomized`` over row shards: the range finder's orthonormalisation works on the all-reduced
    q x q Gram of Y (Q = Y M with M = U S^-1/2 from its eigendecomposition), so Q never leaves its rows
    and every product the method needs (Z^T Q, Q^T Z) is a local GEMM plus a small all-reduce."""
    N, P = Z.shape
    Zd = Z.double()
    q = min(P, k + 10)
    Om = torch.randn(P, q, dtype=torch.float64, generator=gen).to(Z.device)
    Y = Zd @ Om

    def ortho(Y):
        G = coll.all_reduce_(Y.T @ Y)
        s, U = torch.linalg.eigh(G)
        keep = s > s.max().clamp(min=1e-300) * 1e-14
        return U[:, keep] / s[keep].sqrt()[None, :]
    for _ in range(min(iters, 5)):
        M = ortho(Y)
        Y = Zd @ (coll.all_reduce_(Zd.T @ Y) @ M)
    M = ortho(Y)
    B = M.T @ coll.all_reduce_(Y.T @ Zd)
    _, s, Vt = torch.linalg.svd(B, full_matrices=False)
    return (s[:k] ** 2), Vt[:k].T


class PCAModel(Model):
    algo = "pca"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.output["model_category"] = "DimReduction"
        self.V = None
        self.expander = None

    @property
    def model_category(self):
        return "DimReduction"

    def _predict_tensor(self, X, offset=None):
        Z = _transform(self.expander, X.to(self.device))
        return (Z.double() @ self.V.to(Z.device)).float()

    def prediction_names(self):
        return [f"PC{i + 1}" for i in range(self.V.shape[1])]

    def varimp(self, use_pandas=False):
        return self.output.get("importance")

    def to_state(self):
        s = super().to_state()
        s["V"] = self.V.cpu().tolist()
        s["expander"] = self.expander.to_state()
        return s

    def _restore(self, s):
        super()._restore(s)
        self.V = torch.tensor(s["V"], dtype=torch.float64)
        self.expander = Expander.from_state(self.info, s["expander"])


class PCATrainer:
    defaults = PCA_DEFAULTS
    model_cls = PCAModel

    def __init__(self, params):
        p = dict(self.defaults)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def _k(self):
        return int(self.p["k"])

    def _method(self):
        return str(self.p.get("pca_method", "GramSVD")).lower()

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .shared_tree import resolve_seed
        t0 = time.time()
        p = self.p
        N = X.shape[1]
        dev = X.device
        w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
        if not p.get("impute_missing", True) and str(p.get("transform")).upper() != "NONE":
            w = torch.where(torch.isnan(X).any(0), torch.zeros_like(w), w)
        ex = _expander(info, p["transform"], p["use_all_factor_levels"], X, w)
        Z = _transform(ex, X)
        P = Z.shape[1]
        k = min(self._k(), P)
        gen = torch.Generator().manual_seed(resolve_seed(p.get("seed", -1)) & 0x7FFFFFFF)
        method = self._method()
        Zw = Z * w.float().sqrt()[:, None]
        if method in ("gramsvd", "glrm"):
            G = gram(Z, w.float())
            if coll.is_dist():
                G = coll.all_reduce_(G)
            ev, V = _eig_top(G, k)
        elif method == "power":
            ev, V = _power(Zw, k, int(p["max_iterations"]), gen)
        elif coll.is_dist():
            ev, V = _randomized_sharded(Zw, k, int(p["max_iterations"]), gen)
        else:
            ev, V = _randomized(Zw, k, int(p["max_iterations"]), gen)
        # sign convention: largest |loading| positive (stable across methods)
        sgn = torch.sign(V.gather(0, V.abs().argmax(0, keepdim=True)))
        V = V * torch.where(sgn == 0, torch.ones_like(sgn), sgn)
        W = coll.all_reduce_scalar(float(w.sum()))
        sdev = (ev / max(W - 1, 1)).sqrt()
        G_all = gram(Z, w.float())
        if coll.is_dist():
            G_all = coll.all_reduce_(G_all)
        total_var = float(torch.diagonal(G_all).sum()) / max(W - 1, 1)
        prop = (sdev ** 2) / max(total_var, 1e-300)
        model = self.model_cls(model_key or make_key(self.model_cls.algo), p, info)
        model.device = dev
        model.expander = ex
        model.V = V
        model.output["eigenvectors"] = dict(names=ex.names, vectors=V.cpu().tolist())
        model.output["importance"] = dict(standard_deviation=sdev.cpu().tolist(), proportion_of_variance=prop.cpu().tolist(),
                                          cumulative_proportion=torch.cumsum(prop, 0).cpu().tolist())
        model.output["std_deviation"] = sdev.cpu().tolist()
        model.output["d"] = ev.sqrt().cpu().tolist()
        self._extra(model, Z, V, ev)
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model

    def _extra(self, model, Z, V, ev):
        pass


class SVDModel(PCAModel):
    algo = "svd"

    def prediction_names(self):
        return [f"PC{i + 1}" for i in range(self.V.shape[1])]

    def d(self):
        return self.output["d"]

    def v(self):
        return self.output["eigenvectors"]["vectors"]


class SVDTrainer(PCATrainer):
    defaults = SVD_DEFAULTS
    model_cls = SVDModel

    def _k(self):
        return int(self.p["nv"])

    def _method(self):
        return str(self.p.get("svd_method", "GramSVD")).lower()

    def _extra(self, model, Z, V, ev):
        d = ev.sqrt()
        model.output["v"] = V.cpu().tolist()
        if self.p.get("keep_u", True):
            from ..frame import H2OFrame
            U = (Z.double() @ V) / d.clamp(min=1e-300)[None, :]
            # U keeps the training frame's row distribution (a sharded frame when the rows are sharded)
            import contextlib
            from ..parallel import dframe
            ctx = dframe.shard_ctx(dframe.make_shard(U.shape[0])) if coll.is_dist() else contextlib.nullcontext()
            with ctx:
                fr = H2OFrame.from_tensor(U.float(), [f"u{i + 1}" for i in range(U.shape[1])])
            model.output["u_key"] = fr.frame_id
