"""K-Means (reference: ``hex/kmeans/KMeans.java``, ``KMeansModel.java``).

Init: Random, PlusPlus (k-means++), Furthest, User; ``standardize`` via the expander (one-hot
categoricals, mean-imputed numerics — H2O's DataInfo for KMeans); Lloyd iterations with the fused
HIP assign kernel (``ops.dense.kmeans_assign``) and device ``index_add_`` centroid sums, all-reduced
across ranks; empty clusters are re-seeded from the farthest point; ``estimate_k`` grows k until
the relative reduction of within-SS falls below the H2O criterion. Outputs centers (raw and
standardized), within/between/total SS, cluster sizes.
"""
from __future__ import annotations

import math
import time

import numpy as np
import torch

from .. import metrics as mm
from ..ops.dense import kmeans_assign, kmeans_lloyd_step, kmeans_step
from ..parallel import collectives as coll
from .base import DataInfo, Model, make_key
from .datainfo import Expander
from ..ops.segment import segment_sum

KM_DEFAULTS = dict(k=1, max_iterations=10, standardize=True, init="Furthest", user_points=None, estimate_k=False,
                   seed=-1, cluster_size_constraints=None)


class KMeansModel(Model):
    algo = "kmeans"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.output["model_category"] = "Clustering"
        self.centers_std = None
        self.expander = None

    @property
    def model_category(self):
        return "Clustering"

    def _predict_tensor(self, X, offset=None):
        Z = self.expander.transform(X.to(self.device))
        a, _ = kmeans_assign(Z, self.centers_std.to(Z.device))
        return a.float()

    def predict(self, frame):
        from ..frame import Column, H2OFrame
        X, _ = frame.model_matrix(self.info, device=self.device)
        a = self._predict_tensor(X)
        return H2OFrame._from_columns([Column("predict", "int", a.double())])

    def metrics_for(self, X, y, w=None, offset=None):
        """Clustering metrics of a scored frame (ModelMetricsClustering: within / between / total SS, sizes) in the
        model's standardized space (the sums of squares are translation invariant)."""
        Z = self.expander.transform(X.to(self.device))
        C = self.centers_std.to(Z.device)
        if Z.shape[1] < C.shape[1]:
            Z = torch.nn.functional.pad(Z, (0, C.shape[1] - Z.shape[1]))
        a, _ = kmeans_assign(Z, C)
        return mm.clustering_metrics(Z, C, a, None if w is None else w.to(Z.device).double())

    def num_iterations(self):
        return int(self.output.get("iterations") or 0)

    def centroid_stats(self, train=False, valid=False):
        """Per-centroid table (centroid, size, within_cluster_sum_of_squares) as in ModelMetricsClustering."""
        import pandas as pd
        m = self.output.get("validation_metrics" if valid else "training_metrics") or {}
        size, within = m.get("size") or [], m.get("withinss") or []
        return pd.DataFrame(dict(centroid=list(range(1, len(size) + 1)), size=size,
                                 within_cluster_sum_of_squares=within))

    def centers(self):
        return self.output["centers"]

    def centers_std(self):  # noqa: F811 - h2o-py accessor
        return self.output["centers_std"]

    def size(self):
        return self.output["training_metrics"]["size"]

    def tot_withinss(self, *a, **k):
        return self.output["training_metrics"]["tot_withinss"]

    def betweenss(self, *a, **k):
        return self.output["training_metrics"]["betweenss"]

    def totss(self, *a, **k):
        return self.output["training_metrics"]["totss"]

    def withinss(self, *a, **k):
        return self.output["training_metrics"]["withinss"]

    def to_state(self):
        s = super().to_state()
        s["centers_std"] = self.centers_std.cpu().tolist()
        s["expander"] = self.expander.to_state()
        return s

    def _restore(self, s):
        super()._restore(s)
        self.centers_std = torch.tensor(s["centers_std"], dtype=torch.float32)
        self.expander = Expander.from_state(self.info, s["expander"])


class KMeansTrainer:
    def __init__(self, params):
        p = dict(KM_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    # ---- global-row helpers: the init / re-seed rules pick rows by GLOBAL index, so a row-sharded run
    # picks exactly the rows of the single-process run (the owner rank contributes the row)
    def _row(self, Z, j: int) -> torch.Tensor:
        """Row ``j`` (global index) of Z on every rank."""
        if not coll.is_dist():
            return Z[j:j + 1].clone()
        r = torch.zeros(1, Z.shape[1], dtype=torch.float64, device=Z.device)
        if self.row0 <= j < self.row0 + Z.shape[0]:
            r[0] = Z[j - self.row0].double()
        return coll.all_reduce_(r).float()

    def _argmax(self, v: torch.Tensor) -> int:
        """Global index of the first maximum of a row vector."""
        if not coll.is_dist():
            return int(torch.argmax(v))
        j = int(torch.argmax(v)) if v.numel() else 0
        best = float(v[j]) if v.numel() else float("-inf")
        parts = coll.all_gather_object((best, self.row0 + j))
        top = max(p[0] for p in parts)
        return min(p[1] for p in parts if p[0] == top)

    def _init_centers(self, Z, k, rng, how):
        N = self.N_glob
        dev = Z.device
        if how == "user" and self.p.get("user_points") is not None:
            up = self.p["user_points"]
            U = up.as_tensor() if hasattr(up, "as_tensor") else torch.as_tensor(np.asarray(up, dtype=np.float32))
            # decide the space of the points BEFORE transforming / padding them: original-feature points are
            # centred by ex_train.transform already; only design-space points still need the shift
            orig = U.shape[1] == self.info.F
            U = self.ex_train.transform(U.T.contiguous().to(dev)) if orig else U.to(dev).float()
            if U.shape[1] < Z.shape[1]:
                U = torch.nn.functional.pad(U, (0, Z.shape[1] - U.shape[1]))
            if self.ex_train is not self.ex and not orig:   # user points given in design space
                U = U - torch.nn.functional.pad(self._shift, (0, Z.shape[1] - self._shift.numel())).float()
            return U
        first = int(rng.integers(N))
        C = self._row(Z, first)
        if how == "random":
            idx = rng.choice(N, size=min(k, N), replace=False)
            if not coll.is_dist():
                return Z.index_select(0, torch.as_tensor(idx, dtype=torch.long, device=dev)).clone()
            return torch.cat([self._row(Z, int(j)) for j in idx], 0)
        if not coll.is_dist() and Z.is_cuda:
            state = rng.bit_generator.state
            Cd = self._init_device(Z, C, k, rng, how)
            if Cd is not None:
                return Cd
            rng.bit_generator.state = state
        while C.shape[0] < k:
            _, d = kmeans_assign(Z, C)
            if how == "plusplus":
                pr = d.double().clamp(min=0)
                s = coll.all_reduce_scalar(float(pr.sum()))
                if s <= 0:
                    break
                u = rng.random() * s
                before = 0.0
                if coll.is_dist():      # mass held by lower ranks: exclusive scan of the per-rank sums
                    sums = coll.all_gather_object(float(pr.sum()))
                    before = float(sum(sums[:coll.rank()]))
                cs = torch.cumsum(pr, 0) + before
                jl = int(torch.searchsorted(cs, torch.tensor([u], dtype=torch.float64, device=dev))[0])
                mine = jl < pr.numel() and (before < u or coll.rank() == 0)
                j = self.row0 + jl if mine else N
                j = int(min(coll.all_gather_object(j))) if coll.is_dist() else j
                j = min(j, N - 1)
            else:  # furthest
                j = self._argmax(d)
            C = torch.cat([C, self._row(Z, j)], 0)
        return C

    def _init_device(self, Z, C, k, rng, how):
        """Furthest / PlusPlus seeding with every choice made on the device (no host sync per center).
        PlusPlus draws the same uniforms as the host loop; if some step had no distance mass left (the
        host loop stops early there) the result is discarded and the host loop runs instead."""
        dev = Z.device
        masses = []
        while C.shape[0] < k:
            _, d = kmeans_assign(Z, C)
            if how == "plusplus":
                pr = d.double().clamp(min=0)
                s = pr.sum()
                masses.append(s)
                u = float(rng.random()) * s
                j = torch.searchsorted(torch.cumsum(pr, 0), u.view(1)).clamp_(max=Z.shape[0] - 1)
            else:
                j = torch.argmax(d).view(1)            # first maximum, as _argmax
            C = torch.cat([C, Z.index_select(0, j)], 0)
        if masses and bool((torch.stack(masses) <= 0).any()):
            return None
        return C

    @staticmethod
    def constrained_assign(D, mins):
        """Assignment with minimum cluster sizes (KMeans cluster_size_constraints: the reference solves a
        min-cost flow per iteration): the transportation LP min Σ D_ik x_ik, Σ_k x_ik = 1, Σ_i x_ik >= m_k,
        whose constraint matrix is totally unimodular, so HiGHS returns an integral assignment."""
        import scipy.sparse as sp
        from scipy.optimize import linprog
        N, K = D.shape
        Dn = D.double().cpu().numpy()
        rows = np.repeat(np.arange(N), K)
        cols = np.arange(N * K)
        A_eq = sp.csr_matrix((np.ones(N * K), (rows, cols)), shape=(N, N * K))
        A_ub = sp.csr_matrix((-np.ones(N * K), (np.tile(np.arange(K), N), cols)), shape=(K, N * K))
        res = linprog(Dn.reshape(-1), A_ub=A_ub, b_ub=-np.asarray(mins, dtype=np.float64), A_eq=A_eq,
                      b_eq=np.ones(N), bounds=(0, 1), method="highs")
        if not res.success:
            raise ValueError(f"cluster_size_constraints cannot be met: {res.message}")
        return torch.as_tensor(res.x.reshape(N, K).argmax(1), device=D.device)

    def _lloyd_constrained(self, Z, w, C, max_it, mins):
        K = C.shape[0]
        if len(mins) != K:
            raise ValueError(f"cluster_size_constraints needs {K} values")
        if sum(mins) > Z.shape[0]:
            raise ValueError("the sum of cluster_size_constraints exceeds the number of rows")
        if Z.shape[0] * K > 4_000_000:
            raise ValueError("cluster_size_constraints is available for frames with rows x k <= 4e6")
        wd = torch.ones(Z.shape[0], dtype=torch.float64, device=Z.device) if w is None else w.double()
        a_prev = None
        for it in range(max_it):
            D = torch.cdist(Z.double(), C.double()) ** 2
            a = self.constrained_assign(D, mins)
            oh = torch.nn.functional.one_hot(a, K).double() * wd[:, None]
            cnt = oh.sum(0)
            C = torch.where(cnt[:, None] > 0, (oh.T @ Z.double()) / cnt.clamp(min=1e-300)[:, None], C.double()).float()
            if a_prev is not None and bool((a == a_prev).all()):
                break
            a_prev = a
        d = ((Z.double() - C.double()[a]) ** 2).sum(1).float()
        return C, a, d, it + 1

    def _step(self, Z, w, C):
        """One Lloyd step on the device: (assign, min distance, new centers, cnt, flags [#empty, shift])."""
        if not coll.is_dist():
            # the kernel's row weights: none for unit weights (no 40 MB weight read and no fp64 -> fp32 cast per
            # iteration), else the fp32 copy made once per Lloyd loop
            wk = getattr(self, "_wk", w)
            if wk is not None and wk.numel() != Z.shape[0]:
                wk = w
            r = kmeans_lloyd_step(Z, C, wk)      # MFMA step + fused center update (2 launches + the slab sum)
            if r is not None:
                d, newC, cnt, flags = r
                return None, d, newC, cnt, flags
        a, d, sums, cnt = kmeans_step(Z, C, w, need_assign=False)
        if coll.is_dist():
            sums = coll.all_reduce_(sums)
            cnt = coll.all_reduce_(cnt)
        newC = torch.where(cnt[:, None] > 0, sums / cnt.clamp(min=1e-300)[:, None], C.double()).float()
        flags = torch.stack([(cnt == 0).sum().double(), (newC - C).abs().max().double()])
        return a, d, newC, cnt, flags

    def _reseed(self, Z, newC, cnt, d):
        """Empty clusters are re-seeded, in cluster order, at the currently worst-fit row (KMeans.java)."""
        for e in torch.nonzero(cnt == 0).flatten().tolist():
            j = self._argmax(d)
            newC[e] = self._row(Z, j)[0]
            if 0 <= j - self.row0 < d.numel():
                d[j - self.row0] = 0
        return newC

    def _lloyd(self, Z, w, C, max_it):
        self._wk = None if getattr(self, "_unit_w", False) else w.float().contiguous()
        csc = self.p.get("cluster_size_constraints")
        if csc:
            if coll.is_dist():
                raise ValueError("cluster_size_constraints needs a single-process frame")
            return self._lloyd_constrained(Z, w, C, max_it, [int(v) for v in csc])
        tol = 1e-6
        if not Z.is_cuda or coll.is_dist():
            it = 0
            for it in range(max_it):
                a, d, newC, cnt, flags = self._step(Z, w, C)
                n_empty, shift = flags.tolist()          # one host sync per iteration
                if n_empty > 0:
                    newC = self._reseed(Z, newC, cnt, d)
                    shift = float((newC - C).abs().max())
                C = newC
                if self.job is not None:
                    self.job.check_cancelled()
                if shift < tol:
                    break
            a, d = kmeans_assign(Z, C)
            return C, a, d, it + 1
        # single device: no blocking host sync inside the loop. Iteration i's flags travel to pinned host
        # memory while iteration i+1 is already queued on the speculation that i re-seeded nothing and did
        # not converge; a (rare) re-seed discards the speculative step, convergence discards it unused.
        # Same iterates and iteration count as the synchronous loop.
        pinned = torch.empty(2, dtype=torch.float64, pin_memory=True)
        ev = torch.cuda.Event()
        it = 0
        cur = self._step(Z, w, C)
        while True:
            a, d, newC, cnt, flags = cur
            pinned.copy_(flags, non_blocking=True)
            ev.record()
            nxt = self._step(Z, w, newC) if it + 1 < max_it else None
            ev.synchronize()
            n_empty, shift = float(pinned[0]), float(pinned[1])
            if n_empty > 0:
                newC = self._reseed(Z, newC, cnt, d)
                shift = float((newC - C).abs().max())
                nxt = None
            it += 1
            C = newC
            if self.job is not None:
                self.job.check_cancelled()
            if shift < tol or it >= max_it:
                break
            cur = nxt if nxt is not None else self._step(Z, w, C)
        a, d = kmeans_assign(Z, C)
        return C, a, d, it

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .shared_tree import resolve_seed
        t0 = time.time()
        p = self.p
        self.info = info
        dev = X.device
        N = X.shape[1]
        seed = resolve_seed(p["seed"])
        rng = np.random.default_rng(seed & 0xFFFFFFFF)
        self._unit_w = w is None
        w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
        self.row0, self.N_glob = (coll.exclusive_offset(N) if coll.is_dist() else (0, N))
        self.ex = Expander(info, standardize=p["standardize"], use_all_factor_levels=True).fit(
            X, w, reduce=coll.all_reduce_ if coll.is_dist() else None)
        # Training runs in a translated space: without standardisation the numeric columns are still centred
        # (k-means is translation invariant) so the MFMA distance GEMM ||c||^2 - 2 x.c does not cancel on
        # data with large column offsets; centers move back by `shift` at the end.
        import copy
        self.ex_train = self.ex
        shift = None
        if not self.ex.standardize and self.ex.nums:
            self.ex_train = copy.copy(self.ex)
            self.ex_train.center_only = True
            shift = torch.zeros(self.ex.P, dtype=torch.float64, device=dev)
            shift[self.ex.num_off:] = self.ex.num_mean.to(dev).double()
        self._shift = shift
        Z = self.ex_train.transform(X)
        P0 = Z.shape[1]
        if Z.is_cuda and P0 % 4 and P0 <= 64:      # the MFMA Lloyd kernel streams rows as float4 groups
            Z = torch.nn.functional.pad(Z, (0, 4 - P0 % 4))
        how = str(p["init"]).lower().replace("_", "")
        max_it = int(p["max_iterations"])
        if p["estimate_k"]:
            # KMeans.java: deterministic growth from k=1, split the worst cluster, stop when the relative
            # within-SS improvement falls under min(0.02 + 10/N + 2.5/F^2, 0.8) and keep the previous k
            kmax = int(p["k"])
            cutoff = min(0.02 + 10.0 / self.N_glob + 2.5 / max(info.F, 1) ** 2, 0.8)
            sw = coll.all_reduce_scalar(float(w.sum()))
            C0 = (coll.all_reduce_((Z.double() * w[:, None]).sum(0, keepdim=True)) / sw).float()
            prev = None
            best = None
            for k in range(1, kmax + 1):
                Ck, ak, dk, it = self._lloyd(Z, w, C0, max_it)
                wss = coll.all_reduce_scalar(float((dk.double() * w).sum()))
                if prev is not None and (prev - wss) / max(prev, 1e-300) < cutoff:
                    break
                best, prev = (Ck, ak, dk, it), wss
                if k == kmax:
                    break
                per = coll.all_reduce_(segment_sum(ak, dk.double() * w, Ck.shape[0]))
                worst = int(torch.argmax(per))
                far = self._argmax(torch.where(ak == worst, dk, torch.full_like(dk, -1.0)))
                C0 = torch.cat([Ck, self._row(Z, far)], 0)
            C, a, d, iters = best
        else:
            C0 = self._init_centers(Z, int(p["k"]), rng, how)
            C, a, d, iters = self._lloyd(Z, w, C0, max_it)
        met = mm.clustering_metrics(Z, C, a, w)           # translation invariant: the training space is fine
        if valid is not None:
            Zv = self.ex_train.transform(valid[0])
            if Zv.shape[1] < Z.shape[1]:
                Zv = torch.nn.functional.pad(Zv, (0, Z.shape[1] - Zv.shape[1]))
            av, _ = kmeans_assign(Zv, C)
            vmet = mm.clustering_metrics(Zv, C, av)
        C = C[:, :P0]
        if shift is not None:
            C = (C.double() + shift[None, :]).float()
        model = KMeansModel(model_key or make_key("kmeans"), p, info)
        model.device = dev
        model.expander = self.ex
        model.centers_std = C
        raw = C.double().clone()
        if self.ex.standardize and self.ex.nums:
            k0 = self.ex.num_off
            raw[:, k0:] = raw[:, k0:] * self.ex.num_sd[None, :] + self.ex.num_mean[None, :]
        model.output["centers_std"] = C.cpu().tolist()
        model.output["centers"] = raw.cpu().tolist()
        model.output["center_names"] = self.ex.names
        model.output["k"] = C.shape[0]
        model.output["iterations"] = iters
        model.output["training_metrics"] = met
        if valid is not None:
            model.output["validation_metrics"] = vmet
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
