"""Training-frame adaptation shared by every builder (reference: ``hex/Model.java``
``CategoricalEncodingScheme`` + ``water/util/CategoricalEncoders``/``hex/ModelBuilder.java``
``_catEncoder`` (frame-level categorical encodings), ``hex/DataInfo.java`` interaction columns
(GLM ``interactions`` / ``interaction_pairs``, ``InteractionWrappedVec``) and
``hex/ModelBuilder.java:1531-1577`` / ``water/util/MRUtils.sampleFrameStratified``
(``balance_classes``, ``class_sampling_factors``, ``max_after_balance_size``, and the prior /
model class distributions used by ``GenModel.correctProbabilities``).

A :class:`FrameAdapter` records the column transforms fitted on the training frame (level lists,
eigen weights, interaction level sets) and replays them on any scoring frame, so ``predict`` /
``model_performance`` see exactly the training layout. Transforms are row-local, so they run on a
row-sharded frame without communication once their level lists are known (domains are identical on
every rank by the sharded-frame invariant).
"""
from __future__ import annotations

import math

import numpy as np
import torch

ENCODINGS = ("auto", "enum", "onehotinternal", "onehotexplicit", "binary", "eigen", "labelencoder", "sortbyresponse",
             "enumlimited")


def _codes_for(col, levels):
    """Column -> int64 codes into ``levels`` (by level string; NA / unseen -> -1)."""
    from ..frame import _level_str
    dev = col.data.device if col.type != "string" else torch.device("cpu")
    if col.type == "enum":
        lut = {s: i for i, s in enumerate(levels)}
        m = torch.tensor([lut.get(s, -1) for s in col.domain] + [-1], dtype=torch.long, device=dev)
        c = col.data.long()
        return m[torch.where(c < 0, torch.full_like(c, len(col.domain)), c)]
    lut = {s: i for i, s in enumerate(levels)}
    vals = col.to_numpy()
    out = np.array([lut.get(_level_str(v), -1) if v is not None and not (isinstance(v, float) and math.isnan(v)) else -1
                    for v in vals], dtype=np.int64)
    return torch.as_tensor(out, device=dev)


class FrameAdapter:
    def __init__(self, steps=None):
        self.steps = list(steps or [])

    def __bool__(self):
        return bool(self.steps)

    def to_state(self):
        return dict(steps=self.steps)

    @staticmethod
    def from_state(s):
        return FrameAdapter(s.get("steps") if s else [])

    def apply(self, fr):
        """Replay the fitted transforms on ``fr`` (returns a new frame with the derived columns)."""
        from ..frame import Column, H2OFrame
        from ..parallel import dframe
        if not self.steps:
            return fr
        cols = {n: fr._col(n) for n in fr.names}
        dev = next(iter(cols.values())).data.device if cols and next(iter(cols.values())).type != "string" else None
        n = fr._nlocal
        out = dict(cols)
        for st in self.steps:
            k = st["kind"]
            src = cols.get(st["col"]) if "col" in st else None
            if k in ("onehotexplicit", "binary", "eigen", "labelencoder", "sortbyresponse", "enumlimited") and src is None:
                continue
            if k == "onehotexplicit":
                c = _codes_for(src, st["levels"])
                for i, lv in enumerate(st["levels"]):
                    out[f"{st['col']}.{lv}"] = Column(f"{st['col']}.{lv}", "int", (c == i).double())
                out[f"{st['col']}.missing(NA)"] = Column(f"{st['col']}.missing(NA)", "int", (c < 0).double())
                out.pop(st["col"], None)
            elif k == "binary":
                c = _codes_for(src, st["levels"]) + 1          # 0 = NA / unseen
                for b in range(st["nbits"]):
                    out[f"{st['col']}:{b}"] = Column(f"{st['col']}:{b}", "int", ((c >> b) & 1).double())
                out.pop(st["col"], None)
            elif k == "labelencoder":
                c = _codes_for(src, st["levels"]).double()
                out[st["col"]] = Column(st["col"], "int", torch.where(c < 0, torch.full_like(c, float("nan")), c))
            elif k == "sortbyresponse":
                c = _codes_for(src, st["levels"])
                rank = torch.tensor(st["rank"] + [-1], dtype=torch.float64, device=c.device)
                v = rank[torch.where(c < 0, torch.full_like(c, len(st["levels"])), c)]
                out[st["col"]] = Column(st["col"], "int", torch.where(v < 0, torch.full_like(v, float("nan")), v))
            elif k == "enumlimited":
                c = _codes_for(src, st["levels"])
                keep = st["keep_idx"]
                m = torch.full((len(st["levels"]) + 1,), len(keep), dtype=torch.int32, device=c.device)
                for i, j in enumerate(keep):
                    m[j] = i
                m[-1] = -1
                codes = m[torch.where(c < 0, torch.full_like(c, len(st["levels"])), c)]
                out[st["col"]] = Column(st["col"], "enum", codes.to(torch.int32), [st["levels"][j] for j in keep] + ["other"])
            elif k == "eigen":
                c = _codes_for(src, st["levels"])
                vec = torch.tensor(st["vec"] + [0.0], dtype=torch.float64, device=c.device)
                out[f"{st['col']}.Eigen"] = Column(f"{st['col']}.Eigen", "real",
                                                   vec[torch.where(c < 0, torch.full_like(c, len(st["levels"])), c)])
                out.pop(st["col"], None)
            elif k == "interaction":
                a, b = cols.get(st["a"]), cols.get(st["b"])
                if a is None or b is None:
                    continue
                t = st["type"]
                if t == "nn":
                    out[st["name"]] = Column(st["name"], "real", a.as_float().double() * b.as_float().double())
                elif t == "cn":
                    ca = _codes_for(a, st["levels"])
                    xb = b.as_float().double()
                    for i, lv in enumerate(st["levels"]):
                        nm = f"{st['a']}_{lv}:{st['b']}"
                        out[nm] = Column(nm, "real", torch.where(ca == i, xb, torch.zeros_like(xb)))
                else:
                    ca, cb = _codes_for(a, st["la"]), _codes_for(b, st["lb"])
                    key = ca * (len(st["lb"]) + 1) + cb
                    lut = torch.full(((len(st["la"]) + 1) * (len(st["lb"]) + 1),), -1, dtype=torch.int32, device=ca.device)
                    for i, (ia, ib) in enumerate(st["pairs"]):
                        lut[ia * (len(st["lb"]) + 1) + ib] = i
                    codes = torch.where((ca < 0) | (cb < 0), torch.full_like(ca, -1), lut[key.clamp(min=0)].long())
                    dom = [f"{st['la'][ia]}_{st['lb'][ib]}" for ia, ib in st["pairs"]]
                    out[st["name"]] = Column(st["name"], "enum", codes.to(torch.int32), dom)
        with dframe.shard_ctx(fr._shard):
            return H2OFrame._from_columns([Column(c.name if c.name == nm else nm, c.type, c.data, c.domain, c.strings)
                                           for nm, c in out.items()])


def fit_adapter(algo: str, p: dict, fr, x: list, y):
    """Fit the frame transforms the parameters ask for. Returns (adapter, adapted frame, new x)."""
    from ..parallel import dframe
    steps = []
    enc = str(p.get("categorical_encoding") or "AUTO").lower().replace("_", "")
    if enc not in ENCODINGS:
        raise ValueError(f"categorical_encoding must be one of {ENCODINGS}, got {p.get('categorical_encoding')!r}")
    if enc == "onehotinternal" and algo not in ("glm", "deeplearning", "gam", "anovaglm", "modelselection", "kmeans",
                                                 "pca", "svd", "glrm", "psvm", "coxph", "naivebayes", "aggregator"):
        raise ValueError(f"categorical_encoding=OneHotInternal is not available for {algo} (ModelBuilder.init)")
    cat_x = [n for n in x if fr.type(n) == "enum"]
    new_x = list(x)
    if enc in ("onehotexplicit", "binary", "eigen", "labelencoder", "sortbyresponse", "enumlimited") and cat_x:
        yv = None
        if enc == "sortbyresponse":
            if y is None:
                raise ValueError("categorical_encoding=SortByResponse needs a response")
            yc = fr._col(y)
            yv = yc.as_float().double() if yc.type != "enum" else yc.data.double()
            if yc.type == "enum":
                yv = torch.where(yc.data < 0, torch.full_like(yv, float("nan")), yv)
        maxl = int(p.get("max_categorical_levels") or 10)
        for n in cat_x:
            c = fr._col(n)
            levels = list(c.domain)
            if enc == "onehotexplicit":
                steps.append(dict(kind="onehotexplicit", col=n, levels=levels))
                i = new_x.index(n)
                new_x[i:i + 1] = [f"{n}.{lv}" for lv in levels] + [f"{n}.missing(NA)"]
            elif enc == "binary":
                nbits = max(1, int(math.ceil(math.log2(len(levels) + 1))))
                steps.append(dict(kind="binary", col=n, levels=levels, nbits=nbits))
                i = new_x.index(n)
                new_x[i:i + 1] = [f"{n}:{b}" for b in range(nbits)]
            elif enc == "labelencoder":
                steps.append(dict(kind="labelencoder", col=n, levels=levels))
            elif enc == "sortbyresponse":
                codes = c.data.long()
                ok = (codes >= 0) & ~torch.isnan(yv)
                L = len(levels)
                s = torch.zeros(L, dtype=torch.float64, device=codes.device).index_add_(0, codes[ok], yv[ok])
                k = torch.zeros(L, dtype=torch.float64, device=codes.device).index_add_(0, codes[ok], torch.ones_like(yv[ok]))
                if fr._shard is not None:
                    from ..parallel import collectives as coll
                    parts = coll.all_gather_object((s.cpu().numpy(), k.cpu().numpy()))
                    s = torch.as_tensor(np.sum([q[0] for q in parts], 0))
                    k = torch.as_tensor(np.sum([q[1] for q in parts], 0))
                mean = (s / k.clamp(min=1)).cpu().numpy()
                mean = np.where(k.cpu().numpy() > 0, mean, np.inf)
                order = np.argsort(mean, kind="stable")
                rank = np.empty(L, dtype=np.int64)
                rank[order] = np.arange(L)
                steps.append(dict(kind="sortbyresponse", col=n, levels=levels, rank=rank.tolist()))
            elif enc == "enumlimited":
                cnt = torch.bincount(c.data[c.data >= 0].long(), minlength=len(levels)).double().cpu().numpy()
                if fr._shard is not None:
                    from ..frame import coll_all_reduce_np
                    cnt = coll_all_reduce_np(cnt)
                keep = sorted(np.argsort(-cnt, kind="stable")[:maxl].tolist())
                steps.append(dict(kind="enumlimited", col=n, levels=levels, keep_idx=keep))
            elif enc == "eigen":
                # first eigenvector of the one-hot covariance (CategoricalEncoders EigenEncoder)
                L = len(levels)
                cnt = torch.bincount(c.data[c.data >= 0].long(), minlength=L).double().cpu().numpy()
                if fr._shard is not None:
                    from ..frame import coll_all_reduce_np
                    cnt = coll_all_reduce_np(cnt)
                tot = max(cnt.sum(), 1.0)
                pr = cnt / tot
                cov = np.diag(pr) - np.outer(pr, pr)
                ev, V = np.linalg.eigh(cov)
                v = V[:, np.argmax(ev)]
                v = v * (1.0 if v[np.argmax(np.abs(v))] >= 0 else -1.0)
                steps.append(dict(kind="eigen", col=n, levels=levels, vec=v.tolist()))
                i = new_x.index(n)
                new_x[i] = f"{n}.Eigen"
    if algo in ("glm", "gam", "coxph") and (p.get("interactions") or p.get("interaction_pairs")):
        pairs = []
        inter = p.get("interactions") or []
        inter = [inter] if isinstance(inter, str) else list(inter)
        for i, a in enumerate(inter):
            for b in inter[i + 1:]:
                pairs.append((a, b))
        for pr in p.get("interaction_pairs") or []:
            pairs.append(tuple(pr))
        for a, b in pairs:
            if a not in fr.names or b not in fr.names:
                raise ValueError(f"interaction column {a if a not in fr.names else b} is not in the frame")
            ta, tb = fr.type(a) == "enum", fr.type(b) == "enum"
            if ta and not tb:
                steps.append(dict(kind="interaction", type="cn", a=a, b=b, levels=list(fr._col(a).domain)))
                new_x += [f"{a}_{lv}:{b}" for lv in fr._col(a).domain]
            elif tb and not ta:
                steps.append(dict(kind="interaction", type="cn", a=b, b=a, levels=list(fr._col(b).domain)))
                new_x += [f"{b}_{lv}:{a}" for lv in fr._col(b).domain]
            elif not ta and not tb:
                steps.append(dict(kind="interaction", type="nn", a=a, b=b, name=f"{a}:{b}"))
                new_x.append(f"{a}:{b}")
            else:
                ca, cb = fr._col(a), fr._col(b)
                la, lb = list(ca.domain), list(cb.domain)
                key = ca.data.long() * (len(lb) + 1) + cb.data.long()
                ok = (ca.data >= 0) & (cb.data >= 0)
                u = torch.unique(key[ok])
                if fr._shard is not None:
                    u = dframe.global_unique(u.double()).long()
                seen = [(int(v) // (len(lb) + 1), int(v) % (len(lb) + 1)) for v in u.cpu().tolist()]
                steps.append(dict(kind="interaction", type="cc", a=a, b=b, la=la, lb=lb, pairs=seen, name=f"{a}_{b}"))
                new_x.append(f"{a}_{b}")
        if algo == "coxph" and p.get("interactions_only"):
            # CoxPH interactions_only: these columns enter the model only through their interaction terms
            only = p["interactions_only"]
            only = {only} if isinstance(only, str) else set(only)
            new_x = [c for c in new_x if c not in only]
    if not steps:
        return None, fr, x
    ad = FrameAdapter(steps)
    return ad, ad.apply(fr), new_x


# ------------------------------------------------------------------------------------------------
def balance_indices(p: dict, y: torch.Tensor, K: int, row0: int = 0):
    """Row replication counts for ``balance_classes`` (MRUtils.sampleFrameStratified semantics:
    per-class sampling factors — given, or computed for equal class counts — scaled so the balanced
    frame is at most ``max_after_balance_size`` x the original). Each row of class c appears
    floor(f_c) times plus once more with probability frac(f_c), drawn per GLOBAL row index.
    Returns (index tensor, prior class distribution, model class distribution)."""
    from ..parallel import collectives as coll
    dev = y.device
    yl = torch.nan_to_num(y.double(), nan=-1).long()
    cnt = torch.bincount(yl[yl >= 0], minlength=K).double()
    cnt = coll.all_reduce_(cnt) if coll.is_dist() else cnt
    n = float(cnt.sum())
    f = p.get("class_sampling_factors")
    if f:
        f = torch.tensor([float(v) for v in f], dtype=torch.float64, device=dev)
        if f.numel() != K:
            raise ValueError(f"class_sampling_factors must have {K} entries")
    else:
        f = (n / K) / cnt.clamp(min=1)
    after = float((f * cnt).sum())
    cap = float(p.get("max_after_balance_size") or 5.0) * n
    if after > cap:
        f = f * (cap / after)
    fr_ = f[yl.clamp(min=0)]
    fr_ = torch.where(yl >= 0, fr_, torch.ones_like(fr_))
    u = coll.row_uniform(int(p.get("seed") or 0), 0xBA1A, row0, y.numel(), dev)
    reps = torch.floor(fr_).long() + (u < (fr_ - torch.floor(fr_))).long()
    idx = torch.repeat_interleave(torch.arange(y.numel(), device=dev), reps)
    prior = (cnt / max(n, 1.0)).cpu().tolist()
    mcnt = cnt * f
    model_dist = (mcnt / mcnt.sum().clamp(min=1e-300)).cpu().tolist()
    return idx, prior, model_dist


def correct_probabilities(P: torch.Tensor, prior, model_dist) -> torch.Tensor:
    """GenModel.correctProbabilities: undo the class re-weighting of a balanced training frame."""
    pr = torch.as_tensor(prior, dtype=P.dtype, device=P.device)
    md = torch.as_tensor(model_dist, dtype=P.dtype, device=P.device)
    Q = P * (pr / md.clamp(min=1e-300))[None, :]
    return Q / Q.sum(1, keepdim=True).clamp(min=1e-300)
