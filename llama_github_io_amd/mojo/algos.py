"""Reference-layout MOJO payloads beyond the tree / GLM / KMeans families.

Each ``write_*`` fills ``model.ini`` keys (``kv``) and binary/text entries (``blobs``) exactly as the
reference writer does, so the zip is readable by h2o-genmodel; each ``score_*`` reproduces the
reference genmodel scorer on device tensors (``GenericModel`` dispatches to them):

* DeepLearning — ``h2o-algos/.../deeplearning/DeepLearningMojoWriter.java:writeModelData``,
  ``h2o-genmodel/.../algos/deeplearning/DeeplearningMojoModel.java:score0`` / ``NeuralNetwork.java``
  (weights ``[out][in]`` row-major, Maxout ``[out][in][k]``; categoricals first, one-hot with an extra
  NA level per column; numerics ``(x - norm_sub) * norm_mul``, NA -> 0).
* PCA — ``algos/pca/PCAMojoReader.java`` / ``PCAMojoModel.java:score0`` (``eigenvectors_raw``
  big-endian doubles, ``permutation`` cats-then-nums).
* Word2Vec — ``algos/word2vec/Word2VecMojoReader.java`` (``vectors`` big-endian float32 blob,
  ``vocabulary`` text).
* Isotonic regression — ``ModelMojoReader.readIsotonicCalibrator`` (``calib/thresholds_x|y``: int32
  count + big-endian doubles).
* Stacked ensemble — ``MultiModelMojoReader`` / ``StackedEnsembleMojoReader.java`` (nested MOJOs under
  ``models/<key>/``, ``base_model<i>`` / ``metalearner`` keys).
* Extended isolation forest — ``algos/isoforextended/ExtendedIsolationForestMojoModel.java:scoreTree0``
  (heap-numbered 'N'/'L' node records per ``trees/tNN.bin``).

Our own trainers differ from H2O in two imputation details that the writers fold into the exported
parameters so the reference scorer reproduces this framework's predictions: DeepLearning imputes a
missing categorical with its training mode (exported as an NA level whose first-layer weights are the
mode level's), and dropout is inverted at training time (exported ratios are 0).
"""
from __future__ import annotations

import struct

import numpy as np
import torch

_ACT = {"rectifier": "Rectifier", "tanh": "Tanh", "exprectifier": "ExpRectifier", "maxout": "Maxout",
        "linear": "Linear"}


def _arr(v):
    return "[" + ", ".join(repr(float(x)) if isinstance(x, float) else str(x) for x in v) + "]"


def _darr(v):
    return "[" + ", ".join(repr(float(x)) for x in v) + "]"


# ================================================================================================ DL
def dl_columns(model):
    """DeepLearning MOJOs list categorical predictors first (the reference DataInfo column order)."""
    info = model.info
    ex = model.expander
    order = list(ex.cats) + list(ex.nums)
    cols = [info.x[j] for j in order] + ([info.response] if info.response else [])
    doms = [info.domains[j] for j in order] + ([info.response_domain] if info.response else [])
    return cols, doms


def write_deeplearning(model, kv, blobs):
    if getattr(getattr(model, "expander", None), "cat_hash", None):
        raise NotImplementedError("DeepLearning with max_categorical_features hashing has no MOJO/POJO layout")
    ex = model.expander
    cfg = model._cfg
    info = model.info
    start = 0 if ex.use_all else 1
    # reference one-hot block per categorical: (L - start) levels + 1 NA level
    ref_off, src_cols = [0], []
    for i, j in enumerate(ex.cats):
        L = len(info.domains[j] or [])
        n = L - start
        src_cols += [ex.cat_offsets[i] + c for c in range(n)]
        mode_col = ex.cat_offsets[i] + ex.cat_modes[i] - start if ex.cat_modes[i] - start >= 0 else -1
        src_cols.append(mode_col)                      # NA level -> the mode level's weights (our imputation)
        ref_off.append(ref_off[-1] + n + 1)
    src_cols += [ex.num_off + k for k in range(len(ex.nums))]
    lins = list(model.net.hidden) + [model.net.out]
    units = [len(src_cols)] + list(cfg["hidden"]) + [int(cfg["n_out"])]
    maxout = bool(cfg["maxout"])
    act = "Maxout" if maxout else _ACT.get(str(cfg["act"]).lower(), "Rectifier")
    kv["mini_batch_size"] = 1
    kv["nums"] = len(ex.nums)
    kv["cats"] = len(ex.cats)
    kv["cat_offsets"] = _arr(ref_off)
    if ex.standardize and ex.nums:
        kv["norm_mul"] = _darr((1.0 / ex.num_sd).cpu().tolist())
        kv["norm_sub"] = _darr(ex.num_mean.cpu().tolist())
    else:
        kv["norm_mul"] = "null"
        kv["norm_sub"] = "null"
    dist = model.output.get("distribution", "gaussian")
    if model.model_category in ("Binomial", "Multinomial"):
        dist = "bernoulli" if model.model_category == "Binomial" else "multinomial"
    regress = model.model_category == "Regression"
    if regress and dist not in ("poisson", "gamma", "tweedie") and (model.resp_sd != 1.0 or model.resp_mu != 0.0):
        kv["norm_resp_mul"] = _darr([1.0 / model.resp_sd])
        kv["norm_resp_sub"] = _darr([model.resp_mu])
    else:
        kv["norm_resp_mul"] = "null"
        kv["norm_resp_sub"] = "null"
    kv["use_all_factor_levels"] = "true" if ex.use_all else "false"
    kv["activation"] = act
    kv["distribution"] = dist
    kv["mean_imputation"] = "true"
    if ex.cats:
        kv["cat_modes"] = _arr(ex.cat_modes)
    kv["neural_network_sizes"] = _arr(units)
    for li, lin in enumerate(lins):
        W = lin.weight.detach().double().cpu()
        b = lin.bias.detach().double().cpu()
        if li == 0:
            Wr = torch.zeros(W.shape[0], len(src_cols), dtype=torch.float64)
            for c, s in enumerate(src_cols):
                if s >= 0:
                    Wr[:, c] = W[:, s]
            W = Wr
        if maxout and li < len(lins) - 1:
            H = W.shape[0] // 2
            # ours: rows [0, H) and [H, 2H) are the two maxout pieces; reference: [out][in][k]
            W = torch.stack([W[:H], W[H:]], 2)               # [H, in, 2]
            b = torch.stack([b[:H], b[H:]], 1)               # [H, 2]
        kv[f"weight_layer{li}"] = _darr(W.reshape(-1).tolist())
        kv[f"bias_layer{li}"] = _darr(b.reshape(-1).tolist())
    kv["hidden_dropout_ratios"] = _darr([0.0] * len(lins))
    kv["_genmodel_encoding"] = "AUTO"


def _floats(s):
    s = (s or "").strip()
    if s in ("null", ""):
        return []
    return [float(x) for x in s.strip("[]").split(",") if x.strip()]


def load_deeplearning(ki):
    units = [int(v) for v in _floats(ki["neural_network_sizes"])]
    layers = []
    for li in range(len(units) - 1):
        layers.append((torch.tensor(_floats(ki[f"weight_layer{li}"]), dtype=torch.float64),
                       torch.tensor(_floats(ki[f"bias_layer{li}"]), dtype=torch.float64)))
    return dict(units=units, layers=layers, nums=int(ki["nums"]), cats=int(ki["cats"]),
                cat_offsets=[int(v) for v in _floats(ki.get("cat_offsets"))], norm_mul=_floats(ki.get("norm_mul")),
                norm_sub=_floats(ki.get("norm_sub")), resp_mul=_floats(ki.get("norm_resp_mul")),
                resp_sub=_floats(ki.get("norm_resp_sub")), use_all=ki.get("use_all_factor_levels") == "true",
                act=ki["activation"], dist=ki.get("distribution", "gaussian"),
                drop=_floats(ki.get("hidden_dropout_ratios")))


def _ref_input(st, X):
    """GenModel.setInput: [F, N] (MOJO column order) -> [N, P] one-hot + normalised numerics."""
    N = X.shape[1]
    dev = X.device
    off = st["cat_offsets"]
    ncat = st["cats"]
    P = (off[ncat] if ncat else 0) + st["nums"]
    Z = torch.zeros(N, P, dtype=torch.float64, device=dev)
    for i in range(ncat):
        c = X[i]
        na = torch.isnan(c)
        ci = torch.where(na, torch.zeros_like(c), c).long()
        idx = ci + off[i] if st["use_all"] else ci - 1 + off[i]
        valid = st["use_all"] | (ci != 0)
        idx = torch.where(na | (idx >= off[i + 1]), torch.full_like(idx, off[i + 1] - 1), idx)
        valid = valid | na
        rows = torch.nonzero(valid, as_tuple=True)[0]
        Z[rows, idx[rows]] = 1.0
    base = off[ncat] if ncat else 0
    for k in range(st["nums"]):
        v = X[ncat + k].double()
        if st["norm_mul"]:
            v = (v - st["norm_sub"][k]) * st["norm_mul"][k]
        Z[:, base + k] = torch.nan_to_num(v, nan=0.0)
    return Z


def score_deeplearning(st, X, category):
    a = _ref_input(st, X)
    units, act = st["units"], st["act"]
    nl = len(units) - 1
    for li in range(nl):
        W, b = st["layers"][li]
        W, b = W.to(a.device), b.to(a.device)
        out_n = units[li + 1]
        last = li == nl - 1
        name = act if (not last or category == "AutoEncoder") else ("Softmax" if category in ("Binomial", "Multinomial")
                                                                    else "Linear")
        if name.startswith("Maxout"):
            k = b.numel() // out_n
            h = torch.einsum("ni,oik->nok", a, W.view(out_n, -1, k)) + b.view(out_n, k)
            a = h.max(2).values
        else:
            h = a @ W.view(out_n, -1).T + b
            if name.startswith("Rectifier"):
                a = h.clamp(min=0)
            elif name.startswith("Tanh"):
                a = torch.tanh(h)
            elif name.startswith("ExpRectifier"):
                a = torch.where(h >= 0, h, torch.expm1(h))
            elif name == "Softmax":
                a = torch.softmax(h, 1)
            else:
                a = h
        if "WithDropout" in name and li < len(st["drop"]) and st["drop"][li] > 0:
            a = a * (1.0 - st["drop"][li])
    if category in ("Binomial", "Multinomial"):
        return a.float()
    if category == "AutoEncoder":
        if st["norm_mul"]:
            nn_ = st["nums"]
            mul = torch.tensor(st["norm_mul"], dtype=torch.float64, device=a.device)
            sub = torch.tensor(st["norm_sub"], dtype=torch.float64, device=a.device)
            a[:, -nn_:] = a[:, -nn_:] / mul + sub
        return a.float()
    f = a[:, 0]
    if st["resp_mul"]:
        f = f / st["resp_mul"][0] + st["resp_sub"][0]
    if st["dist"] in ("poisson", "gamma", "tweedie", "multinomial"):
        f = torch.exp(f).clamp(max=1e19)
    elif st["dist"] in ("bernoulli", "quasibinomial", "modified_huber", "ordinal"):
        f = torch.sigmoid(f)
    return f.float()


# ================================================================================================ PCA
def write_pca(model, kv, blobs):
    ex = model.expander
    info = model.info
    start = 0 if ex.use_all else 1
    offs = list(ex.cat_offsets) + [ex.num_off]
    kv["use_all_factor_levels"] = "true" if ex.use_all else "false"
    kv["pca_methods"] = str(model.params.get("pca_method", "GramSVD"))
    kv["pca_impl"] = str(model.params.get("pca_impl", "MTJ_EVD_SYMMMATRIX"))
    V = model.V.double().cpu()
    kv["k"] = V.shape[1]
    kv["permutation"] = _arr(list(ex.cats) + list(ex.nums))
    kv["ncats"] = len(ex.cats)
    kv["nnums"] = len(ex.nums)
    if ex.nums:
        mu = ex.num_mean.cpu().double()
        sd = ex.num_sd.cpu().double()
        if getattr(ex, "descale_only", False):
            sub, mul = torch.zeros_like(mu), 1.0 / sd
        elif ex.standardize:
            sub, mul = mu, 1.0 / sd
        elif ex.center_only:
            sub, mul = mu, torch.ones_like(mu)
        else:
            sub, mul = torch.zeros_like(mu), torch.ones_like(mu)
        kv["normSub"] = _darr(sub.tolist())
        kv["normMul"] = _darr(mul.tolist())
    kv["catOffsets"] = _arr(offs)
    kv["eigenvector_size"] = V.shape[0]
    blobs["eigenvectors_raw"] = V.numpy().astype(">f8").tobytes()
    _ = (info, start)


def load_pca(ki, raw):
    k, n = int(ki["k"]), int(ki["eigenvector_size"])
    V = np.frombuffer(raw, dtype=">f8", count=n * k).reshape(n, k).astype(np.float64)
    return dict(k=k, V=torch.from_numpy(V.copy()), perm=[int(v) for v in _floats(ki["permutation"])],
                ncats=int(ki["ncats"]), nnums=int(ki["nnums"]), offs=[int(v) for v in _floats(ki["catOffsets"])],
                sub=_floats(ki.get("normSub")), mul=_floats(ki.get("normMul")),
                use_all=ki.get("use_all_factor_levels") == "true")


def score_pca(st, X):
    N = X.shape[1]
    V = st["V"].to(X.device)
    out = torch.zeros(N, st["k"], dtype=torch.float64, device=X.device)
    offs = st["offs"]
    for j in range(st["ncats"]):
        c = X[st["perm"][j]]
        ok = ~torch.isnan(c)
        lvl = torch.where(ok, c, torch.zeros_like(c)).long() - (0 if st["use_all"] else 1)
        last = offs[j + 1] - offs[j] - 1
        ok = ok & (lvl >= 0) & (lvl <= last)
        rows = torch.nonzero(ok, as_tuple=True)[0]
        out[rows] += V[offs[j] + lvl[rows]]
    base = offs[st["ncats"]]
    for j in range(st["nnums"]):
        v = (X[st["perm"][st["ncats"] + j]].double() - st["sub"][j]) * st["mul"][j]
        out += v[:, None] * V[base + j][None, :]
    return out.float()


# ================================================================================================ W2V
def write_word2vec(model, kv, blobs):
    V = model.vectors.detach().float().cpu().numpy()
    kv["vocab_size"] = V.shape[0]
    kv["vec_size"] = V.shape[1]
    blobs["vectors"] = V.astype(">f4").tobytes()
    blobs["vocabulary"] = "".join(str(w).replace("\\", "\\\\").replace("\n", "\\n") + "\n" for w in model.words).encode()


def load_word2vec(ki, raw_vectors, vocab_text):
    from .reader import _unescape
    n, d = int(ki["vocab_size"]), int(ki["vec_size"])
    V = np.frombuffer(raw_vectors, dtype=">f4", count=n * d).reshape(n, d).astype(np.float32)
    words = [_unescape(w) for w in vocab_text.split("\n")[:n]]
    return words, torch.from_numpy(V.copy())


# ================================================================================================ isotonic
def _blob_doubles(v) -> bytes:
    v = np.asarray(v, dtype=np.float64)
    return struct.pack(">i", v.size) + v.astype(">f8").tobytes()


def _read_blob_doubles(b: bytes):
    (n,) = struct.unpack(">i", b[:4])
    return np.frombuffer(b[4:4 + 8 * n], dtype=">f8").astype(np.float64)


def write_isotonic(model, kv, blobs):
    tx, ty = list(model.thresholds_x), list(model.thresholds_y)
    kv["calib_min_x"] = repr(float(tx[0]))
    kv["calib_max_x"] = repr(float(tx[-1]))
    blobs["calib/thresholds_x"] = _blob_doubles(tx)
    blobs["calib/thresholds_y"] = _blob_doubles(ty)


def load_isotonic(files):
    return _read_blob_doubles(files["calib/thresholds_x"]), _read_blob_doubles(files["calib/thresholds_y"])


# ================================================================================================ EIF
def write_eif(model, kv, blobs):
    """``trees/tNN.bin`` (ExtendedIsolationForestMojoModel.scoreTree0, native byte order): int F, then
    per node int number (heap numbering: children 2i+1 / 2i+2), byte 'N' + F doubles normal + F doubles
    point, or byte 'L' + int row count. The point is the hyperplane's closest point to the origin."""
    from ..models.isoforest import c_factor
    kv["ntrees"] = len(model.trees)
    kv["sample_size"] = int(model.output["sample_size"])
    for t, tr in enumerate(model.trees):
        nrm, off = np.asarray(tr["normal"], dtype=np.float64), np.asarray(tr["offset"], dtype=np.float64)
        left, right = np.asarray(tr["left"]), np.asarray(tr["right"])
        F = nrm.shape[1]
        nrows = tr.get("nrows")
        out = [struct.pack("<i", F)]
        stack = [(0, 0, 0)]                        # (node, heap number, depth)
        recs = []
        while stack:
            i, h, dep = stack.pop()
            if left[i] < 0:
                if nrows is not None:
                    n = int(nrows[i])
                else:                              # older models: invert value = depth + c(n)
                    want = float(tr["value"][i]) - dep
                    n = min(range(0, int(model.output["sample_size"]) + 1), key=lambda k: abs(float(c_factor(k)) - want))
                recs.append((h, struct.pack("<ib", h, ord("L")) + struct.pack("<i", n)))
                continue
            nn = float(nrm[i] @ nrm[i])
            pt = nrm[i] * (off[i] / nn) if nn > 0 else np.zeros(F)
            recs.append((h, struct.pack("<ib", h, ord("N")) + nrm[i].astype("<f8").tobytes() + pt.astype("<f8").tobytes()))
            stack.append((int(right[i]), 2 * h + 2, dep + 1))
            stack.append((int(left[i]), 2 * h + 1, dep + 1))
        recs.sort(key=lambda r: r[0])
        blobs[f"trees/t{t:02d}.bin"] = b"".join(out + [r[1] for r in recs])


def load_eif(ki, files):
    """Decode every tree into flat arrays (normal, point, left, right, leaf rows) for batched scoring."""
    trees = []
    for t in range(int(ki["ntrees"])):
        b = files[f"trees/t{t:02d}.bin"]
        (F,) = struct.unpack_from("<i", b, 0)
        pos = 4
        nodes = {}
        while pos + 5 <= len(b):
            h, typ = struct.unpack_from("<ib", b, pos)
            if typ not in (ord("N"), ord("L")):
                break                      # zero padding after the last node (fixed-size byte blocks)
            pos += 5
            if typ == ord("N"):
                n = np.frombuffer(b, "<f8", F, pos); p = np.frombuffer(b, "<f8", F, pos + 8 * F)
                nodes[h] = ("N", n, p)
                pos += 16 * F
            else:
                (rows,) = struct.unpack_from("<i", b, pos)
                nodes[h] = ("L", rows)
                pos += 4
        order = sorted(nodes)
        idx = {h: k for k, h in enumerate(order)}
        M = len(order)
        nrm, pt = np.zeros((M, F)), np.zeros((M, F))
        left, right, rows = -np.ones(M, np.int64), -np.ones(M, np.int64), np.zeros(M, np.int64)
        for h in order:
            k = idx[h]
            if nodes[h][0] == "N":
                nrm[k], pt[k] = nodes[h][1], nodes[h][2]
                left[k], right[k] = idx[2 * h + 1], idx[2 * h + 2]
            else:
                rows[k] = nodes[h][1]
        trees.append(dict(normal=torch.from_numpy(nrm), point=torch.from_numpy(pt), left=torch.from_numpy(left),
                          right=torch.from_numpy(right), rows=torch.from_numpy(rows)))
    return dict(trees=trees, sample_size=int(ki["sample_size"]))


def score_eif(st, X):
    from ..models.isoforest import c_factor
    Xr = X.T.double()
    N = Xr.shape[0]
    dev = Xr.device
    tot = torch.zeros(N, dtype=torch.float64, device=dev)
    for tr in st["trees"]:
        nrm, pt = tr["normal"].to(dev), tr["point"].to(dev)
        left, right, rows = tr["left"].to(dev), tr["right"].to(dev), tr["rows"].to(dev)
        proj = Xr @ nrm.T - (nrm * pt).sum(1)            # (row - p) . n per node
        node = torch.zeros(N, dtype=torch.long, device=dev)
        height = torch.zeros(N, dtype=torch.float64, device=dev)
        for _ in range(64):
            isleaf = left[node] < 0
            if bool(isleaf.all()):
                break
            go_left = proj.gather(1, node[:, None]).squeeze(1) <= 0     # NaN -> right, as in scoreTree0
            node = torch.where(isleaf, node, torch.where(go_left, left[node], right[node]))
            height = height + (~isleaf).double()
        cf = torch.tensor([float(c_factor(int(r))) for r in tr["rows"].tolist()], dtype=torch.float64, device=dev)
        tot += height + cf[node]
    h = tot / max(1, len(st["trees"]))
    c = float(c_factor(st["sample_size"]))
    return torch.stack([torch.pow(2.0, -h / c).float(), h.float()], 1)


# ================================================================================================ CoxPH
def _blob_rect(rows) -> bytes:
    """ModelMojoWriter.writeRectangularDoubleArray payload: row-major big-endian doubles, no header."""
    return np.asarray(rows, dtype=">f8").tobytes()


def coxph_columns(model):
    """CoxPHMojoModel row layout (CoxPHMojoModel.featureValue: strata columns first, then the DataInfo
    categoricals and numerics); the start/stop columns follow and are not read by the scorer."""
    info, keep, ex = model.info, model.keep, model.expander
    order = list(model.strata_idx) + [keep[j] for j in ex.cats] + [keep[j] for j in ex.nums] + list(model.special_idx)
    cols = [info.x[j] for j in order] + ([info.response] if info.response else [])
    doms = [info.domains[j] for j in order] + ([info.response_domain] if info.response else [])
    return cols, doms


def write_coxph(model, kv, blobs):
    """CoxPHMojoWriter.writeModelData layout (h2o-algos/src/main/java/hex/coxph/CoxPHMojoWriter.java):
    coef, cats / cat_offsets / use_all_factor_levels, num_numerical_columns / num_offsets, x_mean_cat /
    x_mean_num per stratum (lp base = x_mean . coef) and strata_count / strata_i."""
    ex = model.expander
    beta = [float(b) for b in model.beta.cpu().tolist()]
    zm = model.output.get("z_mean")
    if zm is None:
        raise ValueError("CoxPH model has no design means (retrain to export a MOJO)")
    strata = [list(map(float, s)) for s in getattr(model, "strata_values", [])]
    S = max(1, len(strata))
    nc = ex.num_off
    kv["coef"] = _arr(beta)
    kv["cats"] = len(ex.cats)
    kv["cat_offsets"] = _arr(list(ex.cat_offsets) + [nc])
    kv["use_all_factor_levels"] = "true" if ex.use_all else "false"
    kv["num_numerical_columns"] = len(ex.nums)
    kv["num_offsets"] = _arr([nc + i for i in range(len(ex.nums))])
    zs = model.output.get("z_mean_strata") if strata else None
    rows = zs if zs is not None else [zm] * S      # one design-mean row per stratum, strata_i order
    for t, sl in (("x_mean_cat", slice(0, nc)), ("x_mean_num", slice(nc, None))):
        kv[f"{t}_size1"] = S
        kv[f"{t}_size2"] = len(zm[sl])
        blobs[t] = _blob_rect([r[sl] for r in rows])
    kv["strata_count"] = len(strata)
    for i, s in enumerate(strata):
        kv[f"strata_{i}"] = _arr(s)
    kv["n_features"] = len(model.info.x)


def load_coxph(ki, files):
    from .reader import _floats
    coef = np.asarray(_floats(ki["coef"]), dtype=np.float64)
    ns = int(ki.get("strata_count", 0))
    strata = [np.asarray(_floats(ki[f"strata_{i}"])) for i in range(ns)]

    def rect(t):
        a, b = int(ki[f"{t}_size1"]), int(ki[f"{t}_size2"])
        return np.frombuffer(files.get(t, b""), dtype=">f8", count=a * b).astype(np.float64).reshape(a, b)
    xc, xn = rect("x_mean_cat"), rect("x_mean_num")
    nstart = xc.shape[1] if xc.shape[0] >= 1 else 0
    lp_base = xc @ coef[:xc.shape[1]] + xn @ coef[nstart:nstart + xn.shape[1]]   # CoxPHMojoModel.computeLpBase
    return dict(coef=coef, cats=int(ki["cats"]), cat_offsets=[int(v) for v in _floats(ki["cat_offsets"])],
                use_all=ki.get("use_all_factor_levels") == "true", nums=int(ki["num_numerical_columns"]),
                num_offsets=[int(v) for v in _floats(ki["num_offsets"])], strata=strata,
                strata_len=len(strata[0]) if strata else 0, lp_base=lp_base)


def score_coxph(st, X):
    """CoxPHMojoModel.score0 on a [F, N] frame: categorical coefficients + numeric terms - lp base of the
    row's stratum (rows of an unseen stratum score NaN)."""
    X = X.double()
    S, coef = st["strata_len"], torch.tensor(st["coef"], dtype=torch.float64, device=X.device)
    N = X.shape[1]
    lp = torch.zeros(N, dtype=torch.float64, device=X.device)
    lo = 0 if st["use_all"] else 1
    co = st["cat_offsets"]
    for c in range(st["cats"]):
        v = X[S + c]
        lvl = torch.nan_to_num(v, nan=-1).long() - lo
        x = lvl + co[c]
        ok = (lvl >= 0) & (x < co[c + 1])
        lp = lp + torch.where(ok, coef[x.clamp(0, coef.numel() - 1)], torch.zeros_like(lp))
        lp = torch.where(torch.isnan(v), torch.full_like(lp, float("nan")), lp)
    for i in range(st["nums"]):
        if st["num_offsets"][i] >= coef.numel():
            break
        lp = lp + coef[st["num_offsets"][i]] * X[S + st["cats"] + i]
    if not st["strata"]:
        return (lp - float(st["lp_base"][0])).float()
    base = torch.full_like(lp, float("nan"))
    for k, s in enumerate(st["strata"]):
        m = torch.ones(N, dtype=torch.bool, device=X.device)
        for j, v in enumerate(s):
            m &= torch.nan_to_num(X[j], nan=-1).long() == int(v)
        base = torch.where(m, torch.full_like(base, float(st["lp_base"][k])), base)
    return (lp - base).float()


# ================================================================================================ TargetEncoder
TE_DIR = "feature_engineering/target_encoding/"


def write_targetencoder(model, kv, blobs):
    """TargetEncoderMojoWriter layout (h2o-extensions/target-encoder/.../TargetEncoderMojoWriter.java):
    blending parameters in model.ini, ``encoding_map.ini`` ([column] sections of ``level = numerator
    denominator [targetclass]``), the NA-presence map and the input->encoding / input->output column maps.
    NA levels are not encoded here (they take the prior), so every column is written with has_NAs = 0."""
    p, info = model.params, model.info
    kv["keep_original_categorical_columns"] = "true" if p.get("keep_original_categorical_columns", True) else "false"
    kv["with_blending"] = "true" if p.get("blending") else "false"
    if p.get("blending"):
        kv["inflection_point"] = repr(float(p["inflection_point"]))
        kv["smoothing"] = repr(float(p["smoothing"]))
    nonp = [c for c in (info.weights, info.offset, info.fold or p.get("fold_column"), info.response) if c]
    kv["non_predictors"] = ";".join(nonp)
    multi = model.K > 1
    enc, nas, inenc, inout = [], [], [], []
    for name in model.output["encoded_columns"]:
        st = model.stats[name]
        num = np.asarray(st["num"].cpu() if torch.is_tensor(st["num"]) else st["num"], dtype=np.float64)
        den = np.asarray(st["den"].cpu() if torch.is_tensor(st["den"]) else st["den"], dtype=np.float64)
        num = num.reshape(den.shape[0], -1)
        enc.append(f"[{name}]")
        for lvl in range(den.shape[0]):
            if den[lvl] <= 0:
                continue
            if multi:
                for k in range(num.shape[1]):
                    enc.append(f"{lvl} = {float(num[lvl, k])!r} {float(den[lvl])!r} {k + 1}")
            else:
                enc.append(f"{lvl} = {float(num[lvl, 0])!r} {float(den[lvl])!r}")
        nas.append(f"{name} = 0")
        inenc += ["[from]", name, "[to]", name]
        outs = ([f"{name}_{info.response_domain[k + 1]}_te" for k in range(model.K)] if multi else [f"{name}_te"])
        inout += ["[from]", name, "[to]"] + outs
    for fn, lines in (("encoding_map.ini", enc), ("te_column_name_to_missing_values_presence.ini", nas),
                      ("input_encoding_columns_map.ini", inenc), ("input_output_columns_map.ini", inout)):
        blobs[TE_DIR + fn] = "".join(s + "\n" for s in lines)


def load_targetencoder(ki, files, info):
    """Encoding maps -> TargetEncoderModel statistics (prior = Σnumerator / Σdenominator over the map, as
    TargetEncoderMojoModel computes it)."""
    from ..models.targetencoder import TargetEncoderModel
    raw = files[TE_DIR + "encoding_map.ini"]
    text = raw.decode() if isinstance(raw, bytes) else raw
    ncls = int(ki.get("n_classes", 1))
    Kp = ncls - 1 if ncls > 2 else 1
    maps, cur = {}, None
    for line in text.splitlines():
        s = line.strip()
        if not s:
            continue
        if s.startswith("[") and s.endswith("]"):
            cur = maps.setdefault(s[1:-1], {})
            continue
        lvl, _, comp = s.partition("=")
        parts = comp.split()
        cls = int(parts[2]) - 1 if len(parts) > 2 else 0
        e = cur.setdefault(int(lvl), [np.zeros(Kp), 0.0])
        e[0][cls] = float(parts[0])
        e[1] = float(parts[1])
    params = dict(blending=ki.get("with_blending") == "true", inflection_point=float(ki.get("inflection_point", 10)),
                  smoothing=float(ki.get("smoothing", 20)),
                  keep_original_categorical_columns=ki.get("keep_original_categorical_columns", "false") == "true",
                  noise=0.0, data_leakage_handling="none")
    m = TargetEncoderModel(None, params, info)
    m.device = torch.device("cpu")
    m.K = Kp
    m.stats = {}
    for name, mp in maps.items():
        j = info.x.index(name) if name in info.x else None
        dom = list(info.domains[j]) if j is not None and info.domains[j] is not None else []
        L = max(len(dom), (max(mp) + 1) if mp else 0)
        num, den = np.zeros((L, Kp)), np.zeros(L)
        for lvl, (nv, dv) in mp.items():
            num[lvl], den[lvl] = nv, dv
        prior = num.sum(0) / max(den.sum(), 1e-300)
        m.stats[name] = dict(num=num, den=den, prior=prior, domain=dom)
    m.output["encoded_columns"] = list(maps)
    return m


# ------------------------------------------------------------------------------------------------ GLRM
def load_glrm(ki, files):
    """GlrmMojoReader layout: ``archetypes`` (nrowY x ncolY big-endian doubles, Y over the expanded
    columns: categorical one-hot blocks at ``catOffsets``, then numerics), ``losses`` (one per
    permuted column), ``cols_permutation`` (cats first), ``num_levels_per_category``,
    ``norm_sub`` / ``norm_mul`` (numeric standardisation)."""
    nrow, ncol = int(ki["nrowY"]), int(ki["ncolY"])
    Y = np.frombuffer(files["archetypes"], ">f8", nrow * ncol).reshape(nrow, ncol).astype(np.float64)
    losses = [ln.strip() for ln in files["losses"].decode().splitlines() if ln.strip()]
    ints = lambda k: [int(float(v)) for v in _floats(ki[k])] if ki.get(k) not in (None, "null") else None  # noqa: E731
    return dict(Y=torch.from_numpy(Y.copy()), losses=losses, perm=ints("cols_permutation"),
                nlev=ints("num_levels_per_category"), cat_off=ints("catOffsets"), ncats=int(ki["num_categories"]),
                nnums=int(ki["num_numeric"]), norm_sub=_floats(ki.get("norm_sub", "[]")),
                norm_mul=_floats(ki.get("norm_mul", "[]")), ncolX=int(ki["ncolX"]),
                gammax=float(ki.get("gammaX", 0.0)), regx=ki.get("regularizationX", "None"))


def glrm_row_data(st, X):
    """GlrmMojoModel.getRowData: permuted columns, unseen categorical levels -> NaN. X: [F, N]."""
    A = X.T.double()[:, st["perm"]].clone()
    for i in range(st["ncats"]):
        A[:, i] = torch.where(A[:, i] >= st["nlev"][i], torch.full_like(A[:, i], float("nan")), A[:, i])
    return A


def score_glrm(st, X, iters=200):
    """X factors of each row for the fixed archetypes: minimise the per-column GLRM losses (one-vs-all
    hinge for categoricals, quadratic for numerics, NAs skipped) + gammaX * regularizer by projected
    gradient from x = 0 (the reference starts from a seeded Gaussian; the optimum is what we return)."""
    from ..models.glrm import _prox
    A = glrm_row_data(st, X)
    N = A.shape[0]
    Y = st["Y"].to(A.device)
    k = Y.shape[0]
    nc, off = st["ncats"], st["cat_off"] or [0]
    sub = torch.tensor(st["norm_sub"] or [0.0] * st["nnums"], dtype=torch.float64, device=A.device)
    mul = torch.tensor(st["norm_mul"] or [1.0] * st["nnums"], dtype=torch.float64, device=A.device)
    nums = (A[:, nc:] - sub) * mul
    ncat_cols = off[-1] if nc else 0
    x = torch.zeros(N, k, dtype=torch.float64, device=A.device, requires_grad=True)
    opt = torch.optim.LBFGS([x], lr=1.0, max_iter=iters, line_search_fn="strong_wolfe")

    def obj():
        opt.zero_grad()
        U = x @ Y
        L = x.new_zeros(())
        for i in range(nc):
            u = U[:, off[i]:off[i + 1]]
            a = A[:, i]
            ok = ~torch.isnan(a)
            if ok.any():
                ai = a[ok].long()
                uu = u[ok]
                hinge = torch.clamp(1 + uu, min=0).sum(1)
                ua = uu.gather(1, ai[:, None])[:, 0]
                L = L + (hinge + torch.clamp(1 - ua, min=0) - torch.clamp(1 + ua, min=0)).sum()
        un = U[:, ncat_cols:ncat_cols + st["nnums"]]
        okn = ~torch.isnan(nums)
        L = L + torch.where(okn, (un - torch.nan_to_num(nums)) ** 2, torch.zeros_like(un)).sum()
        if st["gammax"] > 0 and str(st["regx"]).lower() == "quadratic":
            L = L + st["gammax"] * (x * x).sum()
        L.backward()
        return L
    opt.step(obj)
    xd = x.detach()
    if str(st["regx"]).lower() not in ("none", "quadratic"):
        xd = _prox(st["regx"], xd, 0.0, 1)
    return xd.float()


_GLRM_LOSS = {"quadratic": "Quadratic", "absolute": "Absolute", "huber": "Huber", "poisson": "Poisson",
              "hinge": "Hinge", "logistic": "Logistic", "periodic": "Periodic", "categorical": "Categorical",
              "ordinal": "Ordinal"}
_GLRM_REG = {"none": "None", "quadratic": "Quadratic", "l2": "L2", "l1": "L1", "nonnegative": "NonNegative",
             "onesparse": "OneSparse", "unitonesparse": "UnitOneSparse", "simplex": "Simplex"}


def write_glrm(model, kv, blobs):
    """GlrmMojoWriter layout: the archetypes over the expanded columns (categorical one-hot blocks,
    then numerics), per-column losses, the cats-first column permutation and the numeric
    standardisation, so ``GlrmMojoModel`` (and this package's reader) can solve each row's X."""
    canon = lambda s: str(s).lower().replace("_", "")  # noqa: E731
    p = model.params
    ex = model.expander
    Y = model.Y.double().cpu().numpy()
    k, P = Y.shape
    perm = list(ex.cats) + list(ex.nums)
    nlev = [len(model.info.domains[j] or []) for j in ex.cats]
    offs = [0]
    for n in nlev:
        offs.append(offs[-1] + n)
    nn = len(ex.nums)
    if ex.nums and ex.standardize:
        sub = ex.num_mean.double().cpu().tolist()
        mul = (1.0 / ex.num_sd.double().clamp(min=1e-300)).cpu().tolist()
    elif ex.nums and getattr(ex, "center_only", False):
        sub, mul = ex.num_mean.double().cpu().tolist(), [1.0] * nn
    else:
        sub, mul = [0.0] * nn, [1.0] * nn
    kv["initialization"] = {"plusplus": "PlusPlus", "svd": "SVD", "random": "Random", "user": "User"}.get(
        canon(p.get("init", "PlusPlus")), "PlusPlus")
    kv["regularizationX"] = _GLRM_REG.get(canon(p.get("regularization_x", "None")), "None")
    kv["regularizationY"] = _GLRM_REG.get(canon(p.get("regularization_y", "None")), "None")
    kv["gammaX"] = float(p.get("gamma_x") or 0.0)
    kv["gammaY"] = float(p.get("gamma_y") or 0.0)
    kv["ncolX"] = k
    kv["seed"] = int(p.get("seed") if p.get("seed") not in (None, -1) else 0)
    kv["reverse_transform"] = "true" if p.get("impute_original") else "false"
    kv["cols_permutation"] = "[" + ", ".join(str(int(v)) for v in perm) + "]"
    kv["num_categories"] = len(ex.cats)
    kv["num_numeric"] = nn
    kv["norm_sub"] = "[" + ", ".join(repr(float(v)) for v in sub) + "]"
    kv["norm_mul"] = "[" + ", ".join(repr(float(v)) for v in mul) + "]"
    kv["transposed"] = "false"
    num_loss = _GLRM_LOSS.get(canon(p.get("loss", "Quadratic")), "Quadratic")
    cat_loss = _GLRM_LOSS.get(canon(p.get("multi_loss", "Categorical")), "Categorical")
    kv["ncolA"] = len(perm)
    blobs["losses"] = "".join((cat_loss if i < len(ex.cats) else num_loss) + "\n" for i in range(len(perm)))
    kv["ncolY"] = P
    kv["nrowY"] = k
    kv["num_levels_per_category"] = "[" + ", ".join(str(n) for n in nlev + [-1] * nn) + "]"
    kv["catOffsets"] = "[" + ", ".join(str(o) for o in offs) + "]"
    blobs["archetypes"] = Y.astype(">f8").tobytes()


# ---- RuleFit (RuleFitMojoWriter: MultiModelMojoWriter with the GLM as the one sub-model) ----------------
def _jbool(b) -> str:
    return "true" if b else "false"


def write_rulefit(model, kv, blobs):
    from .writer import _mojo_files
    glm = model.glm
    key = glm.key
    kv["submodel_count"] = 1
    kv["submodel_key_0"] = key
    kv["submodel_dir_0"] = f"models/{key}/"
    blobs.update(_mojo_files(glm, f"models/{key}/"))
    kv["linear_model"] = key
    mtype = str(model.params.get("model_type", "rules_and_linear")).lower()
    classes = model.info.response_domain
    nclasses = len(classes) if classes is not None and len(classes) > 2 else 1
    if mtype != "linear":
        groups = dict(model.rule_groups)
        for i in range(model.depth):
            for j in range(model.ntrees):
                rules = []
                for k in range(nclasses):          # class 0 ... class k, as writeOrderedRuleEnsemble
                    rules += groups.get(f"M{i}T{j}C{k}" if nclasses > 1 else f"M{i}T{j}", [])
                kv[f"num_rules_M{i}T{j}"] = len(rules)
                for r_i, r in enumerate(rules):
                    rid = f"{i}_{j}_{r_i}"
                    kv[f"num_conditions_rule_id_{rid}"] = len(r.conds)
                    for c_i, c in enumerate(r.conds):
                        cid = f"{c_i}_{rid}"
                        kv[f"feature_index_{cid}"] = c.feat
                        if c.ctype == "cat":
                            kv[f"type_{cid}"] = 0
                            kv[f"language_cat_treshold_length_{cid}"] = len(c.level_names)
                            for t, nm in enumerate(c.level_names):
                                kv[f"language_cat_treshold_{t}_{cid}"] = nm
                            kv[f"cat_treshold_length_{cid}"] = len(c.levels)
                            for t, lv in enumerate(c.levels):
                                kv[f"cat_treshold_length_{t}_{cid}"] = int(lv)
                        else:
                            kv[f"type_{cid}"] = 1
                            kv[f"num_treshold{cid}"] = repr(float(c.thr))
                        kv[f"operator_{cid}"] = {"<": 0, ">=": 1}.get(c.op, 2)
                        kv[f"feature_name_{cid}"] = c.name
                        kv[f"nas_included_{cid}"] = _jbool(c.nas)
                        kv[f"language_condition{cid}"] = c.text()
                    kv[f"prediction_value_rule_id_{rid}"] = repr(float(r.pred))
                    kv[f"language_rule_rule_id_{rid}"] = r.text()
                    kv[f"coefficient_rule_id_{rid}"] = repr(float(r.coef))
                    kv[f"var_name_rule_id_{rid}"] = r.var
                    kv[f"support_rule_id_{rid}"] = repr(float(r.support))
    kv["model_type"] = {"linear": 0, "rules_and_linear": 1}.get(mtype, 2)
    kv["type"] = key
    kv["depth"] = model.depth
    kv["ntrees"] = model.ntrees
    codes = model.output["linear_names"]
    kv["data_from_rules_codes_len"] = len(codes)
    for i, n in enumerate(codes):
        kv[f"data_from_rules_codes_{i}"] = n
    if model.info.weights:
        kv["weights_column"] = model.info.weights
    kv["linear_names_len"] = len(codes)
    for i, n in enumerate(codes):
        kv[f"linear_names_{i}"] = n


def load_rulefit(ki):
    """RuleFitMojoReader: rule ensemble [depth][ntrees][rules] + model type + linear names."""
    from ..models.rulefit import Condition, Rule
    mtype = int(ki["model_type"])
    depth, ntrees = int(ki["depth"]), int(ki["ntrees"])
    ordered = []
    if mtype != 0:
        for i in range(depth):
            row = []
            for j in range(ntrees):
                rules = []
                for r_i in range(int(ki[f"num_rules_M{i}T{j}"])):
                    rid = f"{i}_{j}_{r_i}"
                    conds = []
                    for c_i in range(int(ki[f"num_conditions_rule_id_{rid}"])):
                        cid = f"{c_i}_{rid}"
                        op = {0: "<", 1: ">="}.get(int(ki[f"operator_{cid}"]), "in")
                        nas = ki[f"nas_included_{cid}"] == "true"
                        name = ki[f"feature_name_{cid}"]
                        if int(ki[f"type_{cid}"]) == 0:
                            n1 = int(ki[f"language_cat_treshold_length_{cid}"])
                            n2 = int(ki[f"cat_treshold_length_{cid}"])
                            conds.append(Condition(int(ki[f"feature_index_{cid}"]), name, "cat", op, -1.0,
                                                   [int(ki[f"cat_treshold_length_{t}_{cid}"]) for t in range(n2)],
                                                   [ki[f"language_cat_treshold_{t}_{cid}"] for t in range(n1)], nas))
                        else:
                            conds.append(Condition(int(ki[f"feature_index_{cid}"]), name, "num", op,
                                                   float(ki[f"num_treshold{cid}"]), nas=nas))
                    sup = ki.get(f"support_rule_id_{rid}")
                    rules.append(Rule(conds, float(ki[f"prediction_value_rule_id_{rid}"]), ki[f"var_name_rule_id_{rid}"],
                                      float(ki[f"coefficient_rule_id_{rid}"]), float(sup) if sup else float("nan")))
                row.append(rules)
            ordered.append(row)
    n = int(ki["linear_names_len"])
    return dict(model_type=mtype, depth=depth, ntrees=ntrees, rules=ordered,
                linear_names=[ki[f"linear_names_{i}"] for i in range(n)], linear_key=ki["linear_model"])


def score_rulefit(st, glm, X, parent_info):
    """RuleFitMojoModel.score0: rule codes per (depth, tree[, class]) decoded to the GLM's level index,
    then (rules_and_linear) the raw row, mapped into the GLM's column order by linear_names."""
    import torch
    classes = parent_info.response_domain
    multi = classes is not None and len(classes) > 2
    test = []
    if st["model_type"] != 0:
        gnames = list(glm.info.x)
        for i in range(st["depth"]):
            for j in range(st["ntrees"]):
                rules = st["rules"][i][j]
                per = [[r for r in rules if r.var.endswith(c)] for c in classes] if multi else [rules]
                for k, rl in enumerate(per):
                    col = f"M{i}T{j}" + (f"C{k}" if multi else "")
                    dom = glm.info.domains[gnames.index(col)] or []
                    code = torch.full((X.shape[1],), float("nan"), dtype=torch.float32, device=X.device)
                    for r in rl:
                        if r.var in dom:
                            code = torch.where(r.holds(X), torch.full_like(code, float(dom.index(r.var))), code)
                    test.append(code)
    if st["model_type"] != 2:
        test += [X[f].float() for f in range(X.shape[0])]
    gx = list(glm.info.x)
    rows = [None] * len(gx)
    for i, n in enumerate(st["linear_names"][:len(gx)]):
        rows[gx.index(n)] = test[i]
    return glm._predict_tensor(torch.stack(rows, 0))


# ================================================================================================ GAM
# GAMMojoWriter layout (h2o-algos/src/main/java/hex/gam/GAMMojoWriter.java:writeModelData) read by
# h2o-genmodel GamMojoReader / GamMojoModelBase: the GLM part (cats, cat_offsets, numsCenter, NA fills,
# family / link, beta_center over [categorical one-hot, linear numerics, centred gam columns, intercept] on
# the raw scale) and per smoother, in the reader's SORTED order (cubic regression, I-spline, M-spline):
# knots [gam][1][k], the cubic F rows B^-1 D (``_binvD`` [k-2][k]), the centring transposes
# (``zTranspose`` [k-1][k]; I-splines are not centred), the un-centred beta and the column names.
# Thin-plate smoothers (bs = 1) are refused: their MOJO carries H2O's own polynomial / distance basis.
_BS_ORDER = {0: 0, 2: 1, 3: 2}


def _gam_blocks(model):
    """Smoother blocks of a GAM in reader order: (user index, state, centred names, uncentred names)."""
    if any(g["bs"] == 1 for g in model.gams):
        raise ValueError("GAM MOJO: thin-plate smoothers (bs=1) are not exportable in the reference layout")
    names = list(model.glm.info.x)
    lin = list(model.lin_x)
    off = len(lin)
    blocks = []
    for gi, g in enumerate(model.gams):
        nb = int(g["nb"])
        cn = names[off:off + nb]
        off += nb
        tag = "_".join(g["cols"])
        unc = nb + (1 if g.get("Z") is not None else 0)
        suffix = {0: "cr", 2: "is", 3: "ms"}[g["bs"]]
        blocks.append((gi, g, cn, [f"{tag}_{suffix}_nc_{i}" for i in range(unc)]))
    blocks.sort(key=lambda b: (_BS_ORDER[b[1]["bs"]], b[0]))
    return blocks


def _blob_3d(arrs) -> bytes:
    return b"".join(np.asarray(a, dtype=">f8").tobytes() for a in arrs)


def write_gam(model, kv, blobs):
    glm = model.glm
    ex = glm.expander
    fam = glm.output["family"]
    if fam in ("multinomial", "ordinal"):
        raise ValueError("GAM MOJO: multinomial / ordinal GAMs are not exported")
    blocks = _gam_blocks(model)
    n_lin_num = sum(1 for j in ex.nums if glm.info.x[j] in model.lin_x)
    kv["use_all_factor_levels"] = "true" if ex.use_all else "false"
    kv["cats"] = len(ex.cats)
    kv["cat_offsets"] = _arr(list(ex.cat_offsets) + [ex.num_off])
    kv["numsCenter"] = n_lin_num
    kv["num"] = n_lin_num + len(blocks)
    kv["mean_imputation"] = "true"
    kv["numNAFillsCenter"] = _arr([float(v) for v in ex.num_mean.cpu().tolist()[:n_lin_num]])
    kv["catNAFills"] = _arr([int(v) for v in ex.cat_modes])
    kv["family"] = "bernoulli" if fam == "binomial" else fam
    kv["link"] = glm.output["link"]
    if fam == "tweedie":
        kv["tweedie_link_power"] = float(glm.params.get("tweedie_link_power", 1.0))
    gam_cols = [g["cols"] for g in model.gams]
    kv["num_knots"] = _arr([len(g["knots"]) for g in model.gams])
    kv["num_knots_sorted"] = _arr([len(b[1]["knots"]) for b in blocks])
    blobs["gam_columns"] = "".join(c + "\n" for cs in gam_cols for c in cs)
    blobs["gam_columns_sorted"] = "".join(c + "\n" for b in blocks for c in b[1]["cols"])
    kv["gam_column_dim"] = _arr([len(cs) for cs in gam_cols])
    kv["gam_column_dim_sorted"] = _arr([len(b[1]["cols"]) for b in blocks])
    # raw-scale coefficients: [cat one-hot | linear numerics | gam blocks (user order) | intercept]
    braw, ic = ex.destandardize(glm.beta[0, :-1], float(glm.beta[0, -1]))
    braw = braw.double().cpu().numpy()
    head = braw[: ex.num_off + n_lin_num]
    gam_beta, pos = {}, ex.num_off + n_lin_num
    for gi, g in enumerate(model.gams):
        gam_beta[gi] = braw[pos:pos + int(g["nb"])]
        pos += int(g["nb"])
    center, nocenter, cnames, ncnames = list(head), list(head), [], []
    for gi, g, cn, ncn in blocks:
        bc = gam_beta[gi]
        center += bc.tolist()
        Z = np.asarray(g["Z"]) if g.get("Z") is not None else None
        nocenter += (Z @ bc).tolist() if Z is not None else bc.tolist()
        cnames.append(cn)
        ncnames.append(ncn)
    center.append(ic)
    nocenter.append(ic)
    kv["num_expanded_gam_columns"] = sum(len(n) for n in ncnames)
    kv["num_expanded_gam_columns_center"] = sum(len(n) for n in cnames)
    normal = [glm.info.x[j] for j in list(ex.cats) + [j for j in ex.nums if glm.info.x[j] in model.lin_x]]
    nc_all = normal + [n for ns in ncnames for n in ns]
    blobs["_names_no_centering"] = "".join(n + "\n" for n in nc_all)
    kv["total feature size"] = len(nc_all)
    kv["gamColName_dim"] = _arr([len(n) for n in ncnames])
    blobs["gamColNamesCenter"] = "".join(n + "\n" for ns in cnames for n in ns)
    blobs["gamColNames"] = "".join(n + "\n" for ns in ncnames for n in ns)
    kv["beta"] = _arr([float(v) for v in nocenter])
    kv["beta length per class"] = len(nocenter)
    kv["beta_center"] = _arr([float(v) for v in center])
    kv["beta center length per class"] = len(center)
    kv["bs"] = _arr([int(g["bs"]) for g in model.gams])
    kv["bs_sorted"] = _arr([int(b[1]["bs"]) for b in blocks])
    blobs["knots"] = _blob_3d([[b[1]["knots"]] for b in blocks])
    blobs["zTranspose"] = _blob_3d([np.asarray(b[1]["Z"]).T if b[1].get("Z") is not None else np.zeros((0, 0))
                                    for b in blocks])
    kv["_d"] = _arr([1] * len(blocks))
    kv["num_CS_col"] = sum(1 for b in blocks if b[1]["bs"] == 0)
    kv["num_IS_col"] = sum(1 for b in blocks if b[1]["bs"] == 2)
    kv["num_MS_col"] = sum(1 for b in blocks if b[1]["bs"] == 3)
    if kv["num_IS_col"] or kv["num_MS_col"]:
        kv["spline_orders_sorted"] = _arr([int(b[1].get("order", 0)) for b in blocks])
        kv["spline_orders"] = _arr([int(g.get("order", 0)) for g in model.gams])
    kv["num_TP_col"] = 0
    if kv["num_CS_col"]:
        blobs["_binvD"] = _blob_3d([np.asarray(b[1]["F"])[1:-1] for b in blocks if b[1]["bs"] == 0])
    # this framework imputes a missing smoother input with its training mean before the basis expansion
    kv["gam_na_fill_sorted"] = _arr([float(b[1]["means"][0]) for b in blocks])
    gi = glm.info
    order = list(ex.cats) + [j for j in ex.nums if gi.x[j] in model.lin_x]     # DataInfo order: cats first
    return [gi.x[j] for j in order] + [n for ns in cnames for n in ns], [gi.domains[j] for j in order]


def load_gam(ki, files):
    """GamMojoReader: the fields the scorer needs (reader order)."""
    def f(k, default="[]"):
        from .reader import _floats
        return _floats(ki.get(k, default))

    def lines(name):
        b = files[name]
        return [s for s in (b.decode() if isinstance(b, bytes) else b).split("\n") if s]

    def d3(name, dims):
        raw = np.frombuffer(files[name], dtype=">f8") if name in files else np.zeros(0)
        out, pos = [], 0
        for a, b in dims:
            out.append(raw[pos:pos + a * b].reshape(a, b).astype(np.float64))
            pos += a * b
        return out
    bs = [int(v) for v in f("bs_sorted")]
    nk = [int(v) for v in f("num_knots_sorted")]
    orders = [int(v) for v in f("spline_orders_sorted")] if "spline_orders_sorted" in ki else [0] * len(bs)
    dims = [int(v) for v in f("gam_column_dim_sorted")]
    cols_flat = lines("gam_columns_sorted")
    cols, pos = [], 0
    for d in dims:
        cols.append(cols_flat[pos:pos + d])
        pos += d
    basis = [k if b == 0 else k + o - 2 for b, k, o in zip(bs, nk, orders)]
    zdims = [(0, 0) if b == 2 else (n - 1, n) for b, n in zip(bs, basis)]
    st = dict(bs=bs, num_knots=nk, orders=orders, cols=cols,
              knots=[k[0] for k in d3("knots", [(1, n) for n in nk])],
              zT=d3("zTranspose", zdims),
              binvD=d3("_binvD", [(n - 2, n) for b, n in zip(bs, nk) if b == 0]),
              beta_center=np.asarray(f("beta_center")), cats=int(ki["cats"]),
              cat_offsets=[int(v) for v in f("cat_offsets")], nums=int(ki["numsCenter"]),
              use_all=ki.get("use_all_factor_levels") == "true", num_fill=f("numNAFillsCenter"),
              cat_fill=[int(v) for v in f("catNAFills")], family=ki["family"], link=ki["link"],
              tlp=float(ki.get("tweedie_link_power", 0.0)), gam_fill=f("gam_na_fill_sorted"))
    return st


def score_gam(st, X_lin, gam_x):
    """GamMojoModel.gamScore0: eta = beta_center . [cat one-hot, numerics, centred smoother bases] +
    intercept, then the inverse link (X_lin [F_lin, N] in cats-then-nums order; gam_x: per smoother [N])."""
    from ..models.gam import cr_basis, ispline_basis, mspline_basis
    dev = X_lin.device
    N = X_lin.shape[1]
    beta = torch.as_tensor(st["beta_center"], dtype=torch.float64, device=dev)
    eta = torch.full((N,), float(beta[-1]), dtype=torch.float64, device=dev)
    co = st["cat_offsets"]
    for i in range(st["cats"]):
        v = X_lin[i].double()
        v = torch.where(torch.isnan(v), torch.full_like(v, float(st["cat_fill"][i])), v)
        iv = v.long() if st["use_all"] else v.long() - 1
        idx = iv + co[i]
        ok = (iv >= 0) & (idx < co[i + 1])
        eta = eta + torch.where(ok, beta[idx.clamp(0, beta.numel() - 1)], torch.zeros_like(eta))
    noff = co[st["cats"]]
    for j in range(st["nums"]):
        v = X_lin[st["cats"] + j].double()
        v = torch.where(torch.isnan(v), torch.full_like(v, float(st["num_fill"][j])), v)
        eta = eta + beta[noff + j] * v
    pos = noff + st["nums"]
    cs = 0
    for g, (b, x) in enumerate(zip(st["bs"], gam_x)):
        x = torch.nan_to_num(x.double(), nan=float(st["gam_fill"][g]) if st["gam_fill"] else 0.0)
        kn = torch.as_tensor(st["knots"][g], dtype=torch.float64, device=dev)
        if b == 0:
            F = torch.cat([torch.zeros(1, kn.numel(), dtype=torch.float64),
                           torch.as_tensor(st["binvD"][cs]), torch.zeros(1, kn.numel(), dtype=torch.float64)])
            cs += 1
            B = cr_basis(x, kn.cpu(), F)
        elif b == 2:
            B = ispline_basis(x, kn, st["orders"][g])
        else:
            B = mspline_basis(x, kn, st["orders"][g])
        zT = st["zT"][g]
        if zT.size:
            B = B @ torch.as_tensor(zT.T, dtype=torch.float64, device=dev)
        nb = B.shape[1]
        eta = eta + B @ beta[pos:pos + nb]
        pos += nb
    return eta
