"""XGBoost MOJO in the reference layout (``h2o-extensions/xgboost/.../XGBoostMojoWriter.java``,
``h2o-genmodel-extensions/xgboost/.../XGBoostMojoReader.java``): ``model.ini`` keys ``nums`` / ``cats`` /
``cat_offsets`` / ``use_all_factor_levels`` / ``sparse`` / ``booster`` / ``ntrees`` /
``use_java_scoring_by_default`` / ``has_offset``, the ``feature_map`` blob, and ``boosterBytes`` = the
libxgboost legacy binary model (little endian):

* LearnerModelParam (136 B): ``float base_score, uint num_feature, int num_class, int contain_extra_attrs,
  int contain_eval_metrics, uint major_version, uint minor_version, int reserved[27]``
* ``string name_obj``, ``string name_gbm`` (uint64 length + bytes)
* GBTreeModelParam (160 B): ``int num_trees, num_roots, num_feature, pad, int64 num_pbuffer_deprecated,
  int num_output_group, size_leaf_vector, int reserved[32]``
* per tree: TreeParam (37 ints: ``num_roots, num_nodes, num_deleted, max_depth, num_feature,
  size_leaf_vector, reserved[31]``), nodes (20 B: ``int parent, cleft, cright; uint sindex`` (bit 31 =
  default left); ``float info`` = split condition or leaf value), stats (16 B: ``float loss_chg, sum_hess,
  base_weight; int leaf_child_cnt``) — the layout ``XGBoostRegTree`` reads (NODE_SIZE 20, STATS_SIZE 16)
* ``int tree_info[num_trees]`` (output group of each tree)

Trees are written from the framework's numeric splits (``x < thr`` left, NaN -> default direction);
categorical predictors would need the reference's one-hot encoding, so such models keep the native payload.
``base_score`` is stored in probability space for logistic objectives (the predictor maps it to a margin).
"""
from __future__ import annotations

import math
import struct

import numpy as np

OBJECTIVES = {"bernoulli": "binary:logistic", "multinomial": "multi:softprob", "gaussian": "reg:squarederror",
              "poisson": "count:poisson", "gamma": "reg:gamma", "tweedie": "reg:tweedie"}


def supported(model) -> bool:
    return (model.output.get("booster", "gbtree") in ("gbtree", "dart") and model.forest is not None
            and not any(int(c) for c in model.info.iscat)
            and model.output.get("distribution") in OBJECTIVES)


def _str(s: str) -> bytes:
    b = s.encode()
    return struct.pack("<Q", len(b)) + b


def _margin_to_base_score(obj: str, m: float) -> float:
    if obj == "binary:logistic":
        return 1.0 / (1.0 + math.exp(-m))
    if obj in ("count:poisson", "reg:gamma", "reg:tweedie"):
        return math.exp(m)
    return m


def _base_score_to_margin(obj: str, b: float) -> float:
    if obj == "binary:logistic":
        return math.log(b / (1.0 - b))
    if obj in ("count:poisson", "reg:gamma", "reg:tweedie"):
        return math.log(b)
    return b


def _tree_bytes(t) -> bytes:
    n = t.n_nodes
    parent = np.full(n, -1, dtype=np.int64)
    for i in range(n):
        if t.feat[i] >= 0:
            parent[t.left[i]] = i | (1 << 31)       # RegTree::Node::SetParent: top bit = "is left child"
            parent[t.right[i]] = i
    depth = t.depth()
    out = [struct.pack("<6i31i", 1, n, 0, depth, 0, 0, *([0] * 31))]
    nodes = bytearray()
    stats = bytearray()
    for i in range(n):
        p = int(parent[i])
        p32 = struct.unpack("<i", struct.pack("<I", p & 0xFFFFFFFF))[0] if p >= 0 else -1
        if t.feat[i] >= 0:
            sidx = int(t.feat[i]) | ((1 << 31) if t.na_left[i] else 0)
            nodes += struct.pack("<iiiIf", p32, int(t.left[i]), int(t.right[i]), sidx, float(t.thr[i]))
            stats += struct.pack("<fffi", float(t.gain[i]), float(t.cover[i]), 0.0, 0)
        else:
            nodes += struct.pack("<iiiIf", p32, -1, -1, 0, float(t.value[i]))
            stats += struct.pack("<fffi", 0.0, float(t.cover[i]), float(t.value[i]), 0)
    out.append(bytes(nodes))
    out.append(bytes(stats))
    return b"".join(out)


def booster_bytes(model) -> bytes:
    fr = model.forest
    F = model.info.F
    d = model.output["distribution"]
    obj = OBJECTIVES[d]
    K = max(fr.K, 1)
    init = model.init_f if isinstance(model.init_f, (list, tuple, np.ndarray)) else [model.init_f]
    init = [float(v) for v in np.atleast_1d(np.asarray(init, dtype=np.float64))]
    # one global base margin in xgboost: a per-class init is folded into that class's first tree
    base_m = init[0] if K == 1 else 0.0
    b = [struct.pack("<fIiiiII27i", _margin_to_base_score(obj, base_m), F, K if K > 1 else 0, 0, 0, 1, 0,
                     *([0] * 27))]
    b.append(_str(obj))
    b.append(_str("gbtree"))
    trees = list(fr.trees)
    b.append(struct.pack("<iiiiqii32i", len(trees), 1, F, 0, 0, K, 0, *([0] * 32)))
    seen = set()
    for t, c in zip(trees, fr.tree_class):
        if K > 1 and c not in seen and init[c] != 0.0:
            seen.add(c)
            t = _shift_leaves(t, init[c])
        b.append(_tree_bytes(t))
    b.append(struct.pack(f"<{len(trees)}i", *[int(c) for c in fr.tree_class]))
    return b"".join(b)


def _shift_leaves(t, delta):
    import copy
    t2 = copy.copy(t)
    t2.value = np.where(t.feat < 0, t.value + np.float32(delta), t.value).astype(t.value.dtype)
    return t2


def feature_map(model) -> bytes:
    """``XGBoostUtils.makeFeatureMap``: one ``index name type`` line per input column (q = quantitative)."""
    return "".join(f"{i} {n} q\n" for i, n in enumerate(model.info.x)).encode()


def write(model, kv, blobs):
    blobs["boosterBytes"] = booster_bytes(model)
    blobs["feature_map"] = feature_map(model)
    F = model.info.F
    kv["nums"] = F
    kv["cats"] = 0
    kv["cat_offsets"] = "[0]"
    kv["use_all_factor_levels"] = "true"
    kv["sparse"] = "false"
    kv["booster"] = model.output.get("booster", "gbtree")
    kv["ntrees"] = len(model.forest.trees) // max(model.forest.K, 1)
    kv["use_java_scoring_by_default"] = "true"
    kv["has_offset"] = "true" if model.info.offset else "false"
    kv["distribution"] = model.output["distribution"]


# ------------------------------------------------------------------------------------------------ reader
def read(buf: bytes):
    """Parse ``boosterBytes`` -> (objective, base margin, num_class, [Tree], [tree class])."""
    from ..ops.forest import Tree
    off = 0
    if buf[:4] == b"binf":
        off = 4
    base_score, num_feature, num_class = struct.unpack_from("<fIi", buf, off)
    off += 136

    def rstr(o):
        (n,) = struct.unpack_from("<Q", buf, o)
        return buf[o + 8:o + 8 + n].decode(), o + 8 + n
    obj, off = rstr(off)
    gbm, off = rstr(off)
    if gbm != "gbtree":
        raise NotImplementedError(f"booster {gbm}")
    num_trees = struct.unpack_from("<i", buf, off)[0]
    off += 160
    trees = []
    for _ in range(num_trees):
        _, n = struct.unpack_from("<ii", buf, off)
        off += 37 * 4
        rec = np.frombuffer(buf, dtype=np.dtype([("parent", "<i4"), ("cleft", "<i4"), ("cright", "<i4"),
                                                 ("sindex", "<u4"), ("info", "<f4")]), count=n, offset=off)
        off += 20 * n
        st = np.frombuffer(buf, dtype=np.dtype([("loss", "<f4"), ("hess", "<f4"), ("bw", "<f4"), ("cnt", "<i4")]),
                           count=n, offset=off)
        off += 16 * n
        leaf = rec["cleft"] == -1
        trees.append(Tree(feat=np.where(leaf, -1, (rec["sindex"] & 0x7FFFFFFF).astype(np.int64)),
                          thr=np.where(leaf, 0.0, rec["info"]).astype(np.float32),
                          bin=np.zeros(n, np.int64), na_left=((rec["sindex"] >> 31) & 1).astype(bool) & ~leaf,
                          is_cat=np.zeros(n, bool), cat_bits=[None] * n, cat_nbits=np.zeros(n, np.int64),
                          left=rec["cleft"].astype(np.int64), right=rec["cright"].astype(np.int64),
                          value=np.where(leaf, rec["info"], 0.0).astype(np.float32),
                          cover=st["hess"].astype(np.float64), gain=st["loss"].astype(np.float64)))
    tree_info = list(np.frombuffer(buf, dtype="<i4", count=num_trees, offset=off))
    return obj, _base_score_to_margin(obj, float(base_score)), int(num_class), trees, [int(c) for c in tree_info]
