"""H2OTree: one tree of a GBM / DRF / XGBoost / IF model as linked node objects (reference
``h2o-py/h2o/tree/tree.py``; server side ``hex/tree/TreeHandler.java``). Built from the same TreeV3 arrays GET
/3/Tree returns (``llama_github_io_amd/api/routes_more.py:tree_json``), without the REST round trip."""
from __future__ import annotations

import math


def _model_of(model):
    m = getattr(model, "_model", model)
    if isinstance(m, str):
        from llama_github_io_amd.core import dkv
        m = dkv.get(m)
    if m is None or getattr(m, "forest", None) is None:
        raise ValueError("H2OTree needs a trained tree model (GBM, DRF, XGBoost, IsolationForest, ...)")
    return m


class H2ONode:
    """A node of an :class:`H2OTree` (``id``: the tree's internal node id)."""

    def __init__(self, node_id):
        self._id = node_id

    @property
    def id(self):
        return self._id

    def __str__(self):
        return f"Node ID {self._id}"


class H2OLeafNode(H2ONode):
    def __init__(self, node_id, prediction):
        super().__init__(node_id)
        self._prediction = prediction

    @property
    def prediction(self):
        return self._prediction

    def __str__(self):
        return f"Leaf node ID {self._id}. Predicted value at leaf node is {self._prediction} \n"

    def show(self):
        print(self.__str__())


class H2OSplitNode(H2ONode):
    def __init__(self, node_id, threshold, left_child, right_child, split_feature, na_direction, left_levels,
                 right_levels):
        super().__init__(node_id)
        self._threshold = threshold
        self._left_child, self._right_child = left_child, right_child
        self._split_feature = split_feature
        self._na_direction = na_direction
        self._left_levels, self._right_levels = left_levels, right_levels

    threshold = property(lambda self: self._threshold)
    left_child = property(lambda self: self._left_child)
    right_child = property(lambda self: self._right_child)
    split_feature = property(lambda self: self._split_feature)
    na_direction = property(lambda self: self._na_direction)
    left_levels = property(lambda self: self._left_levels)
    right_levels = property(lambda self: self._right_levels)

    def __str__(self):
        s = f"Node ID {self._id} \n"
        if self._left_child is not None:
            s += f"Left child node ID = {self._left_child.id}\n"
        else:
            s += "There is no left child\n"
        if self._right_child is not None:
            s += f"Right child node ID = {self._right_child.id}\n"
        else:
            s += "There is no right child\n"
        s += f"\nSplits on column {self._split_feature}\n"
        if self._threshold is not None and not (isinstance(self._threshold, float) and math.isnan(self._threshold)):
            s += f"Split threshold < {self._threshold} to the left node, >= {self._threshold} to the right node\n"
        else:
            s += f"Categorical levels going to the left node: {self._left_levels}\n"
            s += f"Categorical levels going to the right node: {self._right_levels}\n"
        return s + f"\nNA values go to the {self._na_direction}\n"

    def show(self):
        print(self.__str__())


class H2OTree:
    """``H2OTree(model, tree_number, tree_class=None, plain_language_rules="AUTO")``: node arrays in breadth-first
    order (children as positions in those arrays, -1 = none), per-node split feature / threshold / NA direction /
    categorical levels / prediction, and the linked ``root_node``."""

    def __init__(self, model, tree_number, tree_class=None, plain_language_rules="AUTO"):
        from llama_github_io_amd.api.routes_more import tree_json
        m = _model_of(model)
        r = tree_json(m, int(tree_number), tree_class, str(plain_language_rules))
        base = r["root_node_id"]
        # children as breadth-first positions (the JSON carries node ids: position + root id)
        self._left_children = [c - base if c != -1 else -1 for c in r["left_children"]]
        self._right_children = [c - base if c != -1 else -1 for c in r["right_children"]]
        self._node_ids = list(range(len(self._left_children)))
        self._descriptions = r["descriptions"]
        self._model_id = m.key
        self._tree_number = r["tree_number"]
        self._tree_class = r["tree_class"]
        self._thresholds = [float("nan") if t == "NaN" else t for t in r["thresholds"]]
        self._features = r["features"]
        self._nas = r["nas"]
        self._predictions = [float("nan") if v is None else v for v in r["predictions"]]
        self._levels = self._level_names(m, r["levels"])
        rules = r["tree_decision_path"]
        self._tree_decision_path = rules if rules is not None else "Plain language rules generation is turned off."
        self._decision_paths = r["decision_paths"] if rules is not None else \
            "Plain language rules generation is turned off."
        self._left_cat_split = [self._levels[c] if c != -1 else None for c in self._left_children]
        self._right_cat_split = [self._levels[c] if c != -1 else None for c in self._right_children]
        self._root_node = self._node(0)

    def _level_names(self, m, levels):
        """Level indices of each node's categorical split side -> level names (None for numeric splits)."""
        out = [None] * len(self._left_children)
        if m.algo == "xgboost":
            return out
        for i, f in enumerate(self._features):
            if f is None:
                continue
            dom = m.info.domains[m.info.x.index(f)] if f in m.info.x else None
            if dom is None:
                continue
            for c in (self._left_children[i], self._right_children[i]):
                if c != -1:
                    out[c] = [dom[lv] for lv in (levels[c] or [])]
        return out

    def _node(self, i):
        if i == -1:
            return None
        lc, rc = self._left_children[i], self._right_children[i]
        if lc == -1 and rc == -1:
            return H2OLeafNode(self._node_ids[i], self._predictions[i])
        return H2OSplitNode(self._node_ids[i], self._thresholds[i], self._node(lc), self._node(rc), self._features[i],
                            self._nas[i], self._levels[lc] if lc != -1 else None,
                            self._levels[rc] if rc != -1 else None)

    left_children = property(lambda self: self._left_children)
    right_children = property(lambda self: self._right_children)
    node_ids = property(lambda self: self._node_ids)
    descriptions = property(lambda self: self._descriptions)
    model_id = property(lambda self: self._model_id)
    tree_number = property(lambda self: self._tree_number)
    tree_class = property(lambda self: self._tree_class)
    thresholds = property(lambda self: self._thresholds)
    features = property(lambda self: self._features)
    levels = property(lambda self: self._levels)
    nas = property(lambda self: self._nas)
    root_node = property(lambda self: self._root_node)
    predictions = property(lambda self: self._predictions)
    tree_decision_path = property(lambda self: self._tree_decision_path)
    decision_paths = property(lambda self: self._decision_paths)
    left_cat_split = property(lambda self: self._left_cat_split)
    right_cat_split = property(lambda self: self._right_cat_split)

    def __len__(self):
        return len(self._node_ids)

    def __str__(self):
        return (f"Tree related to model {self._model_id}. Tree number is {self._tree_number}, "
                f"tree class is '{self._tree_class}'\n\n")

    def show(self):
        print(self.__str__())
