"""MOJO reader + scorer (reference: ``hex/genmodel/ModelMojoReader.java``, ``MojoReaderBackend``,
``algos/gbm/GbmMojoModel.java``, ``algos/drf/DrfMojoModel.java``, ``algos/glm/GlmMojoModel.java``,
``algos/kmeans/KMeansMojoModel.java``, ``algos/isofor/IsolationForestMojoModel.java``).

``import_mojo`` returns a :class:`~llama_github_io_amd.models.generic.GenericModel` that scores
frames without the training engine: tree blobs become flat device trees scored by the HIP forest
kernel; GLM/KMeans score with device tensor ops.
"""
from __future__ import annotations

import json
import zipfile

import numpy as np

from .treebytes import bytes_to_tree


def _unescape(s: str) -> str:
    out, i = [], 0
    while i < len(s):
        if s[i] == "\\" and i + 1 < len(s):
            out.append("\n" if s[i + 1] == "n" else s[i + 1])
            i += 2
        else:
            out.append(s[i])
            i += 1
    return "".join(out)


def parse_mojo(path: str, prefix: str = "") -> dict:
    """model.ini sections, domains and every other entry of the MOJO rooted at ``prefix`` (nested
    sub-models of a multi-model MOJO live under ``models/<key>/``)."""
    with zipfile.ZipFile(path) as z:
        ini = z.read(prefix + "model.ini").decode()
        section = None
        info, columns, domains = {}, [], {}
        for line in ini.splitlines():
            s = line.strip()
            if not s:
                continue
            if s.startswith("[") and s.endswith("]"):
                section = s[1:-1]
                continue
            if section == "info":
                k, _, v = s.partition("=")
                info[k.strip()] = v.strip()
            elif section == "columns":
                columns.append(line)
            elif section == "domains":
                ci, rest = s.split(":", 1)
                n, fname = rest.split()
                lines = z.read(f"{prefix}domains/{fname}").decode().split("\n")[: int(n)]
                domains[int(ci)] = [_unescape(x) for x in lines]
        names = [n for n in z.namelist() if n.startswith(prefix)]
        if not prefix:
            names = [n for n in names if not n.startswith("models/")]
        files = {n[len(prefix):]: z.read(n) for n in names
                 if n != prefix + "model.ini" and not n.startswith(prefix + "domains/")}
    trees = {n: b for n, b in files.items() if n.startswith("trees/") and n.endswith(".bin") and "_aux" not in n}
    state = json.loads(files["model_state.json"]) if "model_state.json" in files else None
    return dict(info=info, columns=columns, domains=domains, trees=trees, state=state, files=files, path=path,
                prefix=prefix)


def _floats(s: str):
    s = s.strip()
    if s in ("null", ""):
        return []
    return [float(x) for x in s.strip("[]").split(",") if x.strip()]


def import_mojo(path: str, model_id: str | None = None):
    from ..core import dkv
    from ..models.generic import GenericModel
    m = GenericModel.from_mojo(path, model_id)
    dkv.put(m.key, m)
    return m


def print_mojo(path: str, format="json", tree_index=None):
    mj = parse_mojo(path)
    out = dict(info=mj["info"], columns=mj["columns"], n_trees=len(mj["trees"]))
    if tree_index is not None and mj["trees"]:
        name = sorted(mj["trees"])[tree_index]
        t = bytes_to_tree(mj["trees"][name])
        out["tree"] = dict(feat=t.feat.tolist(), thr=t.thr.tolist(), left=t.left.tolist(), right=t.right.tolist(),
                           value=t.value.tolist())
    return json.dumps(out, indent=1) if format == "json" else out
