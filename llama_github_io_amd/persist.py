"""Binary model save/load (reference: ``hex/Model.java`` exportBinaryModel/importBinaryModel,
``water/api/ModelsHandler.java``).

A saved model is a directory-free single file: a JSON header (algo, class, parameters, output,
DataInfo) plus every tensor of the model state in one safetensors blob — loadable without
executing anything from the file (no pickle).
"""
from __future__ import annotations

import json
import os
import struct

import numpy as np
import torch

from .core import dkv

MAGIC = b"H2OAMDM1"


def _split_state(obj, tensors, prefix="t"):
    """Move large numeric lists out of the JSON state into tensors (keeps headers small)."""
    if isinstance(obj, dict):
        return {k: _split_state(v, tensors, f"{prefix}.{k}") for k, v in obj.items()}
    if isinstance(obj, list) and len(obj) > 64 and all(isinstance(v, (int, float)) for v in obj[:64]):
        try:
            arr = np.asarray(obj, dtype=np.float64)
            if arr.ndim >= 1 and arr.dtype != object:
                name = f"{prefix}#{len(tensors)}"
                tensors[name] = torch.from_numpy(arr)
                return {"__tensor__": name}
        except (ValueError, TypeError):
            pass
    if isinstance(obj, list):
        return [_split_state(v, tensors, f"{prefix}[{i}]") for i, v in enumerate(obj)]
    return obj


def _join_state(obj, tensors):
    if isinstance(obj, dict):
        if set(obj.keys()) == {"__tensor__"}:
            return tensors[obj["__tensor__"]].numpy().tolist()
        return {k: _join_state(v, tensors) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_join_state(v, tensors) for v in obj]
    return obj


def _default(o):
    if isinstance(o, (np.floating, np.integer)):
        return o.item()
    if isinstance(o, np.ndarray):
        return o.tolist()
    if isinstance(o, torch.Tensor):
        return o.detach().cpu().tolist()
    if hasattr(o, "frame_id"):
        return o.frame_id
    if hasattr(o, "key") and isinstance(getattr(o, "key"), str):
        return o.key
    return str(o)


def save_model(model, path: str = "", force: bool = False, filename: str | None = None) -> str:
    from safetensors.torch import save as st_save
    path = path or "."
    fname = filename or model.key
    full = os.path.join(path, fname) if (os.path.isdir(path) or not os.path.splitext(path)[1]) else path
    os.makedirs(os.path.dirname(full) or ".", exist_ok=True)
    if os.path.exists(full) and not force:
        raise FileExistsError(f"{full} exists (use force=True)")
    state = model.to_state()
    state["__class__"] = type(model).__module__ + ":" + type(model).__name__
    tensors = {}
    state = _split_state(state, tensors)
    header = json.dumps(state, default=_default).encode()
    blob = st_save({k: v.contiguous() for k, v in tensors.items()}) if tensors else b""
    with open(full, "wb") as f:
        f.write(MAGIC)
        f.write(struct.pack("<QQ", len(header), len(blob)))
        f.write(header)
        f.write(blob)
    return full


_ALLOWED_MODULE_PREFIX = "llama_github_io_amd.models."


def load_model(path: str):
    import importlib
    from safetensors.torch import load as st_load
    with open(path, "rb") as f:
        if f.read(8) != MAGIC:
            raise ValueError(f"{path} is not an MI355X-native H2O binary model")
        hl, bl = struct.unpack("<QQ", f.read(16))
        state = json.loads(f.read(hl))
        blob = f.read(bl)
    tensors = st_load(blob) if bl else {}
    state = _join_state(state, tensors)
    m = _from_state(state)
    dkv.put(m.key, m)
    return m


def _from_state(state: dict):
    """Rebuild a model object from its ``to_state()`` dict (only classes of this package)."""
    import importlib
    modname, clsname = state.pop("__class__").split(":")
    if not modname.startswith(_ALLOWED_MODULE_PREFIX):
        raise ValueError(f"refusing to instantiate {modname}")
    cls = getattr(importlib.import_module(modname), clsname)
    from .models.base import DataInfo, default_device
    info = DataInfo.from_state(state["info"])
    m = cls(state["key"], state["params"], info)
    m._restore(state)
    m.device = default_device()
    _to_device(m, m.device)
    return m


def _to_device(m, dev):
    for name in ("beta", "centers_std", "bias"):
        v = getattr(m, name, None)
        if isinstance(v, torch.Tensor):
            setattr(m, name, v.to(dev))
    ex = getattr(m, "expander", None)
    if ex is not None and hasattr(ex, "to"):
        ex.to(dev)
    net = getattr(m, "net", None)
    if net is not None:
        net.to(dev)
