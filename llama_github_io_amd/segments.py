"""Segment models (reference: ``h2o-core/src/main/java/hex/segments/SegmentModelsBuilder.java``,
``SegmentModels.java``; h2o-py ``H2OEstimator.train_segments`` / ``H2OSegmentModels``).

One model per distinct combination of the ``segment_columns`` values (or per row of an explicit
``segments`` frame). Only the segment columns travel to the host to enumerate the segments; each
segment's rows are gathered on device and trained through the ordinary ModelBuilder path,
``parallelism`` models at a time on worker threads. Failures are recorded per segment (status
``FAILED`` + error text) instead of aborting the run, as in the reference.
"""
from __future__ import annotations

import concurrent.futures as cf
import traceback

import numpy as np
import torch

from .core import dkv
from .frame import Column, H2OFrame, engine_device
from .models.base import make_key


class SegmentModels:
    def __init__(self, key, segment_columns, rows):
        self.key = key
        self.segment_columns = list(segment_columns)
        self.rows = rows            # per segment: segment values + model / status / errors / warnings

    def as_frame(self) -> H2OFrame:
        dev = engine_device()
        cols = []
        for c in self.segment_columns:
            vals = [r[c] for r in self.rows]
            if all(isinstance(v, (int, float, np.floating, np.integer)) for v in vals):
                cols.append(Column(c, "real", torch.tensor([float(v) for v in vals], dtype=torch.float64, device=dev)))
            else:
                dom = sorted({str(v) for v in vals})
                lut = {s: i for i, s in enumerate(dom)}
                cols.append(Column(c, "enum", torch.tensor([lut[str(v)] for v in vals], dtype=torch.int32, device=dev), dom))
        for name in ("model", "status", "errors", "warnings"):
            cols.append(Column(name, "string", strings=np.array([r.get(name) for r in self.rows], dtype=object)))
        return H2OFrame._from_columns(cols)

    def models(self):
        return [dkv.get(r["model"]) for r in self.rows if r.get("model")]


def _segments(frame: H2OFrame, segment_columns, segments=None):
    """[(values tuple, row-index tensor)] for every segment present in ``frame`` (and in ``segments``)."""
    df = frame[segment_columns].as_data_frame()
    groups = df.groupby(segment_columns, sort=True, dropna=False).indices
    want = None
    if segments is not None:
        want = {tuple(str(v) for v in r) for r in segments[segment_columns].as_data_frame().itertuples(index=False)}
    out = []
    dev = engine_device()
    for key, idx in groups.items():
        vals = key if isinstance(key, tuple) else (key,)
        if want is not None and tuple(str(v) for v in vals) not in want:
            continue
        out.append((vals, torch.as_tensor(np.asarray(idx), dtype=torch.long, device=dev)))
    return out


def train_segments(algo, params, x, y, training_frame: H2OFrame, segment_columns, segments=None,
                   validation_frame=None, parallelism=1, segment_models_id=None) -> SegmentModels:
    from .models import builder
    segment_columns = [segment_columns] if isinstance(segment_columns, str) else list(segment_columns)
    segs = _segments(training_frame, segment_columns, segments)
    x = [c for c in (x or training_frame.names) if c not in segment_columns and c != y]
    out = [None] * len(segs)

    def one(pos):
        vals, rows = segs[pos]
        rec = {c: (v.item() if hasattr(v, "item") else v) for c, v in zip(segment_columns, vals)}
        try:
            m = builder.train(algo, dict(params), x, y, training_frame._rows(rows), None, None,
                              make_key(f"{algo}_segment"))
            rec.update(model=m.key, status="SUCCEEDED", errors=None, warnings=None)
        except Exception as e:  # noqa: BLE001 - a failed segment is reported, not raised
            rec.update(model=None, status="FAILED", errors=f"{type(e).__name__}: {e}",
                       warnings=traceback.format_exc(limit=1).strip())
        out[pos] = rec

    if int(parallelism) <= 1:
        for pos in range(len(segs)):
            one(pos)
    else:
        with cf.ThreadPoolExecutor(max_workers=int(parallelism)) as ex:
            list(ex.map(one, range(len(segs))))
    sm = SegmentModels(segment_models_id or make_key("segment_models"), segment_columns, out)
    dkv.put(sm.key, sm)
    return sm
