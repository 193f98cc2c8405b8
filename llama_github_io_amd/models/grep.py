"""Grep "model" (reference: ``h2o-algos/src/main/java/hex/grep/Grep.java``, ``GrepModel.java``): run a
regular expression over raw text and keep every match with its byte offset.

The reference scans the chunks of an unparsed ByteVec (a match may straddle into the next chunk). Here
the text is either a file (``path`` parameter, read as bytes) or a frame with one string column whose
rows are joined by newlines, decoded as Latin-1 so character offsets equal byte offsets. The scan walks
fixed-size chunks with a look-ahead overlap, keeping a match only in the chunk where it starts — the
reference's ``m.start() < bs0.length`` rule — so straddling matches are reported exactly once.
"""
from __future__ import annotations

import re

from .base import DataInfo, Model, make_key

_CHUNK = 1 << 22
_OVERLAP = 1 << 12


class GrepModel(Model):
    algo = "grep"

    @property
    def model_category(self):
        return "Unknown"

    def matches(self):
        return list(self.output["matches"])

    def offsets(self):
        return list(self.output["offsets"])

    def _predict_tensor(self, X, offset=None):
        raise NotImplementedError("GrepModel does not score (GrepModel.score0 is unimplemented in H2O too)")


def grep_text(text: str, pattern: str):
    rx = re.compile(pattern)
    matches, offsets = [], []
    n = len(text)
    for start in range(0, max(n, 1), _CHUNK):
        end = min(n, start + _CHUNK)
        window = text[start:min(n, end + _OVERLAP)]
        for m in rx.finditer(window):
            if m.start() + start >= end:        # starts in the next chunk: reported there
                break
            matches.append(m.group(0))
            offsets.append(start + m.start())
    return matches, offsets


class GrepTrainer:
    def __init__(self, params):
        self.p = dict(params)
        self.job = None

    def fit_text(self, training_frame=None, model_key=None):
        p = self.p
        if not p.get("regex"):
            raise ValueError("regex is missing")
        re.compile(p["regex"])                  # validation error at init, like Grep.init
        if p.get("path"):
            with open(p["path"], "rb") as f:
                text = f.read().decode("latin-1")
        else:
            if training_frame is None or training_frame.ncols != 1:
                raise ValueError("Frame must contain exactly 1 column (of raw text)")
            vals = training_frame._col(0).to_numpy()
            text = "\n".join("" if v is None else str(v) for v in vals)
        matches, offsets = grep_text(text, p["regex"])
        info = DataInfo([], [], [], None, None)
        m = GrepModel(model_key or make_key("grep"), p, info)
        m.output.update(matches=matches, offsets=offsets, model_category="Unknown")
        return m
