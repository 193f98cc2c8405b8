"""DeepLearning at H2O's default ``mini_batch_size = 1`` (one ADADELTA step per row, Neurons.java:229-296): the GPU
engine's default step size rule (``models/deeplearning.py``: B = N // 16384 rows per step) keeps one-epoch quality
within 10 % of the per-row reference. Pinned with the fp64 NumPy oracle of ``scripts/dl_default_semantics.py``
(profiles/r6_dl_default_semantics.md holds the 10k / 100k / 1M table)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def test_default_batch_rule_matches_per_row_quality():
    import dl_default_semantics as S
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    n, F = 60000, 100
    X, y = S.data(n, F, 0)
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    m = DeepLearningTrainer(dict(hidden=[32, 32], epochs=1, seed=1, activation="Tanh", score_interval=1e9,
                                 stopping_rounds=0)).fit(torch.tensor(X.T, dtype=torch.float32).contiguous(),
                                                         torch.tensor(y, dtype=torch.float32), None, None, info)
    B = m.output["mini_batch_rows"]
    assert B == n // 16384 == 3
    per_row = S.logloss(S.train_one_epoch(X, y, 1, 32), X, y)
    engine_rule = S.logloss(S.train_one_epoch(X, y, B, 32), X, y)
    old_rule = S.logloss(S.train_one_epoch(X, y, min(256, n // 1024), 32), X, y)
    assert engine_rule <= 1.10 * per_row, (engine_rule, per_row)
    assert old_rule > 1.10 * per_row           # the former N // 1024 rule was not
