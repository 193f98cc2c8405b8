"""Checkpoint / resume: tree models continue from a previous model (== uninterrupted training),
in-training checkpoints are resumable, DeepLearning continues epochs, export_checkpoints_dir."""
import os

import numpy as np
import torch

from llama_github_io_amd import persist
from llama_github_io_amd.core import dkv
from llama_github_io_amd.models.base import DataInfo


def _d():
    g = torch.Generator().manual_seed(0)
    X = torch.randn(4, 3000, generator=g)
    y = (X[0] + X[1] * X[2] > 0).float()
    return X, y, DataInfo(list("abcd"), np.zeros(4, np.int32), [None] * 4, "y", ["0", "1"])


def test_gbm_checkpoint_equals_uninterrupted():
    from llama_github_io_amd.models.gbm import GBMTrainer
    X, y, info = _d()
    full = GBMTrainer(dict(ntrees=10, seed=1)).fit(X, y, None, None, info)
    a = GBMTrainer(dict(ntrees=4, seed=1)).fit(X, y, None, None, info)
    dkv.put(a.key, a)
    b = GBMTrainer(dict(ntrees=10, seed=1, checkpoint=a.key)).fit(X, y, None, None, info)
    assert len(b.forest.trees) == 10
    assert torch.allclose(full._predict_tensor(X), b._predict_tensor(X), atol=1e-5)


def test_in_training_checkpoints_resume(tmp_path):
    from llama_github_io_amd.models.gbm import GBMTrainer
    X, y, info = _d()
    m = GBMTrainer(dict(ntrees=6, seed=1, in_training_checkpoints_dir=str(tmp_path),
                        in_training_checkpoints_tree_interval=2)).fit(X, y, None, None, info)
    files = sorted(os.listdir(tmp_path))
    assert len(files) == 3
    snap = persist.load_model(os.path.join(tmp_path, files[0]))
    assert len(snap.forest.trees) == 2
    b = GBMTrainer(dict(ntrees=6, seed=1, checkpoint=snap.key)).fit(X, y, None, None, info)
    assert torch.allclose(m._predict_tensor(X), b._predict_tensor(X), atol=1e-5)


def test_deeplearning_checkpoint():
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    X, y, info = _d()
    a = DeepLearningTrainer(dict(hidden=[16], epochs=1, seed=1, mini_batch_size=32)).fit(X, y, None, None, info)
    dkv.put(a.key, a)
    c = DeepLearningTrainer(dict(hidden=[16], epochs=4, seed=1, checkpoint=a.key, mini_batch_size=32)).fit(X, y, None, None, info)
    assert abs(c.output["epochs"] - 4) < 0.1
    assert c.output["training_metrics"]["AUC"] >= a.output["training_metrics"]["AUC"] - 0.02


def test_memory_backpressure_triggers(monkeypatch):
    """MemoryManager back-pressure: over the high-water mark a DKV put / model build spills LRU frames,
    and a device OOM inside a build spills then retries once."""
    import torch
    from llama_github_io_amd.utils import memory
    calls = []
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    monkeypatch.setattr(memory, "device_usage", lambda device=None: dict(total=100, free=5, used=95, allocated=90))
    monkeypatch.setattr(memory, "clean", lambda target=None: calls.append(target) or 7)
    assert memory.pressure_check() == 7 and calls == [None]
    n = {"i": 0}

    def flaky():
        n["i"] += 1
        if n["i"] == 1:
            raise torch.cuda.OutOfMemoryError("HIP out of memory")
        return "ok"
    monkeypatch.setattr(torch.cuda, "empty_cache", lambda: None)
    assert memory.with_backpressure(flaky) == "ok" and n["i"] == 2 and calls[-1] == 0.5
