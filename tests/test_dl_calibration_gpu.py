"""DeepLearning calibration regression (r5 root cause, profiles/r5_dl_calibration.md): on uniform [0, 1] inputs the
1-epoch ADADELTA model ends miscalibrated without input standardization (fp32 logloss 0.78 at 10M x 784), while with
H2O's default standardize=True fp32 reaches a logloss at or below bf16's. A scaled-down version of the bench target."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _fit(X, y, info, cd, std):
    from llama_github_io_amd.models.deeplearning import DeepLearningTrainer
    m = DeepLearningTrainer(dict(hidden=[200, 200], epochs=1, compute_dtype=cd, mini_batch_size=1024, seed=1,
                                 stopping_rounds=0, score_interval=1e9, standardize=std,
                                 overwrite_with_best_model=False)).fit(X, y, None, None, info)
    return m.output["training_metrics"]


def test_fp32_calibrates_like_bf16_with_default_standardization():
    from llama_github_io_amd.models.base import DataInfo
    dev = torch.device("cuda", 0)
    N, F = 1_000_000, 196
    g = torch.Generator(device=dev).manual_seed(11)
    X = torch.rand(F, N, device=dev, generator=g)
    y = (X[:10].sum(0) > 5).float()
    info = DataInfo([f"p{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
    f32 = _fit(X, y, info, "float32", True)
    b16 = _fit(X, y, info, "bf16", True)
    assert f32["AUC"] > 0.99 and b16["AUC"] > 0.99, (f32["AUC"], b16["AUC"])
    assert f32["logloss"] < 0.25, f32["logloss"]
    assert f32["logloss"] <= 1.05 * b16["logloss"] + 0.005, (f32["logloss"], b16["logloss"])
