"""Regression: the binomial threshold table indexes ``uniq`` on a float64 lattice.

A float32 ``linspace(0, n - 1)`` rounds ``n - 1`` up past 2^24 distinct scores; the last index then
pointed one element past the end (on the GPU an out-of-bounds gather: the HSA 0x1016 memory fault of
the 100M x 50 XGBoost run)."""
import torch

from llama_github_io_amd import metrics


def test_threshold_table_index_in_bounds_past_2_pow_24():
    n = (1 << 25) + 4          # n - 1 = 2^25 + 3 is not a float32 value (rounds up to 2^25 + 4 = n)
    assert int(torch.linspace(0, n - 1, steps=400)[-1].round()) > n - 1   # the old lattice overflowed
    uniq = torch.arange(n, dtype=torch.float32).flip(0) / n
    tp = torch.arange(1, n + 1, dtype=torch.float32)
    fp = torch.zeros(n, dtype=torch.float32)
    rows = metrics._threshold_table(uniq, tp, fp, 400)
    assert len(rows) == 400
    assert rows[-1]["threshold"] == float(uniq[-1])
