"""Time one K-Means Lloyd step (assignment + centroid sums) on the GPU: MFMA kernel vs the LDS scalar
kernel, 10M x 20, k = 10 (BASELINE.json secondary config). Prints one JSON line per variant."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llama_github_io_amd.ops.dense import kmeans_step  # noqa: E402

N, P, K = int(os.environ.get("KM_N", 10_000_000)), int(os.environ.get("KM_P", 20)), int(os.environ.get("KM_K", 10))
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
X = torch.randn(N, P, device=dev, generator=g)
C = torch.randn(K, P, device=dev, generator=g)
for variant in ("1", "0"):
    os.environ["H2O_KMEANS_MFMA"] = variant
    for _ in range(3):
        kmeans_step(X, C)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    it = 20
    for _ in range(it):
        a, d, s, c = kmeans_step(X, C)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / it
    print(json.dumps(dict(kernel="mfma" if variant == "1" else "lds_scalar", N=N, P=P, K=K, ms_per_lloyd_step=round(ms, 4),
                          effective_GBps=round(N * P * 4 / ms / 1e6, 1))), flush=True)
