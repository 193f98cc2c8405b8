"""fp32 DL at 10M rows: check the expander's row-major Z against X on sampled rows, then short trainings."""
import os, sys, json
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llama_github_io_amd.models.base import DataInfo
from llama_github_io_amd.models.datainfo import Expander

dev = torch.device("cuda")
F, N = 784, int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
g = torch.Generator(device=dev).manual_seed(11)
X = torch.rand(F, N, device=dev, generator=g)
info = DataInfo([f"p{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
for dt in (torch.float32, torch.bfloat16):
    ex = Expander(info, standardize=False).fit(X)
    Z = ex.transform(X, dtype=dt)
    idx = torch.tensor([0, 1, 12345, N // 2, N - 7, N - 1], device=dev)
    ref = X[:, idx].T.to(dt)
    err = (Z[idx].float() - ref.float()).abs().max().item()
    print(json.dumps(dict(dtype=str(dt), N=N, Z_shape=list(Z.shape), Z_stride=list(Z.stride()), max_err=err)), flush=True)
    del Z
    torch.cuda.empty_cache()
