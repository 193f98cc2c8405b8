"""fp32 DL at 5M rows in graph mode: scoring history, overwrite_with_best_model on / off, chunk sizes."""
import json, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llama_github_io_amd.models.base import DataInfo
from llama_github_io_amd.models.deeplearning import DeepLearningTrainer

dev = torch.device("cuda")
F, N = 784, int(sys.argv[1]) if len(sys.argv) > 1 else 5_000_000
g = torch.Generator(device=dev).manual_seed(11)
X = torch.rand(F, N, device=dev, generator=g)
y = (X[:20].sum(0) > 10).float()
info = DataInfo([f"p{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])
dt = sys.argv[2] if len(sys.argv) > 2 else "float32"
for owb in (True,):
    m = DeepLearningTrainer(dict(hidden=[200, 200], epochs=1, compute_dtype=dt, mini_batch_size=4096, seed=1,
                                 stopping_rounds=0, score_interval=1e9, standardize=False,
                                 overwrite_with_best_model=owb)).fit(X, y, None, None, info)
    hist = [(round(h.get("epochs", 0), 3), round(h.get("training_logloss", float("nan")), 5),
             round(h.get("training_auc", float("nan")), 4)) for h in m.output["scoring_history"]]
    print(json.dumps(dict(dt=dt, env={k: v for k, v in os.environ.items() if k.startswith("H2O_DL")}, owb=owb, auc=m.output["training_metrics"]["AUC"], mode=m.output.get("training_step_mode"),
                          best_model_loss=m.output.get("best_model_loss"), history=hist)), flush=True)
