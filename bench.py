#!/usr/bin/env python
"""Headline benchmark: GBM train rows/sec (100 trees, depth 6) on HIGGS-11M-shaped data.

BASELINE.json metric: "GBM train rows/sec (100 trees, depth 6) on HIGGS-11M at 1/2/4/8 MI355X".
Data: synthetic HIGGS-shaped matrix (11,000,000 rows x 28 float features, binary label, ~53 %
positives; 21 "low-level" features incl. discrete b-tag-like columns + 7 "high-level" nonlinear
combinations) generated on device from a fixed seed — no dataset download is possible here.

Model config: H2O GBM, distribution=bernoulli, ntrees=100, max_depth=6, min_rows=10, learn_rate=0.1,
sample_rate=1, histogram_type=QuantilesGlobal (255 global quantile bins), fp32 compute.

A "step" = one boosting iteration (one full tree: gradients, histograms, splits, partition, leaf
values, prediction update). The timed region covers exactly K steps between barrier+synchronize.
``value`` = rows/sec of a 100-tree training = N_total / (100 * ms_per_step / 1000), whole job.
Multi-GPU (torchrun): rows are sharded over ranks (strong scaling: total rows fixed); per-level
histograms and leaf sums are all-reduced over RCCL.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def make_higgs_like(n: int, seed: int, device) -> tuple:
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    F = 28
    X = torch.empty(F, n, device=device, dtype=torch.float32)
    # 21 low-level kinematic features: momenta (lognormal-ish), angles (uniform), b-tags (discrete)
    for f in range(21):
        kind = f % 4
        if kind == 0:
            X[f] = torch.exp(0.5 * torch.randn(n, generator=g, device=device))
        elif kind == 1:
            X[f] = torch.randn(n, generator=g, device=device)
        elif kind == 2:
            X[f] = (torch.rand(n, generator=g, device=device) * 2 - 1) * 3.1416
        else:
            X[f] = torch.randint(0, 3, (n,), generator=g, device=device).float() * 1.0865
    # 7 high-level features: nonlinear combinations (invariant masses)
    for j in range(7):
        a, b, c = X[(3 * j) % 21], X[(3 * j + 1) % 21], X[(3 * j + 5) % 21]
        X[21 + j] = torch.sqrt(torch.abs(a * b + 0.5 * c * c) + 0.1) + 0.05 * torch.randn(n, generator=g, device=device)
    logit = (0.9 * X[21] - 0.7 * X[22] + 0.5 * X[23] * X[24] - 0.4 * torch.sin(X[2]) * X[1]
             + 0.3 * X[3] - 0.35 * (X[25] > 1.2).float() + 0.25 * X[0] * X[5] - 0.3)
    y = (torch.rand(n, generator=g, device=device) < torch.sigmoid(logit)).float()
    return X, y


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _self_launch(n: int) -> int:
    """``bench.py --gpus N`` without a launcher: start N fresh child ranks (one process per GPU, the same env
    contract torch.distributed.run sets) BEFORE this process touches the GPU, wait for them and exit with the
    worst child status. Rank 0 prints the one aggregated JSON line. A failing rank takes the others down (they
    would otherwise wait in a collective forever)."""
    import subprocess
    on_cpu = "cpu" in sys.argv[sys.argv.index("--device") + 1:][:1] if "--device" in sys.argv else False
    ndev = torch.cuda.device_count()          # counting devices does not initialise the GPU on this image
    if not on_cpu and 0 < ndev < n:
        print(f"bench.py: --gpus {n} but only {ndev} visible devices", file=sys.stderr)
        return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            c = procs[r].poll()
            if c is None:
                continue
            alive.discard(r)
            if c != 0:
                rc = rc or (c if c > 0 else 128 - c)
                for o in alive:                 # exactly the PIDs this launcher started
                    procs[o].terminate()
        time.sleep(0.05)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rows", type=int, default=11_000_000)
    ap.add_argument("--depth", type=int, default=6)
    ap.add_argument("--no-job", action="store_true", help="skip the whole 100-tree job measurement")
    ap.add_argument("--no-auto", action="store_true", help="skip the AUTO-histogram side measurement")
    ap.add_argument("--auto-steps", type=int, default=20, help="timed AUTO-histogram trees reported next to the "
                    "headline (auto_ms_per_tree; H2O's default histogram_type)")
    ap.add_argument("--histogram-type", default="QuantilesGlobal",
                    help="H2O histogram_type (the headline config is QuantilesGlobal; AUTO = UniformAdaptive with "
                    "nbins_top_level=1024, H2O's default)")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default: nccl = RCCL on GPUs, gloo on CPU)")
    ap.add_argument("--device", default=None, help="cuda | cpu (default: cuda when available); cpu runs the "
                    "reference builder, for multi-rank rehearsals of the collective protocol")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(_self_launch(args.gpus))
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus:
            print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a rank count the "
                  "launcher did not start", file=sys.stderr)
            sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and args.device != "cpu"
    backend = None
    if world > 1:
        import torch.distributed as dist
        backend = args.backend or ("nccl" if use_gpu else "gloo")
        if use_gpu:
            torch.cuda.set_device(local)
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local) if use_gpu else torch.device("cpu")

    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.gbm import GBMTrainer
    from llama_github_io_amd.parallel import collectives as coll

    comm_world = coll.world() if coll.is_dist() else 1
    n_total = args.rows
    # every rank draws the SAME global dataset and keeps its contiguous row shard: the N-GPU job trains on
    # exactly the rows of the 1-GPU job (strong scaling on one dataset)
    base, rem = divmod(n_total, world)
    r0 = rank * base + min(rank, rem)
    n_local = base + (1 if rank < rem else 0)
    Xg, yg = make_higgs_like(n_total, 1234, dev)
    X, y = Xg[:, r0:r0 + n_local].contiguous(), yg[r0:r0 + n_local].contiguous()
    del Xg, yg
    F = X.shape[0]
    info = DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])

    def sync():
        coll.barrier()
        if dev.type == "cuda":
            torch.cuda.synchronize()

    def max_over_ranks(v: float) -> float:
        if world == 1:
            return v
        import torch.distributed as dist
        t = torch.tensor([v], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed_fit(hist_type: str, warmup: int, steps: int):
        """Train warmup + steps trees; time exactly the last ``steps`` (barrier + synchronize on both sides)."""
        params = dict(ntrees=warmup + steps, max_depth=args.depth, min_rows=10, learn_rate=0.1, seed=42,
                      distribution="bernoulli", histogram_type=hist_type)
        times = {}

        # the trainer exposes a per-tree hook so the bench can time exactly K steps after W warmup steps
        class TimedGBM(GBMTrainer):
            def _prepare(self, t, k):
                if t == warmup and k == 0:
                    sync()
                    coll.stats(reset=True)
                    times["t0"] = time.perf_counter()
                return super()._prepare(t, k)

            def _finish(self, model, built):
                super()._finish(model, built)
                sync()
                times["t1"] = time.perf_counter()
                times["comm"] = coll.stats()

        model = TimedGBM(params).fit(X, y, None, None, info)
        return model, max_over_ranks(times["t1"] - times["t0"]), times["comm"], params

    model, dt, comm, params = timed_fit(args.histogram_type, args.warmup, args.steps)
    # the whole 100-tree job as a user runs it (binning, 100 trees, training metrics), untimed by the
    # driver contract but reported next to the per-tree value
    job_ms = None
    if not args.no_job:
        sync()
        j0 = time.perf_counter()
        GBMTrainer(dict(params, ntrees=100)).fit(X, y, None, None, info)
        sync()
        job_ms = max_over_ranks((time.perf_counter() - j0) * 1000.0)
    # H2O's DEFAULT histogram (AUTO = UniformAdaptive, nbins_top_level 1024) on the same data, same window shape
    auto_ms = None
    if not args.no_auto and args.histogram_type.lower() != "auto" and args.auto_steps > 0:
        _, adt, _, _ = timed_fit("AUTO", args.warmup, args.auto_steps)
        auto_ms = adt * 1000.0 / args.auto_steps
    ms_per_step = dt * 1000.0 / args.steps
    rows_per_sec = n_total / (100 * ms_per_step / 1000.0)
    tm = model.output["training_metrics"]
    if rank == 0:
        print(json.dumps({
            "metric": "GBM train rows/sec (100 trees, depth 6) on HIGGS-11M at 1/2/4/8 MI355X",
            "value": round(rows_per_sec, 1), "unit": "rows/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "fp32", "data": "synthetic HIGGS-shaped 11M x 28",
            # ranks of the RCCL communicator the trees' collectives ran on (0: none — one GPU, or gloo on the CPU)
            "rccl_world": comm_world if backend == "nccl" else 0,
            "comm_backend": backend, "comm_world": comm_world,
            "config": {"model": "GBM bernoulli ntrees=100 max_depth=6 min_rows=10 lr=0.1 " + (
                           "QuantilesGlobal(255 bins)" if args.histogram_type == "QuantilesGlobal" else args.histogram_type),
                       "global_batch": n_total, "seq_len": None, "parallelism": f"dp{world} (row-sharded, hist all-reduce)",
                       "rows": n_total, "rows_per_rank": n_local, "features": F,
                       "train_auc_after_all_trees": tm.get("AUC") if tm else None,
                       "collectives_per_tree": round(comm["calls"] / args.steps, 2),
                       "comm_bytes_per_tree": int(comm["bytes"] / args.steps),
                       "job_100_trees_ms_incl_binning_and_metrics": None if job_ms is None else round(job_ms, 1),
                       "job_rows_per_sec": None if job_ms is None else round(n_total * 1000.0 / job_ms, 1),
                       "auto_ms_per_tree": None if auto_ms is None else round(auto_ms, 4)},
        }), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
