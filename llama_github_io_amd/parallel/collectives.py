"""Collectives of the row-sharded engine (the MI355X replacement of ``water/MRTask.java``'s reduce
tree and ``water/RPC.java``'s fan-out): helpers over ``torch.distributed`` that are no-ops in a single
process.

Row tensors handed to a trainer are either *sharded* (each rank holds a disjoint slice of the rows,
the default under ``WORLD_SIZE > 1``) or *replicated* (every rank holds every row, e.g. a trainer
that runs on gathered data). :func:`is_dist` answers "are the current row tensors sharded?": it is
False in a single process and inside a :func:`replicated` block, so trainers that all-reduce their
sufficient statistics (Gram, histograms, centroid sums, gradients) do so exactly when the rows are
split. Under RCCL (backend ``nccl``) device tensors go straight over xGMI; under gloo (CPU tests)
device tensors are staged through host memory.
"""
from __future__ import annotations

import contextlib
import pickle
import threading

import numpy as np
import torch
import torch.distributed as dist

_tls = threading.local()
_stats = dict(calls=0, bytes=0, row_gathers=0)


def forced_sharded() -> bool:
    """``H2O_FORCE_SHARDED=1``: a process group of ONE rank counts as a cloud, so every trainer takes its
    row-sharded path and its collectives run through the group's backend (ProcessGroupNCCL = RCCL on the
    1-GPU box: device tensors, MIN/MAX on int64, object gathers, stream order) instead of being skipped."""
    import os
    return os.environ.get("H2O_FORCE_SHARDED") == "1"


def world_active() -> bool:
    """A process group of more than one rank exists (independent of the replicated context), or one rank with
    :func:`forced_sharded`."""
    return dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or forced_sharded())


def is_dist() -> bool:
    """True when row tensors are sharded over the ranks (see module docstring)."""
    return world_active() and not getattr(_tls, "replicated", 0)


@contextlib.contextmanager
def replicated():
    """Rows are replicated on every rank inside this block: trainers must not all-reduce."""
    _tls.replicated = getattr(_tls, "replicated", 0) + 1
    try:
        yield
    finally:
        _tls.replicated -= 1


def world() -> int:
    return dist.get_world_size() if world_active() else 1


def rank() -> int:
    return dist.get_rank() if world_active() else 0


def stats(reset: bool = False) -> dict:
    """Collective call / byte counters (bench.py reports them per tree)."""
    out = dict(_stats)
    if reset:
        _stats.update(calls=0, bytes=0, row_gathers=0)
    return out


def add_stats(calls: int, nbytes: int) -> None:
    """Account collectives issued from native code (the tree driver's RCCL calls)."""
    _stats["calls"] += int(calls)
    _stats["bytes"] += int(nbytes)


def _count(t: torch.Tensor):
    _stats["calls"] += 1
    _stats["bytes"] += t.numel() * t.element_size()
    from ..utils import timeline
    timeline.record("collective", "c10d", bytes=t.numel() * t.element_size())


def _staged(t: torch.Tensor) -> bool:
    """The tensor is not on the backend's device: gloo cannot run every collective on device tensors and RCCL
    ('nccl') runs none on host tensors — stage it through the backend's device (host for gloo, the rank's GPU
    for RCCL)."""
    return t.is_cuda != (dist.get_backend() == "nccl")


def _stage(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(comm_device())


def all_reduce_(t: torch.Tensor, op=None) -> torch.Tensor:
    if is_dist():
        _count(t)
        if _staged(t):
            h = _stage(t)
            dist.all_reduce(h, op=op or dist.ReduceOp.SUM)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
    return t


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    return all_reduce_(t)


def all_reduce_max_(t: torch.Tensor) -> torch.Tensor:
    return all_reduce_(t, dist.ReduceOp.MAX)


def all_reduce_min_(t: torch.Tensor) -> torch.Tensor:
    return all_reduce_(t, dist.ReduceOp.MIN)


def reduce_scatter_(out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
    """``out`` (numel = inp.numel() / W) receives this rank's slice of the element-wise sum of ``inp``."""
    if not is_dist():
        out.copy_(inp.view_as(out))
        return out
    _count(inp)
    if _staged(inp):
        h = _stage(inp)
        dist.all_reduce(h)
        n = out.numel()
        out.copy_(h.view(-1)[rank() * n:(rank() + 1) * n].view_as(out))
    else:
        dist.reduce_scatter_tensor(out, inp)
    return out


def all_gather_into_(out: torch.Tensor, inp: torch.Tensor) -> torch.Tensor:
    """Equal-size all-gather: ``out`` = concat over ranks of ``inp`` (rank order)."""
    if not is_dist():
        out.copy_(inp.view_as(out))
        return out
    _count(inp)
    if _staged(inp):
        h = _stage(inp)
        parts = [torch.empty_like(h) for _ in range(world())]
        dist.all_gather(parts, h)
        out.copy_(torch.cat([p.reshape(-1) for p in parts]).view_as(out).to(out.device))
    else:
        dist.all_gather_into_tensor(out, inp.contiguous())
    return out


def comm_device() -> torch.device:
    """Device collectives must use: the rank's GPU under RCCL ('nccl'), the CPU under gloo."""
    if world_active() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_scalar(x: float, device=None, op=None) -> float:
    if not is_dist():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device or comm_device())
    all_reduce_(t, op)
    return float(t.item())


def all_reduce_np(a, op=None) -> np.ndarray:
    """Sum (or ``op``) of a small host array over the ranks (float64)."""
    a = np.asarray(a, dtype=np.float64)
    if not is_dist():
        return a
    t = torch.from_numpy(a.copy()).to(comm_device())
    all_reduce_(t, op)
    return t.cpu().numpy()


def all_gather_object(obj) -> list:
    """Every rank's ``obj`` (picklable), in rank order. Only for the engine's own metadata
    (domains, counts, column kinds), never for data read from outside."""
    if not world_active():
        return [obj]
    out = [None] * world()
    dist.all_gather_object(out, obj)
    return out


def broadcast_object(obj, src: int = 0):
    if not world_active():
        return obj
    box = [obj]
    dist.broadcast_object_list(box, src)
    return box[0]


def shared_entropy(modulus: int) -> int:
    """A fresh random integer in [0, modulus) that every rank agrees on (rank 0's draw): unseeded models of a
    sharded run (seed = -1) must still sample rows / columns alike on every rank."""
    v = int(np.random.SeedSequence().entropy % int(modulus))
    return int(broadcast_object(v)) if world_active() else v


def exclusive_offset(n_local: int) -> tuple:
    """(global index of this rank's first row, global row count) for a rank-ordered row split."""
    if not world_active():
        return 0, int(n_local)
    t = torch.tensor([int(n_local)], dtype=torch.int64, device=comm_device())
    parts = [torch.empty_like(t) for _ in range(world())]
    dist.all_gather(parts, t)
    counts = [int(p.item()) for p in parts]
    return int(sum(counts[:rank()])), int(sum(counts))


def all_gather_cat(t: torch.Tensor, dim: int = 0, force: bool = False, bounded: bool = False) -> torch.Tensor:
    """Variable-size all-gather along ``dim`` (rank order). ``force`` gathers even inside a
    :func:`replicated` block (frame-level gathers of sharded frames). ``bounded``: the caller gathers a
    fixed-size sample (e.g. 256 rows per isolation tree), not rows in proportion to the frame — it is not
    counted in ``stats()['row_gathers']``."""
    if not (world_active() if force else is_dist()):
        return t
    if _staged(t):
        return all_gather_cat(_stage(t), dim, force, bounded).to(t.device)
    if not bounded:
        _stats["row_gathers"] += 1
    n = torch.tensor([t.shape[dim]], device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world())]
    dist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    pad = list(t.shape)
    pad[dim] = mx - t.shape[dim]
    tp = torch.cat([t, torch.zeros(pad, dtype=t.dtype, device=t.device)], dim) if pad[dim] > 0 else t
    outs = [torch.empty_like(tp) for _ in range(world())]
    _count(tp)
    dist.all_gather(outs, tp.contiguous())
    return torch.cat([o.narrow(dim, 0, int(s.item())) for o, s in zip(outs, sizes)], dim)


def gather_rows(t):
    """All rows of a sharded row tensor (dim 0 for 1-D / [N, K], dim 1 for the [F, N] design matrix is
    the caller's choice): None passes through; a no-op when rows are not sharded."""
    if t is None or not is_dist():
        return t
    return all_gather_cat(t.contiguous(), 0)


def exchange_rows(t: torch.Tensor, dest: torch.Tensor) -> torch.Tensor:
    """Variable-size all-to-all of the rows of ``t`` ([n, ...]): row i goes to rank ``dest[i]``; returns the
    rows this rank received, grouped by source rank (source order kept within a group). Each row moves
    once — the partition step of a distributed sort, not a gather."""
    if not is_dist():
        return t
    if _staged(t):
        return exchange_rows(_stage(t), dest.to(comm_device())).to(t.device)
    W = world()
    order = torch.argsort(dest, stable=True)
    ts = t[order].contiguous()
    send = torch.bincount(dest.long(), minlength=W).to(torch.int64)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    sc, rc = send.tolist(), recv.tolist()
    out = torch.empty((sum(rc),) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    _count(ts)
    dist.all_to_all_single(out, ts, rc, sc)
    return out


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if is_dist():
        _count(t)
        if _staged(t):
            h = _stage(t)
            dist.broadcast(h, src)
            t.copy_(h)
        else:
            dist.broadcast(t, src)
    return t


def agree(flag: bool) -> bool:
    """Rank 0's value of a host-side decision (timers, budgets) on every rank: a rank must never leave a
    loop of collectives alone because its own clock ran out first."""
    if not world_active():
        return bool(flag)
    t = torch.tensor([1.0 if flag else 0.0], dtype=torch.float64, device=comm_device())
    dist.broadcast(t, 0)
    return bool(t.item() > 0)


def barrier():
    if world_active():
        dist.barrier()


def abort_world(reason: str) -> None:
    """Abort the process group: the peers' pending and future collectives fail fast instead of waiting for
    a rank that will never join (a one-sided error inside a sharded build). The job then fails on every rank."""
    from ..utils import log
    log.get().error(f"aborting the process group: {reason}")
    try:
        from torch.distributed.distributed_c10d import _abort_process_group
        _abort_process_group()
    except Exception:  # noqa: BLE001 - older torch: tearing the group down has the same effect on peers
        try:
            dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass


def check_same(value, what: str = "value"):
    """Raise on every rank if ``value`` (picklable) differs between ranks (SPMD divergence guard)."""
    if not world_active():
        return
    vals = all_gather_object(pickle.dumps(value))
    if any(v != vals[0] for v in vals):
        raise RuntimeError(f"ranks disagree on {what}")


# ------------------------------------------------------------------------------------------------
# counter-based per-row random numbers: a row's draw depends on (seed, stream, GLOBAL row index) only,
# so row sampling is identical however the rows are sharded (and equal to the single-process run)
_M = (1 << 64) - 1


def _to_i64(x: int) -> int:
    x &= _M
    return x - (1 << 64) if x >= (1 << 63) else x


def _srl(x: torch.Tensor, k: int) -> torch.Tensor:
    return (x >> k) & ((1 << (64 - k)) - 1)


def row_uniform(seed: int, stream: int, start: int, n: int, device) -> torch.Tensor:
    """float64 uniforms in [0, 1) for global rows ``start .. start+n-1`` (splitmix64 of the index)."""
    base = (int(seed) * 0x9E3779B97F4A7C15 + int(stream) * 0xD1B54A32D192ED03) & _M
    x = torch.arange(start, start + n, dtype=torch.int64, device=device) * _to_i64(0x9E3779B97F4A7C15)
    x = x + _to_i64(base)
    x = (x ^ _srl(x, 30)) * _to_i64(0xBF58476D1CE4E5B9)
    x = (x ^ _srl(x, 27)) * _to_i64(0x94D049BB133111EB)
    x = x ^ _srl(x, 31)
    return _srl(x, 11).double() * (1.0 / (1 << 53))


def row_offset(n_local: int) -> int:
    """Global index of this rank's first row when rows are sharded (0 otherwise)."""
    if not is_dist():
        return 0
    return exclusive_offset(n_local)[0]
