"""Collectives used by the distributed algorithms (the MI355X replacement of ``water/MRTask.java``'s
reduce tree): thin helpers over ``torch.distributed`` that are no-ops in a single process."""
from __future__ import annotations

import torch
import torch.distributed as dist


def is_dist() -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world() -> int:
    return dist.get_world_size() if is_dist() else 1


def rank() -> int:
    return dist.get_rank() if is_dist() else 0


def _staged(t: torch.Tensor) -> bool:
    """gloo cannot run every collective on device tensors: stage those through host memory."""
    return t.is_cuda and dist.get_backend() != "nccl"


def all_reduce_(t: torch.Tensor, op=None) -> torch.Tensor:
    if is_dist():
        from ..utils import timeline
        timeline.record("collective", "all_reduce", bytes=t.numel() * t.element_size())
        if _staged(t):
            h = t.detach().cpu()
            dist.all_reduce(h, op=op or dist.ReduceOp.SUM)
            t.copy_(h)
        else:
            dist.all_reduce(t, op=op or dist.ReduceOp.SUM)
    return t


def all_reduce_sum(t: torch.Tensor) -> torch.Tensor:
    return all_reduce_(t)


def comm_device() -> torch.device:
    """Device collectives must use: the rank's GPU under RCCL ('nccl'), the CPU under gloo."""
    if is_dist() and dist.get_backend() == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def all_reduce_scalar(x: float, device=None) -> float:
    if not is_dist():
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device or comm_device())
    dist.all_reduce(t)
    return float(t.item())


def all_gather_cat(t: torch.Tensor, dim: int = 0) -> torch.Tensor:
    if not is_dist():
        return t
    if _staged(t):
        return all_gather_cat(t.cpu(), dim).to(t.device)
    n = torch.tensor([t.shape[dim]], device=t.device)
    sizes = [torch.zeros_like(n) for _ in range(world())]
    dist.all_gather(sizes, n)
    mx = int(max(s.item() for s in sizes))
    pad = list(t.shape)
    pad[dim] = mx - t.shape[dim]
    tp = torch.cat([t, torch.zeros(pad, dtype=t.dtype, device=t.device)], dim) if pad[dim] > 0 else t
    outs = [torch.empty_like(tp) for _ in range(world())]
    dist.all_gather(outs, tp.contiguous())
    return torch.cat([o.narrow(dim, 0, int(s.item())) for o, s in zip(outs, sizes)], dim)


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if is_dist():
        if _staged(t):
            h = t.detach().cpu()
            dist.broadcast(h, src)
            t.copy_(h)
        else:
            dist.broadcast(t, src)
    return t


def barrier():
    if is_dist():
        dist.barrier()
