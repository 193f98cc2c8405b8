"""RCCL probe on a 1-GPU box: 2 ranks on cuda:0 over the nccl (= RCCL) backend run the tree engine's
collectives (all-reduce, reduce-scatter, all-gather) and check the results. RCCL may refuse two ranks on
one device; the script then prints the error (exit 3) instead of hanging."""
import os
import sys

import torch
import torch.distributed as dist


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    try:
        dist.init_process_group("nccl", device_id=dev)
        x = torch.full((1 << 20,), float(rank + 1), device=dev, dtype=torch.float64)
        dist.all_reduce(x)
        ok = bool((x == world * (world + 1) / 2).all())
        rs_in = torch.arange(world * 1024, device=dev, dtype=torch.int64)
        rs = torch.empty(1024, device=dev, dtype=torch.int64)
        dist.reduce_scatter_tensor(rs, rs_in)
        ok &= bool((rs == world * torch.arange(rank * 1024, (rank + 1) * 1024, device=dev)).all())
        ag = torch.empty(world * 16, device=dev, dtype=torch.float32)
        dist.all_gather_into_tensor(ag, torch.full((16,), float(rank), device=dev))
        ok &= bool((ag.view(world, 16)[:, 0] == torch.arange(world, device=dev)).all())
        torch.cuda.synchronize()
        print(f"rank {rank}: RCCL collectives ok={ok}", flush=True)
        dist.destroy_process_group()
        sys.exit(0 if ok else 1)
    except Exception as e:  # noqa: BLE001 - report RCCL's refusal
        print(f"rank {rank}: RCCL error: {type(e).__name__}: {e}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
