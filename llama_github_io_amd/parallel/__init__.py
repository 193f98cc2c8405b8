"""Multi-GPU execution: one process per GPU, torch.distributed over RCCL (xGMI) / gloo (CPU tests)."""
