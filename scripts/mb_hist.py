"""Micro-benchmark of the root histogram kernel under different bin distributions."""
import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from llama_github_io_amd.ops import tree as T, _native as nat

dev = torch.device("cuda", 0)
N, F = 11_000_000, 28
stride = 28
aux = torch.rand(N, 4, device=dev)
aux[:, 0] = 1.0
p = T.SplitParams(min_w=10)


def run(bins, label, reps=5):
    b = T.GpuTreeBuilder(bins, F, np.full(F, 255, np.int32), np.zeros(F, np.int32), None, 2, p)
    lib = b.lib
    s = nat.stream_ptr(dev)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    amax = aux[:, :2].abs().amax(0).double()
    b.qs[:2] = 2.0 ** 40 / amax
    b.qs[2:] = amax / 2.0 ** 40
    for grid in (128, 256, 512):
        ts = []
        for r in range(reps):
            b.hist[0][: b.slot].zero_()
            ev0.record()
            nat.check(lib.h2o_hist_build(bins.data_ptr(), stride, aux.data_ptr(), b._p("nodes0"), b._p("tp0"),
                                         b._p("meta0"), F, b.hist[0].data_ptr(), b.slot, b.qs.data_ptr(), grid, 0, 0, 0, 0, s), "hb")
            ev1.record()
            torch.cuda.synchronize()
            ts.append(ev0.elapsed_time(ev1))
        print(f"{label:28s} grid={grid:5d}  {min(ts):8.3f} ms  ({N * F / min(ts) / 1e6:.1f} G bin-updates/s)", flush=True)
    # correctness of the total count
    h = b.hist[0][: F * 512].view(F, 256, 2)
    print("   sum w per feature ok:", bool(torch.allclose(h[:, :, 0].sum(1), torch.full((F,), float(N), dtype=torch.float64, device=dev))))
    ref = torch.zeros(256, dtype=torch.float64, device=dev).index_add_(0, bins[:, 5].long(), aux[:, 1].double())
    print("   wY feature 5 max abs err vs fp64 reference:", float((h[5, :, 1] - ref).abs().max()))


g = torch.Generator(device=dev).manual_seed(0)
run(torch.randint(0, 255, (N, stride), device=dev, generator=g, dtype=torch.uint8), "uniform random 255 bins")
run(torch.randint(0, 4, (N, stride), device=dev, generator=g, dtype=torch.uint8), "4 distinct bins")
run(torch.zeros(N, stride, device=dev, dtype=torch.uint8), "all same bin")
