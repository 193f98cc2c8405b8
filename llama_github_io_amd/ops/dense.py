"""Fused dense-layer epilogues for DeepLearning (``csrc/dense_kernels.hip``) as autograd ops.

``BiasAct.apply(x, b, act, drop, seed)`` = act(x + b) with inverted dropout, forward and backward in
one HIP pass each on CUDA tensors; the CPU path is the PyTorch reference of the same math (same
counter-hash dropout mask so CPU/GPU runs agree bit-for-bit on which units drop).
"""
from __future__ import annotations

import os

import torch

from . import _native as nat
from ._native import call, stream_ptr

ACT = {"linear": 0, "rectifier": 1, "relu": 1, "tanh": 2, "exprectifier": 3, "elu": 3}

nat.register_hip_signatures({
    "h2o_bias_act_fwd": [nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_ll, nat.c_int, nat.c_int, nat.ctypes.c_float,
                         nat.c_ull, nat.c_void_p, nat.c_int, nat.c_void_p],
    "h2o_bias_act_bwd": [nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_ll, nat.c_int, nat.c_int,
                         nat.ctypes.c_float, nat.c_ull, nat.c_void_p, nat.c_int, nat.c_void_p],
    "h2o_kmeans_assign": [nat.c_void_p, nat.c_ll, nat.c_int, nat.c_void_p, nat.c_int, nat.c_void_p, nat.c_void_p, nat.c_void_p],
    "h2o_kmeans_step": [nat.c_void_p, nat.c_ll, nat.c_int, nat.c_void_p, nat.c_int, nat.c_void_p, nat.c_void_p,
                        nat.c_void_p, nat.c_void_p, nat.c_void_p],
    "h2o_adadelta": [nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_ll, nat.c_ll, nat.ctypes.c_float,
                     nat.ctypes.c_float, nat.ctypes.c_float, nat.ctypes.c_float, nat.c_void_p, nat.c_void_p, nat.c_int,
                     nat.c_int, nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_int, nat.c_ll,
                     nat.c_void_p, nat.c_void_p, nat.c_void_p],
    "h2o_out_grad": [nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_void_p, nat.c_ll, nat.c_int,
                     nat.c_void_p, nat.c_void_p, nat.c_int, nat.c_void_p],
})


class FlatParams:
    """All parameters (weights first, then biases) and their gradients as views of two flat fp32
    buffers: one fused optimizer launch per step and one flat all-reduce for data parallelism."""

    def __init__(self, module: torch.nn.Module):
        params = list(module.parameters())
        ws = [q for q in params if q.dim() > 1]
        bs = [q for q in params if q.dim() <= 1]
        self.params = ws + bs
        self.n_decay = sum(q.numel() for q in ws)
        n = sum(q.numel() for q in self.params)
        dev = self.params[0].device
        self.p = torch.empty(n, dtype=torch.float32, device=dev)
        self.g = torch.zeros(n, dtype=torch.float32, device=dev)
        o = 0
        with torch.no_grad():
            for q in self.params:
                k = q.numel()
                self.p[o:o + k].copy_(q.reshape(-1))
                q.data = self.p[o:o + k].view_as(q)
                q.grad = self.g[o:o + k].view_as(q)
                o += k
        self.eg2 = torch.zeros_like(self.p)
        self.edx2 = torch.zeros_like(self.p)

    def zero_grad(self):
        self.g.zero_()

    def adadelta(self, rho, eps, l1=0.0, l2=0.0, shadow=None, wt=None):
        """``shadow`` (bf16 [n_decay], optional): also written with the updated weights (the bf16 copies the
        explicit MLP step multiplies with). ``wt``: (tensor, layer offsets, n_in, n_out) — the transposed
        weight copy of the fused DL step, written in the same launch (ops/dl.py FusedMLPStep.wt_map)."""
        if self.p.is_cuda:
            wpp, S, inv_off, ts, tj = 0, 0, 0, 0, 0
            if wt is None:
                wtp, f32, L, o, i, u = 0, 0, 0, 0, 0, 0
            else:
                t, o_, i_, u_ = wt[:4]
                wtp, f32, L = t.data_ptr(), int(t.dtype == torch.float32), len(i_)
                o, i, u = o_.ctypes.data, i_.ctypes.data, u_.ctypes.data     # host arrays, copied at launch
                if len(wt) > 4:       # weight gradients from the fused step's split partials
                    wpp, S, inv_off = wt[4].data_ptr(), int(wt[5]), int(wt[6])
                    ts, tj = wt[7].ctypes.data, wt[8].ctypes.data
            call("h2o_adadelta", self.p.data_ptr(), self.g.data_ptr(), self.eg2.data_ptr(), self.edx2.data_ptr(),
                 self.p.numel(), self.n_decay, float(rho), float(eps), float(l1), float(l2),
                 0 if shadow is None else shadow.data_ptr(), wtp, f32, L, o, i, u, wpp, S, inv_off, ts, tj,
                 stream_ptr(self.p.device))
            return
        g = self.g.clone()
        w = slice(0, self.n_decay)
        g[w] += l2 * self.p[w] + l1 * torch.sign(self.p[w])
        self.eg2.mul_(rho).addcmul_(g, g, value=1 - rho)
        d = -torch.sqrt(self.edx2 + eps) / torch.sqrt(self.eg2 + eps) * g
        self.edx2.mul_(rho).addcmul_(d, d, value=1 - rho)
        self.p.add_(d)
        if shadow is not None:
            shadow.copy_(self.p[: self.n_decay])

_M = (1 << 64) - 1
_GOLD = 0x9E3779B97F4A7C15


def step_seed(seed: int, step: int) -> int:
    """Dropout seed of one training step: ``seed ^ step * golden`` (mod 2^64), the same mixing the kernels
    apply to a device-resident step counter (``seed_dev``) so graph replays draw fresh masks."""
    return (int(seed) ^ (int(step) * _GOLD)) & _M


def _mask_ref(shape, drop, seed, device):
    n = shape[0] * shape[1]
    i = torch.arange(n, dtype=torch.int64, device=device)
    # same 64-bit mixing as hash32() in the kernel, computed with wrap-around int64 arithmetic
    x = torch.bitwise_xor(torch.tensor(seed if seed < (1 << 63) else seed - (1 << 64), dtype=torch.int64),
                          i * torch.tensor(0x9E3779B97F4A7C15 - (1 << 64), dtype=torch.int64))

    def srl(v, k):
        return torch.bitwise_and(torch.bitwise_right_shift(v, k), (1 << (64 - k)) - 1)
    x = torch.bitwise_xor(x, srl(x, 33)); x = x * torch.tensor(0xff51afd7ed558ccd - (1 << 64), dtype=torch.int64)
    x = torch.bitwise_xor(x, srl(x, 33)); x = x * torch.tensor(0xc4ceb9fe1a85ec53 - (1 << 64), dtype=torch.int64)
    x = torch.bitwise_xor(x, srl(x, 33))
    h = torch.bitwise_and(x, 0xFFFFFFFF)
    thr = int(drop * 4294967296.0)
    return (h >= thr).reshape(shape)


def _act(a, v):
    if a == 1:
        return torch.relu(v)
    if a == 2:
        return torch.tanh(v)
    if a == 3:
        return torch.where(v > 0, v, torch.expm1(v))
    return v


def bias_act_fwd(x, b, act: int, drop: float, seed: int, seed_dev=None):
    """y = act(x + b) with inverted dropout (no autograd). CUDA: one HIP pass, bf16 in -> bf16 out."""
    x = x.contiguous()
    rows, cols = x.shape
    if x.is_cuda:
        if x.dtype not in (torch.float32, torch.bfloat16):
            x = x.float()
        y = torch.empty_like(x)
        bb = None if b is None else b.float().contiguous()
        nat.call("h2o_bias_act_fwd", x.data_ptr(), 0 if bb is None else bb.data_ptr(), y.data_ptr(), rows, cols,
                 act, float(drop), seed & _M, 0 if seed_dev is None else seed_dev.data_ptr(),
                 int(x.dtype == torch.bfloat16), nat.stream_ptr(x.device))
        return y
    if seed_dev is not None:
        seed = step_seed(seed, int(seed_dev.item()))
    y = _act(act, x + (b if b is not None else 0))
    if drop > 0:
        y = torch.where(_mask_ref(y.shape, drop, seed, y.device), y / (1 - drop), torch.zeros_like(y))
    return y


def bias_act_bwd(gy, y, act: int, drop: float, seed: int, seed_dev=None, db=None):
    """gx = gy * mask * act'(y); the bias gradient Σ_rows gx is ADDED into ``db`` (fp32) when given."""
    gy = gy.contiguous()
    rows, cols = y.shape
    if y.is_cuda:
        gy = gy.to(y.dtype).contiguous()
        gx = torch.empty_like(y)
        nat.call("h2o_bias_act_bwd", gy.data_ptr(), y.data_ptr(), gx.data_ptr(), 0 if db is None else db.data_ptr(),
                 rows, cols, act, float(drop), seed & _M, 0 if seed_dev is None else seed_dev.data_ptr(),
                 int(y.dtype == torch.bfloat16), nat.stream_ptr(y.device))
        return gx
    if seed_dev is not None:
        seed = step_seed(seed, int(seed_dev.item()))
    yy, g = y, gy
    if drop > 0:
        m = _mask_ref(y.shape, drop, seed, y.device)
        g = torch.where(m, gy / (1 - drop), torch.zeros_like(gy))
        yy = torch.where(m, y * (1 - drop), torch.zeros_like(y))
    if act == 1:
        d = (yy > 0).to(y.dtype)
    elif act == 2:
        d = 1 - yy * yy
    elif act == 3:
        d = torch.where(yy > 0, torch.ones_like(yy), yy + 1)
    else:
        d = torch.ones_like(yy)
    gx = g * d
    if db is not None:
        db += gx.sum(0).to(db.dtype)
    return gx


class BiasAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, b, act: int, drop: float, seed: int, seed_dev=None):
        y = bias_act_fwd(x, b, act, drop, seed, seed_dev)
        ctx.save_for_backward(y)
        ctx.act, ctx.drop, ctx.seed, ctx.has_b, ctx.seed_dev = act, drop, seed, b is not None, seed_dev
        return y

    @staticmethod
    def backward(ctx, gy):
        (y,) = ctx.saved_tensors
        db = torch.zeros(y.shape[1], dtype=torch.float32, device=y.device) if ctx.has_b else None
        gx = bias_act_bwd(gy, y, ctx.act, ctx.drop, ctx.seed, ctx.seed_dev, db)
        return gx, db, None, None, None, None


def out_grad(logits, ycls, yreg, w, inv, db):
    """Logit gradient of the output layer (softmax cross-entropy when ``ycls`` is given, squared error on
    ``yreg`` otherwise), scaled by ``w * inv``; adds Σ_rows into ``db`` (fp32). One HIP pass on the GPU."""
    rows, K = logits.shape
    if logits.is_cuda:
        dO = torch.empty_like(logits)
        nat.call("h2o_out_grad", logits.data_ptr(), 0 if ycls is None else ycls.data_ptr(),
                 0 if yreg is None else yreg.data_ptr(), w.data_ptr(), inv.data_ptr(), rows, K, dO.data_ptr(),
                 db.data_ptr(), int(logits.dtype == torch.bfloat16), nat.stream_ptr(logits.device))
        return dO
    o = logits.float()
    s = (w.float() * inv.float())[:, None]
    if ycls is not None:
        g = (torch.softmax(o, 1) - torch.nn.functional.one_hot(ycls.long(), K).float()) * s
    else:
        g = (o - yreg.float()[:, None]) * s
    db += g.sum(0)
    return g.to(logits.dtype)


def bias_act(x, b, act: str | int = "rectifier", drop: float = 0.0, seed: int = 0, seed_dev=None):
    """``seed_dev`` (CUDA int64 [1], optional): per-step counter read by the kernels and mixed into ``seed``
    (``step_seed``), so a captured hipGraph draws a new dropout mask on every replay."""
    a = ACT[act.lower()] if isinstance(act, str) else int(act)
    return BiasAct.apply(x, b, a, float(drop), int(seed), seed_dev)


def _mfma_shape(K, P):
    import ctypes
    out = (ctypes.c_int * 3)()
    ok = nat.hip().h2o_kmeans_mfma_shape(int(K), int(P), out)
    return (out[0], out[1], out[2]) if ok else None


_KM_GRID: dict = {}     # (K, P) -> blocks of one resident round of the MFMA Lloyd kernel (occupancy query, cached)


def kmeans_step(X: torch.Tensor, C: torch.Tensor, w: torch.Tensor | None = None, need_assign: bool = True):
    """One Lloyd step: (assign [N], min sq. distance [N], per-center weighted sums [K, P] fp64, counts [K]).
    ``need_assign=False`` (the Lloyd loop, which reads only distances, sums and counts): the MFMA kernel does not
    store assignments and None is returned in their place.
    On the GPU: ``csrc/kmeans_mfma.hip`` (distance GEMM + argmin + one-hot centroid GEMM on f32 MFMA,
    one pass over X) for K, P <= 64 with P % 4 == 0 (KMeans pads its design matrix); the LDS scalar
    kernel otherwise."""
    N, P = X.shape
    K = C.shape[0]
    sh = _mfma_shape(K, P) if X.is_cuda and N > 0 and P % 4 == 0 else None
    if sh is not None and os.environ.get("H2O_KMEANS_MFMA", "1") == "1":
        KT, PS, PT = sh
        X = X.contiguous().float()
        C = C.contiguous().float()
        wf = None if w is None else w.contiguous().float()
        a = torch.empty(N, dtype=torch.int32, device=X.device) if need_assign else None
        d = torch.empty(N, dtype=torch.float32, device=X.device)
        key = (int(K), int(P))
        full = _KM_GRID.get(key)
        if full is None:
            full = _KM_GRID[key] = int(nat.hip().h2o_kmeans_mfma_grid(*key)) or 1024   # one resident round
        grid = int(max(1, min(full, (N + 63) // 64)))
        slab = torch.empty(grid, KT * 16, PT * 16, dtype=torch.float32, device=X.device)   # one per block
        nat.call("h2o_kmeans_mfma", X.data_ptr(), N, P, C.data_ptr(), K, 0 if wf is None else wf.data_ptr(),
                 0 if a is None else a.data_ptr(), d.data_ptr(), slab.data_ptr(), grid, nat.stream_ptr(X.device))
        tot = slab.sum(0, dtype=torch.float64)
        return (a.long() if a is not None else None), d, tot[:K, :P].contiguous(), tot[:K, P].contiguous()
    if X.is_cuda and (K * P + 256 * (P + 1) + 512) * 4 <= 160 * 1024 and N > 0 and K * (P + 1) <= 8192:
        X = X.contiguous().float()
        C = C.contiguous().float()
        wf = None if w is None else w.contiguous().float()
        a = torch.empty(N, dtype=torch.int32, device=X.device)
        d = torch.empty(N, dtype=torch.float32, device=X.device)
        G = (N + 255) // 256
        slab = torch.empty(G, K, P + 1, dtype=torch.float32, device=X.device)
        nat.call("h2o_kmeans_step", X.data_ptr(), N, P, C.data_ptr(), K, 0 if wf is None else wf.data_ptr(),
                 a.data_ptr(), d.data_ptr(), slab.data_ptr(), nat.stream_ptr(X.device))
        tot = slab.sum(0, dtype=torch.float64)
        return a.long(), d, tot[:, :P], tot[:, P]
    a, d = kmeans_assign(X, C)
    wd = torch.ones(N, dtype=torch.float64, device=X.device) if w is None else w.double()
    # sort-based segment sums (no contended atomics)
    order = torch.argsort(a)
    cnt = torch.bincount(a, weights=wd, minlength=K)
    nrows = torch.bincount(a, minlength=K)
    cs = torch.cumsum(X.double()[order] * wd[order, None], 0)
    cs = torch.cat([torch.zeros(1, P, dtype=torch.float64, device=X.device), cs], 0)
    ends = torch.cumsum(nrows, 0)
    sums = cs[ends] - cs[ends - nrows]
    return a, d, sums, cnt


def kmeans_lloyd_step(X: torch.Tensor, C: torch.Tensor, w: torch.Tensor | None = None):
    """One single-process Lloyd iteration on the MFMA kernel plus the fused center update (k_kmeans_update):
    (min sq. distance [N], new centers [K, P] f32, counts [K] f64, flags [#empty, max shift] f64) — or None where the
    MFMA shape does not apply (the caller runs kmeans_step + its torch update)."""
    N, P = X.shape
    K = C.shape[0]
    sh = _mfma_shape(K, P) if X.is_cuda and N > 0 and P % 4 == 0 else None
    if sh is None or os.environ.get("H2O_KMEANS_MFMA", "1") != "1":
        return None
    KT, PS, PT = sh
    X = X.contiguous().float()
    Cf = C.contiguous().float()
    wf = None if w is None else w.contiguous().float()
    d = torch.empty(N, dtype=torch.float32, device=X.device)
    key = (int(K), int(P))
    full = _KM_GRID.get(key)
    if full is None:
        full = _KM_GRID[key] = int(nat.hip().h2o_kmeans_mfma_grid(*key)) or 1024
    grid = int(max(1, min(full, (N + 63) // 64)))
    slab = torch.empty(grid, KT * 16, PT * 16, dtype=torch.float32, device=X.device)
    s = nat.stream_ptr(X.device)
    nat.call("h2o_kmeans_mfma", X.data_ptr(), N, P, Cf.data_ptr(), K, 0 if wf is None else wf.data_ptr(), 0,
             d.data_ptr(), slab.data_ptr(), grid, s)
    tot = slab.sum(0, dtype=torch.float64)
    newC = torch.empty(K, P, dtype=torch.float32, device=X.device)
    cnt = torch.empty(K, dtype=torch.float64, device=X.device)
    flags = torch.empty(2, dtype=torch.float64, device=X.device)
    nat.call("h2o_kmeans_update", tot.data_ptr(), PT * 16, K, P, Cf.data_ptr(), newC.data_ptr(), cnt.data_ptr(),
             flags.data_ptr(), s)
    return d, newC, cnt, flags


def kmeans_assign(X: torch.Tensor, C: torch.Tensor):
    """Closest center and squared distance for every row. X [N, P], C [K, P] float32."""
    N, P = X.shape
    K = C.shape[0]
    if X.is_cuda and (K * P + 256 * (P + 1)) * 4 <= 160 * 1024 and N > 0:
        X = X.contiguous().float()
        C = C.contiguous().float()
        a = torch.empty(N, dtype=torch.int32, device=X.device)
        d = torch.empty(N, dtype=torch.float32, device=X.device)
        nat.call("h2o_kmeans_assign", X.data_ptr(), N, P, C.data_ptr(), K, a.data_ptr(), d.data_ptr(), nat.stream_ptr(X.device))
        return a.long(), d
    # reference / wide path: ||x||² - 2 x·c + ||c||² via one GEMM
    Xd, Cd = X.double(), C.double()
    D = (Xd * Xd).sum(1, keepdim=True) - 2 * Xd @ Cd.T + (Cd * Cd).sum(1)[None, :]
    d, a = D.clamp(min=0).min(1)
    return a, d.float()
