"""Fused MFMA training step of the DeepLearning MLP (``csrc/dl_kernels.hip``).

Reference: ``hex/deeplearning/Neurons.java`` fprop / bprop (``DeepLearningTask.map``). One step is
``k_dl_rows`` (gather + every layer forward + loss gradient + every layer backward on 16-row tiles, activations
in LDS) -> ``k_dl_wgrad`` (all weight gradients, split over the batch rows inside a workgroup and summed in a
fixed order, plus the bias gradients from the row tiles' partials) straight into the flat gradient buffer;
the optimizer (fused ADADELTA) then refreshes the bf16 weight shadow (bf16 operands; fp32 operands read the
master weights in place) and :meth:`FusedMLPStep.refresh_transposed` the transposed copy of the backward pass.
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import _native as nat

MAXL = 6
ROWS = 16
MAXK = 256          # output classes of the fused step (K > 16: fp32 [16][K] logit tile in LDS)
_vp, _ci, _cll, _cf, _cull = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float, ctypes.c_ulonglong


class _DLArgs(ctypes.Structure):
    """Mirror of ``DLArgs`` in ``csrc/dl_kernels.hip``."""
    _fields_ = ([("Z", _vp), ("ldz", _cll), ("ridx", _vp), ("B", _ci), ("Bpad", _ci),
                 ("w", _vp), ("ycls", _vp), ("yreg", _vp),
                 ("P", _vp), ("W", _vp), ("WT", _vp), ("step_dev", _vp),
                 ("hT", _vp), ("dT", _vp), ("bpart", _vp), ("g", _vp), ("gsum", _vp),
                 ("L", _ci), ("K", _ci), ("act", _ci), ("regression", _ci),
                 ("n", _ci * (MAXL + 1)), ("kp", _ci * (MAXL + 1)), ("ld", _ci * (MAXL + 1)),
                 ("w_off", _cll * MAXL), ("b_off", _cll * MAXL),
                 ("h_off", _cll * (MAXL + 1)), ("d_off", _cll * (MAXL + 1)),
                 ("bias_off", _ci * (MAXL + 1)), ("bias_total", _ci),
                 ("drop", _cf * MAXL), ("seed_base", _cull * MAXL),
                 ("lds_off", _ci * (MAXL + 1)), ("lds_g", _ci * 2), ("lds_w", _ci),
                 ("tiles_i", _ci * MAXL), ("tiles_j", _ci * MAXL), ("tile_start", _ci * (MAXL + 1)),
                 ("n_decay", _cll), ("n_total", _cll), ("f32", _ci), ("pad_", _ci),
                 ("in_drop", _cf), ("lds_lg", _ci), ("in_seed", _cull),
                 ("wsplit", _ci), ("maxout", _ci), ("ng", _ci * (MAXL + 1)), ("kpg", _ci * (MAXL + 1)),
                 ("ldg", _ci * (MAXL + 1)), ("lds_mx", _ci * MAXL), ("ae", _ci), ("no_wsum", _ci),
                 ("wpart", _vp)])


nat.register_hip_signatures({"h2o_dl_args_size": [], "h2o_dl_step": [_vp, _ci, _ci, _vp],
                             "h2o_dl_transpose": [_vp, _vp]})


def _r32(n: int) -> int:
    return (n + 31) // 32 * 32


def _pad(esz: int) -> int:
    """LDS row padding (elements) of the activation tiles: 16 bytes (spreads rows over the banks)."""
    return 16 // esz


def supported(n_in: int, hidden, n_out: int, act_code: int, Z: torch.Tensor, maxout: bool = False) -> bool:
    """Shapes the fused step handles (else the library-GEMM explicit step runs): bf16 or fp32 operands."""
    L = len(hidden) + 1
    if not Z.is_cuda or Z.dtype not in (torch.bfloat16, torch.float32) or L > MAXL or n_out > MAXK or \
            act_code not in (0, 1, 2, 3):
        return False
    esz = Z.element_size()
    pd = _pad(esz)
    widths = [n_in] + list(hidden)
    gw = max([(2 if maxout else 1) * h for h in hidden] or [1])
    lds = (sum(ROWS * (_r32(n) + pd) * esz for n in widths) + ROWS * (_r32(n_out) + pd) * esz
           + 2 * ROWS * (_r32(gw) + pd) * esz + 64 + (ROWS * n_out * 4 if n_out > 16 else 0)
           + (ROWS * sum(hidden) + 16 * L if maxout else 0))
    return lds <= 150 * 1024 and max(widths) <= 8192


class FusedMLPStep:
    """Static launch arguments of the fused step for one network / mini-batch capacity.

    ``lins``: the hidden Linear layers then the output layer (weights ``[out, in]`` views of the flat
    fp32 buffer ``fp.p``); ``shadow``: bf16 copy of ``fp.p[:n_decay]`` kept by the optimizer, or None: fp32
    operands (``Z`` fp32, the master weights read in place, fp32 transposed copies and LDS tiles)."""

    def __init__(self, fp, lins, act_code: int, drops, seed_bases, Z: torch.Tensor, w: torch.Tensor, y: torch.Tensor,
                 regression: bool, cap: int, shadow: torch.Tensor, step_dev: torch.Tensor, out_grad: torch.Tensor,
                 out_gsum: torch.Tensor | None, in_drop: float = 0.0, in_seed: int = 0, maxout: bool = False,
                 autoencoder: bool = False):
        self.lib = nat.hip()
        assert self.lib.h2o_dl_args_size() == ctypes.sizeof(_DLArgs), "DLArgs layout mismatch"
        dev = Z.device
        L = len(lins)
        # n: activation widths; ng: GEMM output widths (Maxout hidden layers hold 2 channels of n[l] rows each)
        ng = [lins[0].weight.shape[1]] + [l_.weight.shape[0] for l_ in lins]
        n = [ng[0]] + [(g // 2 if (maxout and l < L - 1) else g) for l, g in enumerate(ng[1:])]
        Bpad = (cap + ROWS * 8 - 1) // (ROWS * 8) * (ROWS * 8)      # multiple of 128
        base = fp.p.data_ptr()
        esz = fp.p.element_size()
        a = _DLArgs()
        a.Z, a.ldz, a.B, a.Bpad = Z.data_ptr(), Z.stride(0), int(cap), int(Bpad)
        a.w = w.data_ptr()
        if autoencoder:               # the targets are the input rows themselves
            a.ycls, a.yreg, a.regression, a.ae = 0, 0, 1, 1
        elif regression:
            a.yreg, a.ycls, a.regression = y.data_ptr(), 0, 1
        else:
            a.ycls, a.yreg, a.regression = y.data_ptr(), 0, 0
        f32 = shadow is None
        assert Z.dtype == (torch.float32 if f32 else torch.bfloat16)
        cdt = torch.float32 if f32 else torch.bfloat16
        cesz = 4 if f32 else 2
        wsrc = fp.p[: fp.n_decay] if f32 else shadow
        self.WT = torch.empty_like(wsrc)
        a.P, a.W, a.WT, a.step_dev = base, wsrc.data_ptr(), self.WT.data_ptr(), step_dev.data_ptr()
        a.f32 = int(f32)
        a.L, a.K, a.act = L, n[L], int(act_code)
        for i, v in enumerate(n):
            a.n[i] = v
            a.kp[i] = _r32(v)
            a.ld[i] = _r32(v) + _pad(cesz)
            a.ng[i] = ng[i]
            a.kpg[i] = _r32(ng[i])
            a.ldg[i] = _r32(ng[i]) + _pad(cesz)
        a.maxout = int(bool(maxout))
        bias_off, bt = [0] * (MAXL + 1), 0
        for l in range(1, L + 1):
            bias_off[l] = bt
            bt += ng[l]
        for l, lin in enumerate(lins):
            a.w_off[l] = (lin.weight.data_ptr() - base) // esz
            a.b_off[l] = (lin.bias.data_ptr() - base) // esz
            assert a.b_off[l] >= fp.n_decay and a.w_off[l] < fp.n_decay
        for l in range(L + 1):
            a.bias_off[l] = bias_off[l]
        a.bias_total = bt
        for i in range(L - 1):
            a.drop[i] = float(drops[i])
            a.seed_base[i] = int(seed_bases[i]) & ((1 << 64) - 1)
        # transposed activations / gradients: [units][Bpad] per layer (offsets multiples of 8 elements)
        ho, o = [], 0
        for l in range(L):
            ho.append(o)
            o += n[l] * Bpad
        do = [0]
        for l in range(1, L + 1):
            do.append(o)
            o += ng[l] * Bpad
        self.T = torch.zeros(o, dtype=cdt, device=dev)
        for l in range(L):
            a.h_off[l] = ho[l]
        for l in range(1, L + 1):
            a.d_off[l] = do[l]
        a.hT = a.dT = self.T.data_ptr()
        G1 = Bpad // ROWS
        self.bpart = torch.zeros(G1 * (bt + 1), dtype=torch.float32, device=dev)
        a.bpart = self.bpart.data_ptr()
        a.g = out_grad.data_ptr()
        a.gsum = 0 if out_gsum is None else out_gsum.data_ptr()
        # LDS: activation tiles 0..L-1, output-gradient tile, two gradient tiles, row weights (16-B aligned)
        off = 0
        for l in range(L):
            a.lds_off[l] = off
            off += ROWS * a.ld[l]
        a.lds_off[L] = off
        off += ROWS * a.ld[L]
        gl = max([a.ldg[l] for l in range(1, L)] or [8])
        a.lds_g[0], a.lds_g[1] = off, off + ROWS * gl
        off += 2 * ROWS * gl
        a.lds_w = off * cesz
        self.lds = a.lds_w + ROWS * 4
        if maxout:                     # winning-channel bytes of every hidden layer
            for l in range(1, L):
                a.lds_mx[l] = self.lds
                self.lds += (ROWS * n[l] + 15) // 16 * 16
        if n[L] > 16:                  # fp32 [16][K] logits of the wide softmax (16-byte aligned)
            assert (autoencoder or not regression) and n[L] <= MAXK
            a.lds_lg = (self.lds + 15) // 16 * 16
            self.lds = a.lds_lg + ROWS * n[L] * 4
        a.in_drop = float(in_drop)
        a.in_seed = int(in_seed) & ((1 << 64) - 1)
        ts = 0
        for l in range(L):
            a.tiles_i[l] = (ng[l + 1] + 63) // 64
            a.tiles_j[l] = (n[l] + 63) // 64
            a.tile_start[l] = ts
            ts += a.tiles_i[l] * a.tiles_j[l]
        a.tile_start[L] = ts
        # weight-gradient GEMM: 64 x 64 tiles x `wsplit` batch-row ranges (~768 workgroups of 4 waves) into fp32
        # partial tiles, summed in split order by k_dl_wsum
        nch = Bpad // (16 if f32 else 32)
        a.wsplit = max(1, min(nch // 4, -(-768 // ts)))
        if os.environ.get("H2O_DL_WSPLIT"):            # A/B: fewer splits = fewer partial bytes, less parallelism
            a.wsplit = max(1, min(nch // 4, int(os.environ["H2O_DL_WSPLIT"])))
        self.wpart = torch.empty(ts * a.wsplit * 4096 + 1, dtype=torch.float32, device=dev)
        a.wpart = self.wpart.data_ptr()
        a.n_decay, a.n_total = fp.n_decay, fp.p.numel()
        self.args = a
        self.scale_by_w = out_gsum is None
        # the optimizer writes WT in its own launch (FlatParams.adadelta(wt=...)): host arrays of layer shapes
        import numpy as _np
        self.wt_map = (self.WT, _np.ascontiguousarray([a.w_off[l] for l in range(L)] + [fp.n_decay], dtype=_np.int64),
                       _np.ascontiguousarray(n[:L], dtype=_np.int32),
                       _np.ascontiguousarray(ng[1:L + 1], dtype=_np.int32))
        self._tile_start = _np.ascontiguousarray([a.tile_start[l] for l in range(L + 1)], dtype=_np.int32)
        self._tiles_j = _np.ascontiguousarray([a.tiles_j[l] for l in range(L)], dtype=_np.int32)
        self._keep = (Z, w, y, wsrc, step_dev, out_grad, out_gsum)

    def optimizer_reads_partials(self) -> tuple:
        """Skip the split-sum launch: the fused ADADELTA update sums the weight-gradient partials itself (the
        weight part of the gradient buffer is then never written). Returns the optimizer's ``wt`` argument."""
        self.args.no_wsum = 1
        a = self.args
        return self.wt_map + (self.wpart, int(a.wsplit), int(a.tile_start[a.L]) * int(a.wsplit) * 4096,
                              self._tile_start, self._tiles_j)

    def step(self, ridx: torch.Tensor) -> None:
        """One forward/backward of the rows ``ridx`` (int64; -1 = padding row) into the gradient buffer."""
        a = self.args
        a.ridx = ridx.data_ptr()
        a.B = int(ridx.numel())
        nat.check(self.lib.h2o_dl_step(ctypes.byref(a), self.lds, int(self.scale_by_w), nat.stream_ptr(ridx.device)),
                  "dl_step")

    def refresh_transposed(self) -> None:
        nat.check(self.lib.h2o_dl_transpose(ctypes.byref(self.args), nat.stream_ptr(self.T.device)), "dl_transpose")
