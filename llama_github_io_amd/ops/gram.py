"""Weighted Gram / cross-product ops (GLM GramTask, PCA GramSVD, covariance).

CUDA(HIP) tensors run ``csrc/gram_kernels.hip`` (f32-input MFMA tiles, per-slice fp32 slabs summed
in fp64); CPU tensors use the fp64 PyTorch reference (the test oracle).
"""
from __future__ import annotations

import os

import torch

from . import _native as nat

nat.register_hip_signatures({
    "h2o_gram": [nat.c_void_p, nat.c_ll, nat.c_void_p, nat.c_void_p, nat.c_ll, nat.c_int, nat.c_int, nat.c_void_p,
                 nat.c_int, nat.c_void_p],
    "h2o_xtv": [nat.c_void_p, nat.c_ll, nat.c_void_p, nat.c_int, nat.c_ll, nat.c_int, nat.c_int, nat.c_void_p, nat.c_void_p],
    "h2o_zbeta": [nat.c_void_p, nat.c_ll, nat.c_void_p, nat.c_int, nat.c_ll, nat.c_int, nat.c_void_p, nat.c_void_p,
                  nat.c_void_p],
    "h2o_irls_wz": [nat.c_void_p, nat.c_ll, nat.c_void_p, nat.c_ll, nat.c_int, nat.c_void_p, nat.c_void_p, nat.c_void_p,
                    nat.c_int, nat.c_int, nat.c_void_p, nat.c_void_p, nat.c_void_p],
    "h2o_gram_irls": [nat.c_void_p, nat.c_ll, nat.c_void_p, nat.c_ll, nat.c_int, nat.c_void_p, nat.c_void_p,
                      nat.c_void_p, nat.c_int, nat.c_int, nat.c_int, nat.c_void_p, nat.c_void_p],
})

# glm.Family -> the k_zbeta IRLS epilogue's codes (csrc/gram_kernels.hip IrlsOut)
_IRLS_FAM = {"gaussian": 0, "binomial": 1, "quasibinomial": 1, "fractionalbinomial": 1, "poisson": 2, "gamma": 3}
_IRLS_LINK = {"identity": 0, "logit": 1, "log": 2, "inverse": 3}


def irls_wz(Z: torch.Tensor, beta: torch.Tensor, off, y: torch.Tensor, w: torch.Tensor, family: str, link: str):
    """IRLS working weights and response of one iteration, fp32 [N] each, in the z.beta pass (one HIP launch:
    eta = Z beta + off, mu, g'(mu), V(mu) per row) — or None where the family / link / device is not covered and
    the caller keeps the torch chain. Same formulas and clamps as ``glm.Family``."""
    if (not Z.is_cuda or family not in _IRLS_FAM or link not in _IRLS_LINK or beta.dim() != 1
            or Z.shape[1] > 3072 or os.environ.get("H2O_GLM_FUSED_IRLS", "1") == "0"):
        return None
    N, P = Z.shape
    Z = Z.contiguous()
    od = None
    if off is not None:
        od = (off if torch.is_tensor(off) else torch.full((N,), float(off), device=Z.device)).double()
        od = (od.expand(N) if od.numel() == 1 else od).contiguous()
    yd, wd = y.contiguous().double(), w.contiguous().double()
    wi = torch.empty(N, dtype=torch.float32, device=Z.device)
    zi = torch.empty(N, dtype=torch.float32, device=Z.device)
    if N > 0:
        nat.call("h2o_irls_wz", Z.data_ptr(), P, beta.contiguous().double().data_ptr(), N, P,
                 0 if od is None else od.data_ptr(), yd.data_ptr(), wd.data_ptr(), _IRLS_FAM[family], _IRLS_LINK[link],
                 wi.data_ptr(), zi.data_ptr(), nat.stream_ptr(Z.device))
    return wi, zi


def gram_irls(Z: torch.Tensor, beta: torch.Tensor, off, y: torch.Tensor, w: torch.Tensor, family: str, link: str):
    """One IRLS iteration's (Zᵀ W Z, Zᵀ W z) in ONE pass over Z (``k_gram_irls``: eta, mu, g'(mu), V(mu) per row
    inside the Gram pass) — or None where not covered (CPU, family / link outside the epilogue, P + 1 > 64,
    ``H2O_GLM_GRAM_IRLS=0``); the caller then runs ``irls_wz`` + ``gram``. Same formulas as ``irls_wz``."""
    if (not Z.is_cuda or family not in _IRLS_FAM or link not in _IRLS_LINK or beta.dim() != 1
            or Z.shape[1] + 1 > 64 or os.environ.get("H2O_GLM_GRAM_IRLS", "1") == "0"
            or os.environ.get("H2O_GLM_FUSED_IRLS", "1") == "0"):
        return None
    N, P = Z.shape
    Z = Z.contiguous().float()
    od = None
    if off is not None:
        od = (off if torch.is_tensor(off) else torch.full((N,), float(off), device=Z.device)).double()
        od = (od.expand(N) if od.numel() == 1 else od).contiguous()
    yd, wd = y.contiguous().double(), w.contiguous().double()
    S = _splits(N, 1)
    slabs = torch.zeros(S, 64, 64, dtype=torch.float32, device=Z.device)
    if N > 0:
        nat.call("h2o_gram_irls", Z.data_ptr(), P, beta.contiguous().double().data_ptr(), N, P,
                 0 if od is None else od.data_ptr(), yd.data_ptr(), wd.data_ptr(), _IRLS_FAM[family],
                 _IRLS_LINK[link], S, slabs.data_ptr(), nat.stream_ptr(Z.device))
    G = slabs.sum(0, dtype=torch.float64)
    return G[:P, :P].contiguous(), G[:P, P].contiguous()


def zbeta(Z: torch.Tensor, B: torch.Tensor, off=None) -> torch.Tensor:
    """``Z @ B (+ off)`` in float64 without an fp64 copy of Z. Z: [N, P] float32; B: [P] or [P, R] (R <= 8)."""
    vec = B.dim() == 1
    Bm = B[:, None] if vec else B
    N, P = Z.shape
    R = Bm.shape[1]
    if not Z.is_cuda or R > 8:
        out = Z.double() @ Bm.double()
        if off is not None:
            out = out + (off.double()[:, None] if torch.is_tensor(off) and off.dim() == 1 else off)
        return out[:, 0] if vec else out
    Z = Z.contiguous().float()
    Bd = Bm.contiguous().double()
    od = None
    if off is not None:
        od = (off if torch.is_tensor(off) else torch.full((N,), float(off), device=Z.device)).contiguous().double()
        if od.numel() == 1:
            od = od.expand(N).contiguous()
    eta = torch.empty(N, R, dtype=torch.float64, device=Z.device)
    if N > 0:
        nat.call("h2o_zbeta", Z.data_ptr(), P, Bd.data_ptr(), R, N, P, 0 if od is None else od.data_ptr(), eta.data_ptr(),
                 nat.stream_ptr(Z.device))
    return eta[:, 0] if vec else eta


def _splits(N: int, pairs: int) -> int:
    # one wave per (tile pair, slice): ~32 waves per CU. MEASURED r4 (10M x 51 augmented Gram, k_gram):
    # 4096 waves 1163 us, 8192 923, 16384 1004; 16 row pairs in flight per lane (GRAM_UNRG) 907-942 (kept 8)
    waves = int(os.environ.get("H2O_GRAM_WAVES", "8192"))
    target = max(1, waves // max(1, pairs))
    return int(max(1, min(target, (N + 1023) // 1024)))


def gram(Z: torch.Tensor, w: torch.Tensor | None = None, u: torch.Tensor | None = None):
    """Zᵀ diag(w) Z in float64. Z: [N, P] float32 row-major. With ``u`` ([N]) also Zᵀ diag(w) u from the
    same pass over Z (the augmented Gram's last column): returns (G, r)."""
    N, P = Z.shape
    if not Z.is_cuda:
        Zd = Z.double()
        Zw = Zd * (w.double()[:, None] if w is not None else 1.0)
        G = Zw.T @ Zd
        return G if u is None else (G, Zw.T @ u.double())
    Z = Z.contiguous().float()
    wf = None if w is None else w.contiguous().float()
    uf = None if u is None else u.contiguous().float()
    Pa = P + (1 if u is not None else 0)
    Ppad = (Pa + 63) // 64 * 64
    nT = Ppad // 64
    pairs = nT * (nT + 1) // 2
    S = _splits(N, pairs)
    slabs = torch.zeros(S, Ppad, Ppad, dtype=torch.float32, device=Z.device)
    if N > 0:
        nat.call("h2o_gram", Z.data_ptr(), P, 0 if wf is None else wf.data_ptr(), 0 if uf is None else uf.data_ptr(),
                 N, P, S, slabs.data_ptr(), Ppad, nat.stream_ptr(Z.device))
    G = slabs.sum(0, dtype=torch.float64)[:Pa, :Pa]
    # only tiles with ti <= tj were computed: mirror the strictly-lower tile blocks
    up = torch.triu(torch.ones(nT, nT, dtype=torch.bool, device=Z.device))
    mask = up.repeat_interleave(64, 0).repeat_interleave(64, 1)[:Pa, :Pa]
    G = torch.where(mask, G, G.T)
    return G if u is None else (G[:P, :P].contiguous(), G[:P, P].contiguous())


def xtv(Z: torch.Tensor, v: torch.Tensor) -> torch.Tensor:
    """Zᵀ v in float64; v: [N] or [N, R] (R <= 8)."""
    vec = v.dim() == 1
    V = v[:, None] if vec else v
    N, P = Z.shape
    R = V.shape[1]
    if not Z.is_cuda or R > 8:
        out = Z.double().T @ V.double()
        return out[:, 0] if vec else out
    Z = Z.contiguous().float()
    V = V.contiguous().float()
    S = int(max(1, min(1024, (N + 8191) // 8192)))
    slabs = torch.empty(S, P, R, dtype=torch.float32, device=Z.device)
    nat.call("h2o_xtv", Z.data_ptr(), P, V.data_ptr(), R, N, P, S, slabs.data_ptr(), nat.stream_ptr(Z.device))
    out = slabs.sum(0, dtype=torch.float64)
    return out[:, 0] if vec else out
