"""DCT transformer (reference: ``hex/DCTTransformer.java``: 1-D/2-D/3-D discrete cosine transform of
each row of a numeric frame laid out as ``dimensions`` = [width, height, depth]; ``inverse``).

Orthonormal DCT-II (inverse = DCT-III) computed on device as matrix products with the DCT basis
along each dimension (the row batch is the GEMM's M dimension).
"""
from __future__ import annotations

import math

import torch


def _basis(n, device):
    k = torch.arange(n, dtype=torch.float64, device=device)[:, None]
    i = torch.arange(n, dtype=torch.float64, device=device)[None, :]
    C = torch.cos(math.pi * (i + 0.5) * k / n) * math.sqrt(2.0 / n)
    C[0] /= math.sqrt(2.0)
    return C                                   # [k, i], orthonormal


def dct(frame, dimensions, inverse=False):
    from ..frame import H2OFrame
    W, H, D = (list(dimensions) + [1, 1])[:3]
    X = frame.as_tensor(dtype=torch.float64)   # [N, W*H*D]
    N = X.shape[0]
    if X.shape[1] != W * H * D:
        raise ValueError(f"frame has {X.shape[1]} columns, dimensions give {W * H * D}")
    T = X.reshape(N, D, H, W)
    for axis, n in ((3, W), (2, H), (1, D)):
        if n == 1:
            continue
        C = _basis(n, X.device)
        M = C.T if inverse else C
        T = torch.movedim(torch.movedim(T, axis, -1) @ M.T, -1, axis)
    return H2OFrame.from_tensor(T.reshape(N, -1), frame.names)
