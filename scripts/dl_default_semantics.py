"""DeepLearning at H2O's default ``mini_batch_size = 1``: quality after ONE epoch of the reference's per-row ADADELTA
(Neurons.java:229-296, one update per row) against mini-batch steps of B rows on the batch-mean gradient (the GPU
engine's step), at 10k / 100k / 1M rows. fp64, manual forward / backward in NumPy (no autograd: the per-row oracle
must run a million sequential steps in minutes).

Network: F inputs -> [H, H] tanh -> 2-class softmax, UniformAdaptive init, ADADELTA rho 0.99 eps 1e-8 (H2O defaults).
Data: F uniform inputs, class = (sum of the first F/40 inputs > their half), plus 5 % label noise; holdout of 20k rows.

usage: python scripts/dl_default_semantics.py [--rows 10000,100000,1000000] [--batches 1,2,4,8,16,64,256]
"""
import argparse
import json
import math
import time

import numpy as np


def data(n, F, seed):
    rng = np.random.default_rng(seed)
    X = rng.random((n, F))
    k = max(2, F // 40)
    y = (X[:, :k].sum(1) > k / 2).astype(np.int64)
    flip = rng.random(n) < 0.05
    y[flip] = 1 - y[flip]
    return X, y


def init(F, H, seed=1):
    rng = np.random.default_rng(seed)
    ps = []
    for a, b in ((F, H), (H, H), (H, 2)):
        r = math.sqrt(6.0 / (a + b))
        ps += [(rng.random((a, b)) * 2 - 1) * r, np.zeros(b)]
    return ps


def forward(ps, X):
    h1 = np.tanh(X @ ps[0] + ps[1])
    h2 = np.tanh(h1 @ ps[2] + ps[3])
    o = h2 @ ps[4] + ps[5]
    o -= o.max(1, keepdims=True)
    p = np.exp(o)
    p /= p.sum(1, keepdims=True)
    return h1, h2, p


def grads(ps, X, y):
    """Mean gradient of the cross entropy over the rows of X."""
    h1, h2, p = forward(ps, X)
    B = X.shape[0]
    d3 = p.copy()
    d3[np.arange(B), y] -= 1.0
    d3 /= B
    g4, g5 = h2.T @ d3, d3.sum(0)
    d2 = (d3 @ ps[4].T) * (1 - h2 * h2)
    g2, g3 = h1.T @ d2, d2.sum(0)
    d1 = (d2 @ ps[2].T) * (1 - h1 * h1)
    g0, g1 = X.T @ d1, d1.sum(0)
    return [g0, g1, g2, g3, g4, g5]


def logloss(ps, X, y):
    p = forward(ps, X)[2][np.arange(X.shape[0]), y]
    return float(-np.log(np.clip(p, 1e-15, 1)).mean())


def train_one_epoch(X, y, B, H, rho=0.99, eps=1e-8, seed=1, stale=1):
    """stale = S > 1: S consecutive B-row mini-batches take their gradients at the SAME weights, then the S ADADELTA
    updates apply in order (Hogwild-style staleness of up to S - 1 updates: what S concurrent row streams do)."""
    ps = init(X.shape[1], H, seed)
    Eg = [np.zeros_like(p) for p in ps]
    Ed = [np.zeros_like(p) for p in ps]
    perm = np.random.default_rng(seed + 7).permutation(X.shape[0])
    starts = list(range(0, X.shape[0] - B + 1, B))
    for k in range(0, len(starts), stale):
        gs = [grads(ps, X[perm[s:s + B]], y[perm[s:s + B]]) for s in starts[k:k + stale]]
        for gl in gs:
            for p, g, e, d in zip(ps, gl, Eg, Ed):
                e *= rho
                e += (1 - rho) * g * g
                rate = np.sqrt((d + eps) / (e + eps))
                d *= rho
                d += (1 - rho) * rate * rate * g * g
                p -= rate * g
    return ps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", default="10000,100000,1000000")
    ap.add_argument("--batches", default="1,2,4,8,16,64,256")
    ap.add_argument("--feat", type=int, default=100)
    ap.add_argument("--hidden", type=int, default=32)
    ap.add_argument("--stale", default="1", help="comma list of S: gradients of S mini-batches at the same weights")
    a = ap.parse_args()
    Xh, yh = data(20000, a.feat, 99)
    for n in [int(v) for v in a.rows.split(",")]:
        X, y = data(n, a.feat, 0)
        for B, S in [(int(v), int(s_)) for v in a.batches.split(",") for s_ in a.stale.split(",")]:
            t0 = time.time()
            ps = train_one_epoch(X, y, B, a.hidden, stale=S)
            print(json.dumps(dict(rows=n, batch=B, stale=S, steps=n // B, train_logloss=round(logloss(ps, X, y), 5),
                                  holdout_logloss=round(logloss(ps, Xh, yh), 5), seconds=round(time.time() - t0, 1))),
                  flush=True)


if __name__ == "__main__":
    main()
