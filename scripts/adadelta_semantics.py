"""How H2O's ADADELTA behaves under mini-batching, on a scaled-down version of the DL bench target (CPU, fp64).

The reference (hex/deeplearning/Neurons.java:229-296, computeAdaDeltaRateForWeight :350-356) updates every weight ONCE
PER ROW: for each row of a mini-batch, E[g^2] <- rho E[g^2] + (1 - rho) g^2, rate = sqrt((E[dx^2] + eps) /
(E[g^2] + eps)), E[dx^2] <- rho E[dx^2] + (1 - rho) rate^2 g^2, w -= rate g. The GPU engine takes one ADADELTA step
per mini-batch on the batch-MEAN gradient. This script trains the same MLP (tanh, [H, H], softmax over 2 classes)
four ways and prints the training logloss / AUC per epoch:
  rowwise      the reference: one ADADELTA step per row (mini_batch_size = 1)
  batch_mean   one step per batch on the mean gradient (the engine today)
  batch_seq    per-row semantics emulated per batch: n steps folded into one with the per-weight sums S1 = sum g_i and
               S2 = sum g_i^2 (E[g^2] <- rho^n E + (1 - rho^n) S2 / n; rate from it; dx = -rate S1)
usage: python scripts/adadelta_semantics.py [--rows 20000] [--feat 100] [--hidden 32] [--batch 256] [--epochs 3]
"""
import argparse
import json
import math

import numpy as np
import torch


def data(n, F, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, F, generator=g, dtype=torch.float64)
    k = max(2, F // 40)
    y = (X[:, :k].sum(1) > k / 2).long()
    return X, y


def init(F, H, seed=1):
    g = torch.Generator().manual_seed(seed)
    ps = []
    for a, b in ((F, H), (H, H), (H, 2)):
        r = math.sqrt(6.0 / (a + b))           # UniformAdaptive init (DeepLearningModelInfo.randomizeWeights)
        ps += [((torch.rand(b, a, generator=g, dtype=torch.float64) * 2 - 1) * r).requires_grad_(),
               torch.zeros(b, dtype=torch.float64, requires_grad=True)]
    return ps


def fwd(ps, X):
    h = X
    for i in range(0, 4, 2):
        h = torch.tanh(h @ ps[i].T + ps[i + 1])
    return h @ ps[4].T + ps[5]


def metrics(ps, X, y):
    with torch.no_grad():
        p = torch.softmax(fwd(ps, X), 1)[:, 1].clamp(1e-15, 1 - 1e-15)
    ll = float(-(y * p.log() + (1 - y) * (1 - p).log()).mean())
    from sklearn.metrics import roc_auc_score
    return round(ll, 5), round(float(roc_auc_score(y.numpy(), p.numpy())), 4)


SUB = 0


def train(mode, X, y, H, B, epochs, rho=0.99, eps=1e-8, seed=1):
    ps = init(X.shape[1], H, seed)
    Eg = [torch.zeros_like(p) for p in ps]
    Ed = [torch.zeros_like(p) for p in ps]
    n = X.shape[0]
    g = torch.Generator().manual_seed(seed + 7)
    hist = []
    for ep in range(epochs):
        perm = torch.randperm(n, generator=g)
        if mode == "rowwise":
            for i in perm.tolist():
                loss = torch.nn.functional.cross_entropy(fwd(ps, X[i:i + 1]), y[i:i + 1])
                gr = torch.autograd.grad(loss, ps)
                with torch.no_grad():
                    for p, gg, e, d in zip(ps, gr, Eg, Ed):
                        e.mul_(rho).add_((1 - rho) * gg * gg)
                        rate = torch.sqrt((d + eps) / (e + eps))
                        d.mul_(rho).add_((1 - rho) * rate * rate * gg * gg)
                        p.sub_(rate * gg)
        else:
            for s in range(0, n - B + 1, B):
                idx = perm[s:s + B]
                if mode.startswith("batch_scaled"):
                    # linear-scaling rule on ADADELTA: one step on the batch-mean gradient, displacement times
                    # B ("batch_scaled") or sqrt(B) ("batch_scaled_sqrt")
                    mult = B if mode == "batch_scaled" else math.sqrt(B)
                    loss = torch.nn.functional.cross_entropy(fwd(ps, X[idx]), y[idx])
                    gr = torch.autograd.grad(loss, ps)
                    with torch.no_grad():
                        for p, gg, e, d in zip(ps, gr, Eg, Ed):
                            e.mul_(rho).add_((1 - rho) * gg * gg)
                            rate = torch.sqrt((d + eps) / (e + eps))
                            d.mul_(rho).add_((1 - rho) * rate * rate * gg * gg)
                            p.sub_(mult * rate * gg)
                elif mode == "batch_mean":
                    loss = torch.nn.functional.cross_entropy(fwd(ps, X[idx]), y[idx])
                    gr = torch.autograd.grad(loss, ps)
                    with torch.no_grad():
                        for p, gg, e, d in zip(ps, gr, Eg, Ed):
                            e.mul_(rho).add_((1 - rho) * gg * gg)
                            rate = torch.sqrt((d + eps) / (e + eps))
                            d.mul_(rho).add_((1 - rho) * rate * rate * gg * gg)
                            p.sub_(rate * gg)
                elif mode in ("batch_sub", "batch_sub_mean"):
                    # per-row-equivalent sub-steps: B ADADELTA steps per batch, each moving along the batch-mean
                    # gradient; the accumulators see the per-row mean square (batch_sub: (delta^2)^T (x^2), one extra
                    # GEMM on device) or the squared mean (batch_sub_mean: no extra pass)
                    from torch.func import grad, vmap

                    def lossf(pp, xi, yi):
                        return torch.nn.functional.cross_entropy(fwd(pp, xi[None]), yi[None])
                    if mode == "batch_sub":
                        per = vmap(grad(lossf), in_dims=(None, 0, 0))([p.detach() for p in ps], X[idx], y[idx])
                        gms = [gi.mean(0) for gi in per]
                        qs = [(gi * gi).mean(0) for gi in per]
                    else:
                        loss = torch.nn.functional.cross_entropy(fwd(ps, X[idx]), y[idx])
                        gms = list(torch.autograd.grad(loss, ps))
                        qs = [gm * gm for gm in gms]
                    with torch.no_grad():
                        for p, gm, q, e, d in zip(ps, gms, qs, Eg, Ed):
                            for _ in range(SUB if SUB else B):
                                e.mul_(rho).add_((1 - rho) * q)
                                rate = torch.sqrt((d + eps) / (e + eps))
                                d.mul_(rho).add_((1 - rho) * rate * rate * q)
                                p.sub_(rate * gm)
                else:   # batch_seq: exact per-row sums S1, S2 (per-sample gradients via vmap)
                    from torch.func import functional_call, grad, vmap

                    def lossf(pp, xi, yi):
                        return torch.nn.functional.cross_entropy(fwd(pp, xi[None]), yi[None])
                    per = vmap(grad(lossf), in_dims=(None, 0, 0))([p.detach() for p in ps], X[idx], y[idx])
                    with torch.no_grad():
                        rn = rho ** B
                        for p, gi, e, d in zip(ps, per, Eg, Ed):
                            S1, S2 = gi.sum(0), (gi * gi).sum(0)
                            e.mul_(rn).add_((1 - rn) * S2 / B)
                            rate = torch.sqrt((d + eps) / (e + eps))
                            d.mul_(rn).add_((1 - rn) * rate * rate * S2 / B)
                            p.sub_(rate * S1)
        hist.append((ep + 1,) + metrics(ps, X, y))
    return hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=20000)
    ap.add_argument("--feat", type=int, default=100)
    ap.add_argument("--hidden", type=int, default=32)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--epochs", type=int, default=3)
    ap.add_argument("--modes", default="batch_mean,batch_seq,rowwise")
    ap.add_argument("--sub", type=int, default=0, help="sub-steps per batch for batch_sub* (0 = batch size)")
    a = ap.parse_args()
    X, y = data(a.rows, a.feat)
    global SUB
    SUB = a.sub
    for mode in a.modes.split(","):
        print(json.dumps({"mode": mode, "batch": 1 if mode == "rowwise" else a.batch,
                          "epochs_logloss_auc": train(mode, X, y, a.hidden, a.batch, a.epochs)}), flush=True)


if __name__ == "__main__":
    main()
