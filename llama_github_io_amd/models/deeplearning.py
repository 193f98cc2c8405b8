"""Deep Learning: feed-forward MLP (reference: ``hex/deeplearning/DeepLearning.java``,
``DeepLearningModel.java`` (parameters/defaults), ``Neurons.java`` (activations, dropout, ADADELTA /
momentum updates, max_w2), ``DeepLearningTask.java`` (Hogwild! map)).

MI355X design: synchronous mini-batch SGD instead of Hogwild (lock-free races do not map to a GPU).
Hidden layers are hipBLASLt GEMMs (bf16 or fp32 via ``compute_dtype``) followed by the fused HIP
bias+activation+dropout epilogue (``ops.dense.BiasAct``, forward and backward), or the hand-written fused MFMA
step (``csrc/dl_kernels.hip``).

Multi-GPU (row-sharded) follows H2O's map/reduce semantics (``DeepLearningTask.java:169-224``,
``DeepLearningModelInfo.add/div``): every rank trains its OWN copy of the model on its own rows for one
iteration of ``train_samples_per_iteration`` global samples (tspi / W local samples, the single-GPU
hipGraph-chunked step path), then ONE flat all-reduce averages the weights, biases and optimizer state
(ADADELTA E[g^2] / E[dx^2], momenta). With ``elastic_averaging`` the ranks keep their local models and a
consensus model is the time average pa * node-average + (1 - pa) * previous consensus
(``DeepLearningModelInfo.timeAverage``), with the elastic pull ``elastic_averaging_regularization * (w - w_EA)``
in every local gradient (``Neurons.java:263,414``); the consensus is the model scored and returned.
``H2O_DL_DP=sync`` instead all-reduces the gradient of every global mini-batch (1-step averaging).
Supports Rectifier/Tanh/ExpRectifier/Maxout (+WithDropout), input/hidden dropout, L1/L2,
max_w2, ADADELTA (rho, epsilon) or momentum SGD with rate annealing/decay and Nesterov,
autoencoder + ``anomaly`` (per-row reconstruction MSE) + ``deepfeatures``, regression
distributions (gaussian/poisson/gamma/tweedie/laplace/quantile/huber), early stopping.
"""
from __future__ import annotations

import math
import os
import time

import numpy as np
import torch

from .. import metrics as mm
from ..ops.dense import ACT, bias_act, step_seed
from ..parallel import collectives as coll
from .params import canon
from .base import DataInfo, Model, ScoreKeeper, make_key, model_category
from .datainfo import Expander

DL_DEFAULTS = dict(hidden=[200, 200], epochs=10.0, activation="Rectifier", adaptive_rate=True, rho=0.99, epsilon=1e-8,
                   rate=0.005, rate_annealing=1e-6, rate_decay=1.0, momentum_start=0.0, momentum_ramp=1e6,
                   momentum_stable=0.0, nesterov_accelerated_gradient=True, input_dropout_ratio=0.0,
                   hidden_dropout_ratios=None, l1=0.0, l2=0.0, max_w2=float("inf"),
                   initial_weight_distribution="UniformAdaptive", initial_weight_scale=1.0, loss="Automatic",
                   distribution="AUTO", tweedie_power=1.5, quantile_alpha=0.5, huber_alpha=0.9,
                   average_activation=0.0, sparsity_beta=0.0, max_categorical_features=2147483647,
                   mini_batch_size=1, autoencoder=False, standardize=True, use_all_factor_levels=True,
                   stopping_rounds=5, stopping_metric="AUTO", stopping_tolerance=0.0, score_interval=5.0,
                   score_training_samples=10000, seed=-1, shuffle_training_data=True, reproducible=False,
                   export_weights_and_biases=False, missing_values_handling="MeanImputation", max_runtime_secs=0.0,
                   compute_dtype="float32", gpu_batch_size=256, train_samples_per_iteration=-2,
                   overwrite_with_best_model=True, classification_stop=0.0, regression_stop=1e-6,
                   elastic_averaging=False, elastic_averaging_moving_rate=0.9, elastic_averaging_regularization=1e-3)


class MLP(torch.nn.Module):
    def __init__(self, n_in, hidden, n_out, act: str, maxout: bool, in_drop, hid_drop, init_dist, init_scale, gen):
        super().__init__()
        self.act = act
        self.maxout = maxout
        self.in_drop = in_drop
        self.hid_drop = hid_drop
        dims = [n_in] + list(hidden)
        self.hidden = torch.nn.ModuleList()
        for i in range(len(hidden)):
            width = dims[i + 1] * (2 if maxout else 1)
            lin = torch.nn.Linear(dims[i], width)
            self._init(lin, dims[i], width, init_dist, init_scale, gen)
            if act == "rectifier" or maxout:     # DeepLearningModelInfo.initializeMembers: 0.5 / 1 (no dead units)
                with torch.no_grad():
                    lin.bias.fill_(0.5 if i == 0 else 1.0)
            self.hidden.append(lin)
        self.out = torch.nn.Linear(dims[-1], n_out)
        self._init(self.out, dims[-1], n_out, init_dist, init_scale, gen)
        self.step = 0
        self.step_dev = None
        self.track = None       # dict layer -> batch-mean activation (sparse autoencoder)

    @staticmethod
    def _init(lin, fan_in, fan_out, dist, scale, gen):
        with torch.no_grad():
            d = canon(dist)
            if d == "uniformadaptive":
                r = math.sqrt(6.0 / (fan_in + fan_out))
                lin.weight.uniform_(-r, r, generator=gen)
            elif d == "uniform":
                lin.weight.uniform_(-scale, scale, generator=gen)
            else:
                lin.weight.normal_(0, scale, generator=gen)
            lin.bias.zero_()

    def forward(self, x, seed=0, features_layer=None):
        if self.training and self.in_drop > 0:
            keep = (torch.rand(x.shape, device=x.device) >= self.in_drop).to(x.dtype)
            x = x * keep / (1 - self.in_drop)
        for i, lin in enumerate(self.hidden):
            h = torch.nn.functional.linear(x, lin.weight)
            drop = self.hid_drop[i] if self.training else 0.0
            if self.maxout:
                h = h + lin.bias
                a, b = h.chunk(2, dim=1)
                x = torch.maximum(a, b)
                if drop > 0:
                    x = x * (torch.rand(x.shape, device=x.device) >= drop).to(x.dtype) / (1 - drop)
            else:
                # bf16 GEMM outputs stay bf16 through the fused epilogue into the next GEMM (no fp32 round trip)
                xin = h if (h.is_cuda and h.dtype == torch.bfloat16) else h.float()
                base = (seed * 1000003 + i * 7919) & ((1 << 62) - 1)
                if self.step_dev is not None:      # captured step: the kernels read the step counter on device
                    x = bias_act(xin, lin.bias, self.act, drop, base, self.step_dev)
                else:
                    x = bias_act(xin, lin.bias, self.act, drop, step_seed(base, self.step))
                if self.track is not None:
                    self.track[i] = x.detach().float().mean(0)
            if features_layer is not None and i == features_layer:
                return x
        return self.out(x)


class DeepLearningModel(Model):
    algo = "deeplearning"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.net = None
        self.expander = None
        self.resp_mu = 0.0
        self.resp_sd = 1.0

    def _forward(self, X):
        Z = self.expander.transform(X.to(self.device))
        self.net.eval()
        with torch.no_grad():
            return self.net(Z), Z

    def _predict_tensor(self, X, offset=None):
        out, Z = self._forward(X)
        if self.params.get("autoencoder"):
            return out.float()
        cat = self.model_category
        if cat in ("Binomial", "Multinomial"):
            return torch.softmax(out.float(), 1)
        f = out[:, 0].double() * self.resp_sd + self.resp_mu
        d = self.output.get("distribution", "gaussian")
        if d in ("poisson", "gamma", "tweedie"):
            f = torch.exp(out[:, 0].double())
        return f.float()

    @property
    def model_category(self):
        return "AutoEncoder" if self.params.get("autoencoder") else self.output["model_category"]

    def anomaly(self, frame, per_feature=False):
        from ..frame import Column, H2OFrame
        X, _ = frame.model_matrix(self.info, device=self.device)
        out, Z = self._forward(X)
        err = (out.float() - Z.float()) ** 2
        if per_feature:
            return H2OFrame._from_columns([Column(f"reconstr_{n}.SE", "real", err[:, i].double())
                                           for i, n in enumerate(self.expander.names)])
        return H2OFrame._from_columns([Column("Reconstruction.MSE", "real", err.mean(1).double())])

    def deepfeatures(self, frame, layer: int):
        from ..frame import H2OFrame
        X, _ = frame.model_matrix(self.info, device=self.device)
        Z = self.expander.transform(X)
        self.net.eval()
        with torch.no_grad():
            F = self.net(Z, features_layer=layer)
        return H2OFrame.from_tensor(F.float(), [f"DF.L{layer + 1}.C{i + 1}" for i in range(F.shape[1])])

    def weights(self, matrix_id=0):
        lins = list(self.net.hidden) + [self.net.out]
        return lins[matrix_id].weight.detach().cpu().numpy()

    def biases(self, vector_id=0):
        lins = list(self.net.hidden) + [self.net.out]
        return lins[vector_id].bias.detach().cpu().numpy()

    def to_state(self):
        s = super().to_state()
        s["net"] = {k: v.cpu().tolist() for k, v in self.net.state_dict().items()}
        s["net_cfg"] = self._cfg
        s["expander"] = self.expander.to_state()
        s["resp"] = [self.resp_mu, self.resp_sd]
        return s

    def _restore(self, s):
        super()._restore(s)
        self._cfg = s["net_cfg"]
        c = self._cfg
        self.net = MLP(c["n_in"], c["hidden"], c["n_out"], c["act"], c["maxout"], 0.0, [0.0] * len(c["hidden"]),
                       "uniformadaptive", 1.0, torch.Generator().manual_seed(0))
        self.net.load_state_dict({k: torch.tensor(v) for k, v in s["net"].items()})
        self.expander = Expander.from_state(self.info, s["expander"])
        self.resp_mu, self.resp_sd = s["resp"]


class DeepLearningTrainer:
    def __init__(self, params):
        p = dict(DL_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        from .shared_tree import resolve_seed
        t0 = time.time()
        p = self.p
        dev = X.device
        N = X.shape[1]
        seed = resolve_seed(p["seed"])
        torch.manual_seed(seed & 0x7FFFFFFF)
        gen = torch.Generator().manual_seed(seed & 0x7FFFFFFF)
        ae = bool(p["autoencoder"])
        cat = "AutoEncoder" if ae else model_category(info)
        w = torch.ones(N, dtype=torch.float64, device=dev) if w is None else w.double()
        if y is not None and not ae:
            ok = ~torch.isnan(y)
            w = torch.where(ok, w, torch.zeros_like(w))
        if canon(p.get("missing_values_handling") or "MeanImputation") == "skip":
            # DataInfo skipMissing: rows with a missing predictor do not train
            w = torch.where(torch.isnan(X).any(0), torch.zeros_like(w), w)
        sharded = coll.is_dist()
        # data parallelism: per-iteration model averaging (H2O semantics, default) or per-step gradient sync
        dp_avg = sharded and os.environ.get("H2O_DL_DP", "average") != "sync"
        gsync = sharded and not dp_avg
        Wn = coll.world() if sharded else 1
        dp_local = dp_avg and os.environ.get("H2O_DL_DP") == "local"
        elastic = dp_avg and not dp_local and bool(p.get("elastic_averaging"))
        # dropout masks: each rank of a model-averaging run trains on different rows with its own stream
        dseed = (seed ^ (coll.rank() * 0x9E3779B97F4A7C15)) & ((1 << 63) - 1) if dp_avg else seed
        row0, N_glob = coll.exclusive_offset(N) if sharded else (0, N)
        self._row0, self._N_glob = row0, N_glob
        ex = Expander(info, standardize=p["standardize"], use_all_factor_levels=p["use_all_factor_levels"]).fit(
            X, w, reduce=coll.all_reduce_ if sharded else None)
        mcf = p.get("max_categorical_features")
        mcf = 2147483647 if mcf is None else int(mcf)
        if mcf < 1:
            raise ValueError("max_categorical_features must be at least 1")
        ex.set_cat_hash(mcf, seed)
        # bf16 compute: the design matrix is materialised in bf16 (half the HBM footprint and per-step
        # gather bytes; GEMM inputs need no per-step cast)
        bf16 = dev.type == "cuda" and str(p["compute_dtype"]).lower() in ("bf16", "bfloat16") and not bool(p["autoencoder"])
        Z = ex.transform(X, dtype=torch.bfloat16 if bf16 else torch.float32)
        act_name = canon(p["activation"])
        with_drop = act_name.endswith("withdropout")
        base = act_name.replace("withdropout", "")
        maxout = base == "maxout"
        hidden = list(p["hidden"])
        hd = p["hidden_dropout_ratios"]
        if hd is None:
            hd = [0.5 if with_drop else 0.0] * len(hidden)
        K = len(info.response_domain) if cat in ("Binomial", "Multinomial") else 1
        n_out = Z.shape[1] if ae else K
        dist = str(p["distribution"]).lower()
        if dist == "auto":
            dist = "gaussian" if cat == "Regression" else ("bernoulli" if cat == "Binomial" else "multinomial")
        # huber: delta starts at 1 and is re-estimated at every training scoring event as the weighted
        # huber_alpha quantile of |actual - prediction| (DeepLearningModel.doScoring: setHuberDelta); a
        # device scalar so captured step graphs see the update
        self._hdelta = torch.ones((), dtype=torch.float32, device=dev)
        self._dist = dist
        net = MLP(Z.shape[1], hidden, n_out, "rectifier" if maxout else base, maxout, float(p["input_dropout_ratio"]),
                  [float(v) for v in hd], str(p["initial_weight_distribution"]), float(p["initial_weight_scale"]), gen).to(dev)
        prev_epochs = 0.0
        ck = p.get("checkpoint")
        if ck:   # continue from a previous model (DeepLearning.java checkpoint): same architecture, more epochs
            from ..core import dkv
            prev = dkv.get(ck) if isinstance(ck, str) else getattr(ck, "_model", ck)
            if prev is None or getattr(prev, "net", None) is None:
                raise ValueError(f"checkpoint {ck} is not a DeepLearning model")
            if prev._cfg["hidden"] != hidden or prev._cfg["n_in"] != Z.shape[1]:
                raise ValueError("checkpoint architecture (hidden / inputs) differs")
            net.load_state_dict({k: v.to(dev) for k, v in prev.net.state_dict().items()})
            prev_epochs = float(prev.output.get("epochs", 0.0))
            if float(p["epochs"]) <= prev_epochs:
                raise ValueError(f"epochs must exceed the checkpoint's {prev_epochs}")
        self._initial_state(net, p, hidden, Z.shape[1], dev)
        if coll.is_dist():
            flat = torch.cat([q.detach().reshape(-1) for q in net.parameters()])
            coll.broadcast_(flat)
            o = 0
            with torch.no_grad():
                for q in net.parameters():
                    q.copy_(flat[o:o + q.numel()].view_as(q))
                    o += q.numel()
        model = DeepLearningModel(model_key or make_key("deeplearning"), p, info)
        model.device = dev
        model.expander = ex
        model.net = net
        model._cfg = dict(n_in=Z.shape[1], hidden=hidden, n_out=n_out, act="rectifier" if maxout else base, maxout=maxout)
        model.output["distribution"] = dist
        yt = None
        if not ae:
            if cat == "Regression":
                yy = torch.nan_to_num(y.double(), nan=0.0)
                if dist in ("gaussian", "laplace", "quantile", "huber"):
                    sw_all = coll.all_reduce_scalar(float(w.sum()))
                    mu = coll.all_reduce_scalar(float((w * yy).sum())) / sw_all
                    sd = math.sqrt(coll.all_reduce_scalar(float((w * (yy - mu) ** 2).sum())) / sw_all) or 1.0
                    if not p["standardize"]:
                        mu, sd = 0.0, 1.0
                    model.resp_mu, model.resp_sd = mu, sd
                    yt = ((yy - mu) / sd).float()
                else:
                    yt = yy.float()
            else:
                yt = torch.nan_to_num(y, nan=0).long()
        B = int(p["mini_batch_size"])
        if B <= 1:
            # H2O's default mini_batch_size = 1 is one ADADELTA step per ROW (Neurons.java:229-296). ADADELTA warms
            # its step sizes up per STEP, so the GPU's B-row steps (one step on the batch-mean gradient) are sized
            # to keep >= ~16K steps per epoch: B = N // 16384 in [1, gpu_batch_size]. MEASURED (fp64 oracle,
            # scripts/dl_default_semantics.py, profiles/r6_dl_default_semantics.md): one-epoch logloss within
            # 0-3 % of the per-row reference at 10k / 100k / 1M rows; the former rule (N // 1024 up to 256: 9 /
            # 97 / 256-row steps) was 12 / 25 / 18 % worse. Set mini_batch_size for throughput instead.
            B = max(1, min(int(p["gpu_batch_size"]), N_glob // 16384))
        B = max(1, min(B, N_glob))
        if dp_avg:   # local mini-batches: never larger than the smallest shard
            bt = torch.tensor([float(min(B, N))], dtype=torch.float64, device=coll.comm_device())
            B = max(1, int(coll.all_reduce_min_(bt).item()))
        from ..ops.dense import FlatParams
        fp = FlatParams(net)                 # params/grads as views of two flat buffers
        params = fp.params
        adaptive = bool(p["adaptive_rate"])
        mom = torch.zeros_like(fp.p)
        rho, eps = float(p["rho"]), float(p["epsilon"])
        l1, l2 = float(p["l1"]), float(p["l2"])
        max_w2 = float(p["max_w2"])
        nesterov = bool(p["nesterov_accelerated_gradient"])
        # rate_decay (Neurons.java: layer i learns at rate * rate_decay^i) as a per-element multiplier of the
        # flat parameter buffer (weights of every layer first, then biases)
        rdec = float(p.get("rate_decay") or 1.0)
        rmul = None
        if not adaptive and rdec != 1.0:
            lins = list(net.hidden) + [net.out]
            layer_of = {id(l_.weight): i for i, l_ in enumerate(lins)}
            layer_of.update({id(l_.bias): i for i, l_ in enumerate(lins)})
            rmul = torch.cat([torch.full((q.numel(),), rdec ** layer_of[id(q)], dtype=torch.float32, device=dev)
                              for q in params])
        keeper = ScoreKeeper(p["stopping_rounds"], p["stopping_metric"], p["stopping_tolerance"],
                             "Regression" if ae else cat)
        epochs = float(p["epochs"]) - prev_epochs
        Bg = B * Wn if dp_avg else B          # global samples per (local) step
        total = int(math.ceil(epochs * N_glob / Bg))
        # the epoch permutation is drawn on the device (a host randperm of 10M rows costs ~0.3 s per epoch);
        # every rank draws the same one from the same seed (model averaging: each rank its own local one)
        g = torch.Generator(device=dev).manual_seed((seed + (1000003 * coll.rank() if dp_avg else 0)) & 0x7FFFFFFF)
        history = []
        samples = 0
        last_score = time.time()
        dtype = torch.bfloat16 if str(p["compute_dtype"]).lower() in ("bf16", "bfloat16") else None
        wf = w.float()
        # per-step scalars live on the device so one captured step serves every step
        step_t = torch.zeros(1, dtype=torch.int64, device=dev)
        rate_t = torch.zeros((), dtype=torch.float32, device=dev)
        mom_t = torch.zeros((), dtype=torch.float32, device=dev)
        on_t = torch.zeros((), dtype=torch.float32, device=dev)
        gbuf = torch.empty(fp.g.numel() + 1, dtype=fp.g.dtype, device=fp.g.device) if gsync else None
        # elastic averaging: consensus parameters w_EA and the device switch of the elastic pull (off until
        # the first consensus exists, as the reference's null _wEA in the first iteration)
        ea_lam = float(p.get("elastic_averaging_regularization") or 0.0)
        ea_pa = float(p.get("elastic_averaging_moving_rate") or 0.9)
        if elastic and not (0.0 < ea_pa <= 1.0):
            raise ValueError("elastic_averaging_moving_rate must be in (0, 1]")
        # (allocated up front: captured step graphs read it in place)
        ea = torch.zeros(fp.p.numel() * (3 if bool(p["adaptive_rate"]) else 2) if elastic else 0,
                         dtype=torch.float32, device=dev)
        ea_on = torch.zeros((), dtype=torch.float32, device=dev)
        tdim = tuple(yt.shape[1:]) if yt is not None else ()

        # sparse autoencoder (Neurons.compute_sparsity / update_bias): a rolling mean activation per neuron
        # of every hidden layer but the last (decay 0.999 per row) pulls each bias by
        # sparsity_beta * (mean activation - average_activation): here as that gradient on the bias
        beta_sp = float(p.get("sparsity_beta") or 0.0)
        sparse = ae and beta_sp > 0 and len(hidden) > 1 and not maxout
        avg_a = [torch.zeros(int(hidden[l]), dtype=torch.float32, device=dev) for l in range(len(hidden) - 1)] if sparse else []
        tgt_a = float(p.get("average_activation") or 0.0)

        def fwd_bwd(xb, wb, tb):
            """Forward + backward of one (local) batch into fp.g: the gradient of the weighted loss sum,
            normalised by the batch weight (single process) or raw + batch weight in gbuf (sharded)."""
            fp.zero_grad()
            net.track = {} if sparse else None
            with torch.autocast(device_type=dev.type, dtype=dtype, enabled=dtype is not None):
                o = net(xb, dseed)
            ls = self._loss(o.float(), xb if ae else tb, wb, cat, dist, ae)
            if sparse:
                dec = 0.999 ** xb.shape[0]
                for l, a in enumerate(avg_a):
                    a.mul_(dec).add_(net.track[l] * (1.0 - dec))
                    ls = ls + wb.sum() * beta_sp * ((a - tgt_a) * net.hidden[l].bias.float()).sum()
                net.track = None
            if gsync:
                ls.backward()
                gbuf[:-1].copy_(fp.g)
                gbuf[-1:].copy_(wb.sum().view(1))
            else:
                (ls / wb.sum().clamp(min=1e-12)).backward()

        def update(rate_t=rate_t, mom_t=mom_t, on_t=on_t):
            """Optimizer step on the flat buffers (ADADELTA: one fused HIP launch; momentum SGD with rate
            annealing / Nesterov from the device scalars rate_t, mom_t, on_t), then max_w2 row clipping."""
            with torch.no_grad():
                if gsync:         # data parallel: the all-reduced [sum-gradient, batch weight] -> mean gradient
                    fp.g.copy_(gbuf[:-1] / gbuf[-1].clamp(min=1e-12))
                if elastic and ea_lam > 0:   # elastic pull towards the consensus (Neurons.java:263,414)
                    fp.g.add_((fp.p - ea[: fp.p.numel()]) * (ea_on * ea_lam))
                fobj = fz.get("obj")
                if adaptive:      # ADADELTA (Neurons.java: rho, epsilon); also refreshes the bf16 weights and
                    # (fused step) the transposed copy its backward pass reads
                    fp.adadelta(rho, eps, l1, l2, shadow, None if fobj is None else fz["wt"])
                else:
                    gg = fp.g.clone()
                    nd = fp.n_decay
                    if l2 > 0 or l1 > 0:
                        gg[:nd] += l2 * fp.p[:nd] + l1 * torch.sign(fp.p[:nd])
                    upd = gg * -rate_t if rmul is None else gg * rmul * -rate_t
                    mom.mul_(mom_t).add_(upd * on_t)
                    if nesterov:
                        fp.p.add_(mom * mom_t + upd)
                    else:
                        fp.p.add_(mom * on_t + upd * (1 - on_t))
                if max_w2 < float("inf"):
                    for q in params:
                        if q.dim() > 1:
                            n2 = (q * q).sum(1, keepdim=True)
                            q.mul_(torch.where(n2 > max_w2, torch.sqrt(max_w2 / n2), torch.ones_like(n2)))
                if shadow is not None and (not adaptive or max_w2 < float("inf")):
                    shadow.copy_(fp.p[: fp.n_decay])
                if fobj is not None and (not adaptive or max_w2 < float("inf")):
                    fobj.refresh_transposed()

        # Explicit training step (no autograd) for the common MLPs: GEMMs on bf16 weight copies kept by the
        # fused ADADELTA kernel, fused bias/activation/dropout epilogues, one fused softmax-CE / squared-error
        # output-gradient pass; weight gradients land in the flat buffer, bias gradients are accumulated by
        # the epilogue kernels straight into it (~20 launches per step instead of ~45).
        lname = str(p["loss"]).lower()
        from ..ops import dl as dlops
        in_drop = float(p["input_dropout_ratio"])
        # input dropout runs in the fused step only (the library-GEMM explicit step has no input mask)
        fused_shape = (dev.type == "cuda" and os.environ.get("H2O_DL_FUSED", "1") == "1" and net.act in ACT
                       and (Z.dtype == torch.bfloat16 or os.environ.get("H2O_DL_FUSED_F32", "1") == "1")
                       and dlops.supported(int(Z.shape[1]), [int(h_) for h_ in hidden], int(net.out.weight.shape[0]),
                                           ACT[net.act], Z, maxout))
        # Maxout and input dropout run in the fused step only (the library-GEMM explicit step has neither)
        # the autoencoder (quadratic reconstruction loss, no sparsity penalty) runs in the fused step only
        ae_fused = ae and fused_shape and not sparse and lname in ("automatic", "quadratic")
        explicit = (os.environ.get("H2O_DL_EXPLICIT", "1") == "1" and (not ae or ae_fused)
                    and (not maxout or fused_shape) and (in_drop == 0 or fused_shape) and net.act in ACT
                    and ((cat in ("Binomial", "Multinomial") and dist in ("bernoulli", "multinomial")
                          and lname in ("automatic", "crossentropy", "cross_entropy"))
                         or (cat == "Regression" and dist == "gaussian" and lname in ("automatic", "quadratic"))
                         or ae_fused))
        if explicit and p.get("reproducible"):
            # reproducible=True (bit-identical seeded runs): the library-GEMM explicit step accumulates bias
            # gradients with float atomics; only the fused step (fixed-order reductions) or autograd qualify
            if not (dev.type == "cuda" and os.environ.get("H2O_DL_FUSED", "1") == "1" and dlops.supported(
                    int(Z.shape[1]), [int(h_) for h_ in hidden], int(net.out.weight.shape[0]), ACT[net.act], Z,
                    maxout)):
                explicit = False
        shadow = None
        if explicit:
            lins = list(net.hidden) + [net.out]
            base_ptr, esz = fp.p.data_ptr(), fp.p.element_size()
            w_off = [(l_.weight.data_ptr() - base_ptr) // esz for l_ in lins]
            b_off = [(l_.bias.data_ptr() - base_ptr) // esz for l_ in lins]
            cdt = torch.bfloat16 if (dtype is not None and dev.type == "cuda") else torch.float32
            if cdt == torch.bfloat16:
                shadow = fp.p[: fp.n_decay].to(torch.bfloat16)
                Wc = [shadow[o:o + l_.weight.numel()].view_as(l_.weight) for o, l_ in zip(w_off, lins)]
            else:
                Wc = [l_.weight.data for l_ in lins]
            gW = [fp.g[o:o + l_.weight.numel()].view_as(l_.weight) for o, l_ in zip(w_off, lins)]
            gB = [fp.g[o:o + l_.bias.numel()] for o, l_ in zip(b_off, lins)]
            bO = net.out.bias.data
            act_code = ACT[net.act]
            inv_t = torch.ones(1, dtype=torch.float32, device=dev)
            from ..ops.dense import bias_act_bwd, bias_act_fwd, out_grad

            def fwd_bwd(xb, wb, tb):      # noqa: F811 - the explicit step replaces the autograd one
                with torch.no_grad():
                    fp.g[fp.n_decay:].zero_()
                    if not gsync:
                        torch.reciprocal(wb.sum().clamp(min=1e-12).view(1), out=inv_t)
                    hs = [xb if xb.dtype == cdt else xb.to(cdt)]
                    seeds = []
                    for i, lin in enumerate(net.hidden):
                        drop = net.hid_drop[i]
                        base = (dseed * 1000003 + i * 7919) & ((1 << 62) - 1)
                        sd = (base, net.step_dev) if net.step_dev is not None else (step_seed(base, net.step), None)
                        seeds.append(sd)
                        a_ = torch.mm(hs[-1], Wc[i].t())
                        hs.append(bias_act_fwd(a_, lin.bias.data, act_code, drop, sd[0], sd[1]))
                    logits = torch.addmm(bO.to(cdt), hs[-1], Wc[-1].t())
                    wf32 = wb.float()
                    if cat == "Regression":
                        dO = out_grad(logits, None, tb.float(), wf32, inv_t, gB[-1])
                    else:
                        dO = out_grad(logits, tb.long(), None, wf32, inv_t, gB[-1])
                    gW[-1].copy_(torch.mm(dO.t(), hs[-1]))
                    dh = torch.mm(dO, Wc[-1])
                    for i in range(len(net.hidden) - 1, -1, -1):
                        dA = bias_act_bwd(dh, hs[i + 1], act_code, net.hid_drop[i], seeds[i][0], seeds[i][1], gB[i])
                        gW[i].copy_(torch.mm(dA.t(), hs[i]))
                        if i > 0:
                            dh = torch.mm(dA, Wc[i])
                    if gsync:
                        gbuf[:-1].copy_(fp.g)
                        gbuf[-1:].copy_(wb.sum().view(1))

        # Fused MFMA step (ops/dl.py, csrc/dl_kernels.hip): gather + forward + loss gradient + backward on
        # 16-row tiles with the activations in LDS, all weight gradients in one launch, fixed-order reduce;
        # bf16 (v_mfma_f32_16x16x32_bf16) or the default fp32 compute (v_mfma_f32_16x16x4_f32).
        # Built per batch capacity in alloc(); the library-GEMM explicit step above stays for other shapes.
        fz = dict(obj=None, ok=False, sridx=None)
        if (explicit and os.environ.get("H2O_DL_FUSED", "1") == "1"
                and (cdt == torch.bfloat16 or os.environ.get("H2O_DL_FUSED_F32", "1") == "1")
                and dlops.supported(int(Z.shape[1]), [int(h_) for h_ in hidden], int(net.out.weight.shape[0]),
                                    act_code, Z, maxout)):
            fz["ok"] = True
            fz["bases"] = [(dseed * 1000003 + i * 7919) & ((1 << 62) - 1) for i in range(len(net.hidden))]

        def fused_build(cap):
            gout = gbuf[:-1] if gsync else fp.g
            gsum = gbuf[-1:] if gsync else None
            fz["obj"] = dlops.FusedMLPStep(fp, list(net.hidden) + [net.out], act_code, list(net.hid_drop),
                                           fz["bases"], Z, wf, yt, cat == "Regression", cap, shadow, step_t, gout,
                                           gsum, in_drop, (dseed * 1000003 + 104729) & ((1 << 62) - 1), maxout,
                                           ae)
            fz["obj"].refresh_transposed()
            fz["sridx"] = torch.full((cap,), -1, dtype=torch.long, device=dev)
            # nothing but ADADELTA reads the weight gradient (no all-reduce, no elastic pull): the update sums
            # the fused step's split partials itself (one launch fewer per step)
            if (adaptive and not gsync and not (elastic and ea_lam > 0)
                    and os.environ.get("H2O_DL_FUSE_WSUM", "1") == "1"):
                fz["wt"] = fz["obj"].optimizer_reads_partials()
            else:
                fz["wt"] = fz["obj"].wt_map

        if fz["ok"]:
            fwd_bwd_lib = fwd_bwd

            def fwd_bwd(xb, wb, tb):      # noqa: F811 - rows come from the static index buffer, not xb
                if fz["obj"] is None:     # eager steps (no graph capture): the library-GEMM explicit step
                    return fwd_bwd_lib(xb, wb, tb)
                fz["obj"].args.step_dev = step_t.data_ptr()
                fz["obj"].step(fz["sridx"])

        # hipGraph capture of the training step (fwd + bwd (+ update)): a fixed launch sequence on static
        # batch buffers, replayed per step. Row-sharded runs capture fwd+bwd and the update separately with
        # the one flat gradient all-reduce between them; their local batch buffer is sized to the largest
        # per-rank share of a global batch in the epoch (padding rows carry weight 0).
        use_graph = dev.type == "cuda" and os.environ.get("H2O_DL_GRAPH", "1") == "1"
        net.step_dev = step_t if use_graph else None
        gstate = dict(cap=0, g1=None, g2=None, warm=0)
        sx = sw = sy = None
        side = torch.cuda.Stream(dev) if use_graph else None

        def alloc(cap):
            nonlocal sx, sw, sy
            if fz["ok"]:
                fused_build(cap)
            sx = torch.zeros(cap, Z.shape[1], dtype=Z.dtype, device=dev)
            sw = torch.zeros(cap, dtype=wf.dtype, device=dev)
            sy = None if ae else torch.zeros((cap,) + tdim, dtype=yt.dtype, device=dev)
            gstate.update(cap=cap, g1=None, g2=None, warm=0)

        def run_step():
            if gstate["warm"] < 2:      # warm-up steps on a side stream before capture (allocator, libraries)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    fwd_bwd(sx, sw, sy)
                    if not gsync:
                        update()
                torch.cuda.current_stream(dev).wait_stream(side)
                gstate["warm"] += 1
                if gsync:
                    coll.all_reduce_(gbuf)
                    update()
                return
            if gstate["g1"] is None:
                try:
                    g1 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g1):
                        fwd_bwd(sx, sw, sy)
                        if not gsync:
                            update()
                    g2 = None
                    if gsync:
                        g2 = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g2):
                            update()
                    gstate.update(g1=g1, g2=g2)
                except Exception as e:  # noqa: BLE001 - capture unsupported here: eager steps on the static buffers
                    gstate.update(g1=False, error=f"{type(e).__name__}: {e}")
            if gstate["g1"] is False:
                fwd_bwd(sx, sw, sy)
                if gsync:
                    coll.all_reduce_(gbuf)
                update()
                return
            gstate["g1"].replay()
            if gsync:
                coll.all_reduce_(gbuf)
                gstate["g2"].replay()

        # Single process (and each rank of a model-averaging run): CH consecutive steps (gather of the batch
        # rows from the resident design matrix included) are captured in ONE graph and replayed per chunk — the
        # host issues one index copy, one arange and one replay per CH steps instead of ~40 kernels per step.
        CH = max(1, int(os.environ.get("H2O_DL_CHUNK", "16"))) if (use_graph and not gsync) else 1
        chunk = dict(g=None)
        if CH > 1:
            ridx = torch.zeros(CH * B, dtype=torch.long, device=dev)
            step_v = torch.zeros(CH, dtype=torch.int64, device=dev)
            rate_v = torch.zeros(CH, dtype=torch.float32, device=dev)
            mom_v = torch.zeros(CH, dtype=torch.float32, device=dev)
            on_v = torch.zeros(CH, dtype=torch.float32, device=dev)

            def chunk_body():
                for k in range(CH):
                    r = ridx[k * B:(k + 1) * B]
                    net.step_dev = step_v[k:k + 1]
                    if fz.get("obj") is not None:         # the fused step gathers its rows itself
                        fz["obj"].args.step_dev = step_v[k:k + 1].data_ptr()
                        fz["obj"].step(r)
                    else:
                        torch.index_select(Z, 0, r, out=sx)
                        torch.index_select(wf, 0, r, out=sw)
                        if sy is not None:
                            torch.index_select(yt, 0, r, out=sy)
                        fwd_bwd(sx, sw, sy)
                    update(rate_v[k], mom_v[k], on_v[k])
                net.step_dev = step_t

            def run_chunk(rows, step0, samples0):
                ridx.copy_(rows)
                torch.arange(step0, step0 + CH, out=step_v)
                if not adaptive:
                    rs, ms = [], []
                    for k in range(CH):
                        smp = samples0 + (k + 1) * Bg     # the global sample count, as the single-step path
                        rs.append(float(p["rate"]) / (1 + float(p["rate_annealing"]) * smp))
                        ms.append(self._momentum(smp))
                    rate_v.copy_(torch.tensor(rs, dtype=torch.float32))
                    mom_v.copy_(torch.tensor(ms, dtype=torch.float32))
                    on_v.copy_(torch.tensor([1.0 if m_ > 0 else 0.0 for m_ in ms], dtype=torch.float32))
                if chunk["g"] is None:
                    try:
                        gc = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(gc):
                            chunk_body()
                        chunk["g"] = gc
                    except Exception as e:  # noqa: BLE001 - fall back to per-step replays
                        chunk.update(g=False, error=f"{type(e).__name__}: {e}")
                        net.step_dev = step_t
                        return False
                chunk["g"].replay()
                return True

        # global row order per epoch: mini-batches are consecutive B-slices of a permutation of the GLOBAL
        # rows; under row sharding each rank takes the members of the batch it owns (one host sync per
        # epoch for the per-step counts), so the summed gradient is the single-process one
        N_perm = N if dp_avg else N_glob       # model averaging: each rank walks its own rows
        S_ep = N_perm // B
        perm = None
        sel = offs = None
        s_in = S_ep
        owb = bool(p.get("overwrite_with_best_model", True)) and not int(p.get("nfolds") or 0)
        best_loss, best_p, last_ev, best_ev = float("inf"), None, {}, None
        # train_samples_per_iteration (DeepLearning.computeTrainSamplesPerIteration): scoring / stopping is
        # decided at the end of each iteration of tspi samples. 0 and -1 (no replicated data): one epoch;
        # -2 (auto): the reference's caps of its hardware-timed estimate, min(epochs * N / 10, 100k x nodes)
        tspi = int(p.get("train_samples_per_iteration", -2))
        if tspi in (0, -1):
            tspi = N_glob
        elif tspi == -2:
            tspi = int(max(1, min(epochs * N_glob / 10, 100000 * coll.world())))
        elif tspi < -2:
            raise ValueError("train_samples_per_iteration must be -2, -1, 0 or > 0")
        spi = 0
        if dp_avg:
            # steps per iteration (the averaging period), a multiple of the graph chunk when it is longer: the
            # collective falls between two chunk replays
            spi = max(1, int(round(tspi / Bg)))
            if spi >= CH > 1:
                spi = max(CH, int(round(spi / CH)) * CH)
            tspi = spi * Bg
        model.output["actual_train_samples_per_iteration"] = tspi
        n_avg = 0

        def dp_average():
            """End of an iteration (DeepLearningTask.reduce + postGlobal): ONE all-reduce of [weights+biases,
            optimizer state] / W; elastic: the consensus time average (DeepLearningModelInfo.timeAverage)."""
            nonlocal n_avg
            if dp_local:          # H2O_DL_DP=local (tests): the per-rank local models, never averaged
                n_avg += 1
                return
            st = [fp.p] + ([fp.eg2, fp.edx2] if adaptive else [mom])
            buf = torch.cat(st)
            coll.all_reduce_(buf)
            buf.div_(Wn)
            n_avg += 1
            if elastic:
                if n_avg == 1:
                    ea.copy_(buf)
                else:
                    ea.mul_(1.0 - ea_pa).add_(buf, alpha=ea_pa)
                ea_on.fill_(1.0)
                return
            o = 0
            with torch.no_grad():
                for t_ in st:
                    t_.copy_(buf[o:o + t_.numel()])
                    o += t_.numel()
                if shadow is not None:
                    shadow.copy_(fp.p[: fp.n_decay])
                if fz.get("obj") is not None:
                    fz["obj"].refresh_transposed()

        def consensus_swap():
            """elastic: put the consensus weights in place for scoring; returns the local ones."""
            if not elastic or n_avg == 0:
                return None
            loc = fp.p.detach().clone()
            with torch.no_grad():
                fp.p.copy_(ea[: fp.p.numel()])
            return loc

        def local_restore(loc):
            if loc is not None:
                with torch.no_grad():
                    fp.p.copy_(loc)
        n_iter_done = 0
        step = 0
        spe = max(1, N_perm // B)
        t_loop0 = time.time()
        t_scoring = 0.0
        while step < total:
            if s_in >= S_ep:
                perm = torch.randperm(N_perm, generator=g, device=dev)
                s_in = 0
                if gsync:
                    mine = (perm >= row0) & (perm < row0 + N)
                    mine[S_ep * B:] = False
                    sel = torch.nonzero(mine).squeeze(1)
                    cnt = torch.bincount(sel // B, minlength=S_ep)[:S_ep].cpu()
                    offs = [0] + np.cumsum(cnt.numpy()).tolist()
                    cmax = int(cnt.max()) if S_ep > 0 else 0
                    if use_graph and cmax > gstate["cap"]:
                        alloc(max(64, (cmax + 63) // 64 * 64))
                elif use_graph and gstate["cap"] != B:
                    alloc(B)
            net.train()
            n = 1
            if (CH > 1 and gstate["warm"] >= 2 and chunk["g"] is not False and s_in + CH <= S_ep
                    and step + CH <= total and (not dp_avg or step % spi + CH <= spi)):
                net.step = step
                if run_chunk(perm[s_in * B:(s_in + CH) * B], step, samples):
                    n = CH
            if n == 1:
                if gsync:
                    rows = perm[sel[offs[s_in]:offs[s_in + 1]]] - row0
                else:
                    rows = perm[s_in * B:(s_in + 1) * B]
                net.step = step
                if not adaptive:
                    m = self._momentum(samples + Bg)
                    rate_t.fill_(float(p["rate"]) / (1 + float(p["rate_annealing"]) * (samples + Bg)))
                    mom_t.fill_(m)
                    on_t.fill_(1.0 if m > 0 else 0.0)
                if use_graph:
                    c = rows.numel()
                    if fz.get("obj") is not None:
                        fz["sridx"][:c].copy_(rows)
                        if c < fz["sridx"].numel():
                            fz["sridx"][c:].fill_(-1)
                    else:
                        torch.index_select(Z, 0, rows, out=sx[:c])
                        torch.index_select(wf, 0, rows, out=sw[:c])
                        if c < sw.numel():
                            sw[c:].zero_()
                        if sy is not None:
                            torch.index_select(yt, 0, rows, out=sy[:c])
                    step_t.fill_(step)
                    run_step()
                else:
                    fwd_bwd(Z.index_select(0, rows), wf.index_select(0, rows), None if ae else yt.index_select(0, rows))
                    if gsync:
                        coll.all_reduce_(gbuf)
                    update()
            s_in += n
            samples += n * Bg
            last = step + n - 1
            if self.job is not None and (step // 50) != ((last + 1) // 50):
                self.job.set_progress(last / max(total, 1))
            end = last == total - 1
            it_end = samples // tspi > n_iter_done          # an iteration of tspi samples completed
            first_it = it_end and n_iter_done == 0
            if it_end:
                n_iter_done = samples // tspi
            timed = it_end and time.time() - last_score > float(p["score_interval"])
            # every rank must take the same scoring decision. The collective runs only at iteration ends: ranks
            # may take different step paths (a graph chunk of CH steps vs single steps, from rank-local shard
            # sizes / epoch boundaries / capture success), so the number of loop turns differs per rank, but a
            # chunk never straddles an iteration end (spi is a multiple of CH), so every rank sees it_end at the
            # same global step and issues the same sequence of collectives (agree, then dp_average)
            if sharded and it_end:
                timed = coll.agree(timed)
            step = last + 1
            if dp_avg and (it_end or end):
                dp_average()
            if end or timed or first_it:
                last_score = time.time()
                loc = consensus_swap()
                ev = self._score(model, X, y, w, samples / N_glob, valid)
                t_scoring += time.time() - last_score
                history.append({k: v for k, v in ev.items() if not k.startswith("_")})
                last_ev = ev
                if owb:
                    lv = self._model_loss(ev.get("_valid") or ev.get("_train"), cat, ae)
                    if lv < best_loss:     # DeepLearningModel.doScoring: keep the lowest-loss weights
                        best_loss, best_p, best_ev = lv, fp.p.detach().clone(), ev
                local_restore(loc)
                mref = ev.get("_valid") or ev.get("_train")
                if mref is not None and not end and keeper.add(mref):
                    break
                if not end and not ae and self._accuracy_reached(ev.get("_train"), cat):
                    model.output["stopped_early"] = "achieved requested predictive accuracy on the training data"
                    break
                if float(p["max_runtime_secs"] or 0) > 0 and coll.agree(time.time() - t0 > float(p["max_runtime_secs"])):
                    break
        model.output["training_step_explicit"] = bool(explicit)
        model.output["mini_batch_rows"] = int(B)           # rows per optimizer step (see the default rule above)
        model.output["training_step_fused_mfma"] = fz.get("obj") is not None
        model.output["phase_seconds"] = dict(setup=t_loop0 - t0, train_loop=time.time() - t_loop0 - t_scoring,
                                             scoring=t_scoring)
        model.output["training_step_mode"] = (
            "eager" if not use_graph else
            ("graph_chunk%d" % CH if chunk.get("g") not in (None, False) else
             ("graph_step" if gstate.get("g1") not in (None, False) else "eager (" + str(gstate.get("error") or chunk.get("error")) + ")")))
        net.step_dev = None
        if elastic and n_avg:               # the consensus is the model (DeepLearningTask.postGlobal)
            with torch.no_grad():
                fp.p.copy_(ea[: fp.p.numel()])
        model.output["data_parallel"] = ("model_averaging" + ("_elastic" if elastic else "")) if dp_avg else (
            "gradient_sync" if gsync else None)
        model.output["averaging_rounds"] = n_avg
        final_ev = last_ev
        if owb and best_p is not None:
            final = self._model_loss(last_ev.get("_valid") or last_ev.get("_train"), cat, ae)
            if best_loss < final:
                with torch.no_grad():
                    fp.p.copy_(best_p)
                model.output["best_model_loss"] = best_loss
                final_ev = best_ev
        model.output["scoring_history"] = history
        model.output["epochs"] = prev_epochs + samples / N_glob
        # DeepLearningModel.doScoring: the model's training / validation metrics are those of its scoring
        # event — on the score_training_samples sample (0 = every row) — not an extra pass over all rows
        t_fm = time.time()
        if final_ev.get("_train") is not None:
            model.output["training_metrics"] = final_ev["_train"]
        elif ae:
            model.output["training_metrics"] = self._ae_metrics(model, X)
        else:
            model.output["training_metrics"] = model.metrics_for(X, y, w.float())
        if valid is not None and not ae:
            if final_ev.get("_valid") is not None:
                model.output["validation_metrics"] = final_ev["_valid"]
            else:
                Xv, yv, wv, ov = valid
                model.output["validation_metrics"] = model.metrics_for(Xv, yv, wv, ov)
        model.output["phase_seconds"]["final_metrics"] = time.time() - t_fm
        self._score_rows = None
        # Gedeon variable importance from the first layer weights
        W1 = net.hidden[0].weight.detach().abs() if net.hidden else net.out.weight.detach().abs()
        imp = W1.sum(0).double()
        agg = {}
        for nme, v in zip(ex.names, imp.cpu().tolist()):
            base_n = nme.split(".")[0] if nme not in info.x else nme
            agg[base_n] = agg.get(base_n, 0.0) + v
        from .base import variable_importance
        model.output["variable_importances"] = variable_importance(list(agg), list(agg.values()))
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model

    @staticmethod
    def _initial_state(net, p, hidden, n_in, dev):
        """``pretrained_autoencoder`` (hidden layers copied from an autoencoder of the same shape,
        DeepLearning.java pretrained AE), ``initial_weights`` / ``initial_biases`` (one frame per layer:
        weights [units out x units in], biases [units out x 1])."""
        from ..core import dkv
        lins = list(net.hidden) + [net.out]

        def resolve(ref):
            if ref is None:
                return None
            obj = dkv.get(ref) if isinstance(ref, str) else ref
            return getattr(obj, "_model", obj)

        pa = resolve(p.get("pretrained_autoencoder"))
        if p.get("pretrained_autoencoder"):
            if pa is None or getattr(pa, "net", None) is None or not pa.params.get("autoencoder"):
                raise ValueError(f"pretrained_autoencoder {p['pretrained_autoencoder']} is not a DeepLearning autoencoder")
            if list(pa._cfg["hidden"]) != list(hidden) or pa._cfg["n_in"] != n_in:
                raise ValueError("pretrained_autoencoder: hidden layers / input width differ from this model's")
            with torch.no_grad():
                for a, b in zip(net.hidden, pa.net.hidden):
                    a.weight.copy_(b.weight.to(dev))
                    a.bias.copy_(b.bias.to(dev))

        def mats(key):
            refs = p.get(key)
            if not refs:
                return None
            if len(refs) != len(lins):
                raise ValueError(f"{key} needs {len(lins)} frames (one per layer), got {len(refs)}")
            out = []
            for r in refs:
                fr = dkv.get(r) if isinstance(r, str) else r
                fr = getattr(fr, "_frame", fr)
                if fr is None:
                    raise ValueError(f"{key}: frame {r!r} not found")
                out.append(torch.as_tensor(fr.as_data_frame().to_numpy(dtype=np.float64)))
            return out

        W, Bs = mats("initial_weights"), mats("initial_biases")
        with torch.no_grad():
            for i, lin in enumerate(lins):
                if W is not None:
                    if tuple(W[i].shape) != tuple(lin.weight.shape):
                        raise ValueError(f"initial_weights[{i}] must be {tuple(lin.weight.shape)}, got {tuple(W[i].shape)}")
                    lin.weight.copy_(W[i].to(lin.weight))
                if Bs is not None:
                    if Bs[i].numel() != lin.bias.numel():
                        raise ValueError(f"initial_biases[{i}] must have {lin.bias.numel()} values")
                    lin.bias.copy_(Bs[i].reshape(-1).to(lin.bias))

    def _model_loss(self, m, cat, ae) -> float:
        """hex/Model.java loss(): the stopping metric, or logloss / MSE (autoencoder) / deviance."""
        if m is None:
            return float("inf")
        sm = str(self.p.get("stopping_metric") or "AUTO").lower()
        key = {"mse": "MSE", "rmse": "RMSE", "mae": "mae", "rmsle": "rmsle", "logloss": "logloss",
               "deviance": "mean_residual_deviance", "misclassification": "err", "mean_per_class_error": "mean_per_class_error"}.get(sm)
        if sm in ("auc", "aucpr"):
            v = m.get("AUC" if sm == "auc" else "pr_auc")
            return float("inf") if v is None else 1.0 - float(v)
        if key is None:
            key = "logloss" if cat in ("Binomial", "Multinomial") else ("MSE" if ae else "mean_residual_deviance")
        v = m.get(key)
        if v is None and key == "mean_residual_deviance":
            v = m.get("MSE")
        if v is None and key == "err":
            cm = m.get("mean_per_class_error")
            v = cm
        return float("inf") if v is None else float(v)

    def _momentum(self, samples):
        p = self.p
        ms, mr, mst = float(p["momentum_start"]), float(p["momentum_ramp"]), float(p["momentum_stable"])
        if samples >= mr:
            return mst
        return ms + (mst - ms) * samples / mr

    def _loss(self, out, target, w, cat, dist, ae):
        p = self.p
        lname = str(p["loss"]).lower()
        if ae:
            return (w[:, None] * (out - target.float()) ** 2).sum() / out.shape[1]
        if cat in ("Binomial", "Multinomial"):
            return (w * torch.nn.functional.cross_entropy(out, target, reduction="none")).sum()
        f = out[:, 0]
        t = target
        if lname == "absolute" or dist == "laplace":
            return (w * (f - t).abs()).sum()
        if lname == "quantile" or dist == "quantile":
            a = float(p["quantile_alpha"])
            r = t - f
            return (w * torch.where(r >= 0, a * r, (a - 1) * r)).sum()
        if lname == "huber" or dist == "huber":
            d = self._hdelta if hasattr(self, "_hdelta") else torch.ones((), device=f.device)
            a = (f - t).abs()
            return (w * torch.where(a <= d, 0.5 * a * a, d * (a - 0.5 * d))).sum()
        if dist == "poisson":
            return (w * (torch.exp(f) - t * f)).sum()
        if dist == "gamma":
            return (w * (t * torch.exp(-f) + f)).sum()
        if dist == "tweedie":
            r = float(p["tweedie_power"])
            return (w * (-t * torch.exp((1 - r) * f) / (1 - r) + torch.exp((2 - r) * f) / (2 - r))).sum()
        return 0.5 * (w * (f - t) ** 2).sum()

    def _accuracy_reached(self, m, cat) -> bool:
        """DeepLearningModel.doScoring: stop once the training classification error <= classification_stop
        (classifiers) or the training MSE <= regression_stop (regression); -1 disables either."""
        if m is None:
            return False
        p = self.p
        if cat in ("Binomial", "Multinomial"):
            cs = float(p.get("classification_stop", 0.0))
            if cs < 0:
                return False
            tab = (m.get("cm") or {}).get("table")
            if not tab:
                return False
            t = np.asarray(tab, dtype=np.float64)
            tot = t.sum()
            err = (tot - np.trace(t)) / tot if tot > 0 else 1.0
            return err <= cs
        rs = float(p.get("regression_stop", 1e-6))
        return rs >= 0 and m.get("MSE") is not None and float(m["MSE"]) <= rs

    def _ae_metrics(self, model, X):
        out, Z = model._forward(X)
        return mm.autoencoder_metrics(((out.float() - Z.float()) ** 2).mean(1))

    def _score(self, model, X, y, w, epochs, valid):
        p = self.p
        N = X.shape[1]
        Ng, r0 = getattr(self, "_N_glob", N), getattr(self, "_row0", 0)
        n = int(p["score_training_samples"]) or Ng
        key = (N, Ng, r0, n)
        cached = getattr(self, "_score_idx", None)
        if cached is not None and cached[0] == key:
            idx = cached[1]          # the same seeded sample at every scoring event
        elif n >= Ng:
            idx = torch.arange(N, device=X.device)
        else:
            # MRUtils.sampleFrame: every GLOBAL row kept with probability n / N (counter-based per-row uniforms:
            # the same rows however the frame is sharded; no device randperm / sort of the whole frame)
            from ..parallel import collectives as _c
            u = _c.row_uniform(int(p.get("seed") or 0), 0x5C0BE, r0, N, X.device)
            idx = torch.nonzero(u < n / Ng).squeeze(1)
        # the sampled rows are gathered once per fit (X, y and w do not change while it trains)
        samp = getattr(self, "_score_rows", None)
        if samp is None or samp[0] != key or samp[1] != (X.data_ptr(), tuple(X.shape)):
            samp = (key, (X.data_ptr(), tuple(X.shape)), X[:, idx], None if y is None else y[idx], w[idx].float())
            self._score_rows = samp
        self._score_idx = (key, idx)
        Xs, ys, ws = samp[2], samp[3], samp[4]
        ev = dict(epochs=epochs, timestamp=time.time())
        if p["autoencoder"]:
            m = self._ae_metrics(model, Xs)
        else:
            m = model.metrics_for(Xs, ys, ws)
            if self._dist == "huber" and hasattr(self, "_hdelta"):
                from .quantile import weighted_quantiles
                r = (ys.double() - model._predict_tensor(Xs).reshape(-1).double()).abs()
                dq = float(weighted_quantiles(r, [float(p["huber_alpha"])], w=w[idx])[0])
                if math.isfinite(dq):
                    self._hdelta.fill_(dq)
        ev["_train"] = m
        for k in ("RMSE", "logloss", "AUC", "mean_per_class_error", "MSE"):
            if m is not None and k in m:
                ev["training_" + k.lower()] = m[k]
        if valid is not None and not p["autoencoder"]:
            Xv, yv, wv, ov = valid
            nv = int(p.get("score_validation_samples") or 0)
            if 0 < nv < Xv.shape[1]:        # score_validation_samples: a fixed random subset of the validation rows
                vi = torch.randperm(Xv.shape[1], generator=torch.Generator().manual_seed(
                    (int(p.get("seed") or 0) + 1) & 0x7FFFFFFF))[:nv].to(Xv.device)
                Xv, yv = Xv[:, vi], yv[vi]
                wv = None if wv is None else wv[vi]
                ov = None if ov is None else ov[vi]
            vm = model.metrics_for(Xv, yv, wv, ov)
            ev["_valid"] = vm
            for k in ("RMSE", "logloss", "AUC", "mean_per_class_error"):
                if vm is not None and k in vm:
                    ev["validation_" + k.lower()] = vm[k]
        return ev
