"""Word2Vec (reference: ``hex/word2vec/Word2Vec.java``, ``Word2VecModel.java``, ``WordVectorTrainer.java``).

Skip-gram or CBOW (``word_model``) with hierarchical softmax (H2O's only ``norm_model``): vocabulary from the training
string column (NA rows separate sentences), words below ``min_word_freq`` dropped, frequent words
sub-sampled with ``sent_sample_rate``, a Huffman tree over counts gives each word its path
(inner-node ids + binary codes). Training is batched on device: (center, context) pairs of a
window of random width ≤ ``window_size`` are gathered per epoch and every pair updates the
context vector and the inner-node vectors along the center's Huffman path (padded path tensors,
one masked logistic loss per batch, SGD with linear learning-rate decay as in the reference).
API: ``find_synonyms(word, count)``, ``transform(frame, aggregate_method)``, ``to_frame()``.
"""
from __future__ import annotations

import heapq
import math
import time
from collections import Counter

import numpy as np
import torch

from .base import DataInfo, Model, make_key

W2V_DEFAULTS = dict(vec_size=100, window_size=5, sent_sample_rate=1e-3, norm_model="HSM", epochs=5, min_word_freq=5,
                    init_learning_rate=0.025, word_model="SkipGram", seed=-1, pre_trained=None, batch_pairs=65536)


def huffman(counts):
    """Codes and inner-node paths for each word (word2vec.c CreateBinaryTree)."""
    V = len(counts)
    heap = [(int(c), i) for i, c in enumerate(counts)]
    heapq.heapify(heap)
    parent = {}
    code_bit = {}
    nxt = V
    while len(heap) > 1:
        c1, a = heapq.heappop(heap)
        c2, b = heapq.heappop(heap)
        parent[a], code_bit[a] = nxt, 0
        parent[b], code_bit[b] = nxt, 1
        heapq.heappush(heap, (c1 + c2, nxt))
        nxt += 1
    root = heap[0][1] if heap else 0
    paths, codes = [], []
    for w in range(V):
        pth, cd = [], []
        n = w
        while n != root and n in parent:
            cd.append(code_bit[n])
            pth.append(parent[n] - V)
            n = parent[n]
        paths.append(pth[::-1])
        codes.append(cd[::-1])
    return paths, codes, max(1, nxt - V)


class Word2VecModel(Model):
    algo = "word2vec"

    def __init__(self, key, params, info):
        super().__init__(key, params, info)
        self.output["model_category"] = "WordEmbedding"

    @property
    def model_category(self):
        return "WordEmbedding"

    def _predict_tensor(self, X, offset=None):
        raise NotImplementedError("use transform()")

    def find_synonyms(self, word, count=20):
        if word not in self.vocab:
            return {}
        V = self.vectors
        v = V[self.vocab[word]]
        sims = (V @ v) / (V.norm(dim=1) * v.norm()).clamp(min=1e-12)
        sims[self.vocab[word]] = -2
        top = torch.topk(sims, min(count, len(self.words) - 1))
        return {self.words[i]: float(s) for s, i in zip(top.values.tolist(), top.indices.tolist())}

    def transform(self, words, aggregate_method="NONE"):
        from ..frame import H2OFrame
        toks = words._col(0).to_numpy()
        D = self.vectors.shape[1]
        out = []
        cur = []
        for t in list(toks) + [None]:
            if t is None or (isinstance(t, float) and math.isnan(t)):
                if aggregate_method.upper() == "AVERAGE":
                    out.append(torch.stack(cur).mean(0) if cur else torch.full((D,), float("nan")))
                cur = []
                if aggregate_method.upper() != "AVERAGE" and t is None and len(out) < len(toks):
                    out.append(torch.full((D,), float("nan")))
                continue
            vec = self.vectors[self.vocab[t]].cpu() if t in self.vocab else torch.full((D,), float("nan"))
            if aggregate_method.upper() == "AVERAGE":
                if t in self.vocab:
                    cur.append(vec)
            else:
                out.append(vec)
        M = torch.stack(out[: len(toks)] if aggregate_method.upper() != "AVERAGE" else out)
        return H2OFrame.from_tensor(M.float(), [f"C{i + 1}" for i in range(D)])

    def to_frame(self):
        from ..frame import Column, H2OFrame
        cols = [Column("Word", "string", strings=np.array(self.words, dtype=object))]
        V = self.vectors.double()
        cols += [Column(f"V{i + 1}", "real", V[:, i]) for i in range(V.shape[1])]
        return H2OFrame._from_columns(cols)

    def to_state(self):
        s = super().to_state()
        s["words"] = self.words
        s["vectors"] = self.vectors.cpu().tolist()
        return s

    def _restore(self, s):
        super()._restore(s)
        self.words = s["words"]
        self.vocab = {w: i for i, w in enumerate(self.words)}
        self.vectors = torch.tensor(s["vectors"], dtype=torch.float32)


MAX_EXP = 6.0   # WordVectorTrainer.MAX_EXP: dot products beyond +-6 skip the update (saturated sigmoid)


class Word2VecTrainer:
    def __init__(self, params):
        p = dict(W2V_DEFAULTS)
        p.update({k: v for k, v in params.items() if v is not None})
        self.p = p
        self.job = None
        self.strings = None    # the builder passes the raw string column via fit_strings

    def from_pretrained(self, frame, model_key=None):
        """Word2Vec.java pre-trained mode: a frame of [word (string/enum), v1 .. vD (numeric)] becomes the
        embedding as is."""
        from ..core import dkv
        fr = dkv.get(frame) if isinstance(frame, str) else frame
        fr = getattr(fr, "_frame", fr)
        if fr is None or fr.ncols < 2:
            raise ValueError("pre_trained needs a frame of a word column followed by the vector columns")
        wc = fr._col(fr.names[0])
        if fr.type(fr.names[0]) == "enum":
            words = [wc.domain[int(c)] for c in wc.data.cpu().tolist()]
        else:
            words = [str(v) for v in wc.to_numpy()]
        V = torch.stack([fr._col(n).as_float().double() for n in fr.names[1:]], 1).float()
        info = DataInfo([fr.names[0]], np.zeros(1, np.int32), [None], None, None)
        m = Word2VecModel(model_key or make_key("word2vec"), dict(self.p, vec_size=V.shape[1]), info)
        m.words = words
        m.vocab = {w_: i for i, w_ in enumerate(words)}
        m.vectors = V
        m.output["model_category"] = "WordEmbedding"
        m.output["vec_size"] = V.shape[1]
        m.output["vocab_size"] = len(words)
        return m

    def _cbow_epoch(self, ids, counts, total, ss, win, rng, gen, syn0, syn1, P_idx, P_code, P_mask, lr0, B, step,
                    n_steps_est, epochs, dev):
        """One CBOW epoch (WordVectorTrainer.map / CBOW / hierarchicalSoftmaxCBOW), batched on the device:
        every center word's context bag (random window shrink b <= window_size, sentence-bounded) is
        averaged into neu1, the center's Huffman path is trained against neu1 (updates skipped where
        |neu1 . syn1| >= MAX_EXP), and the accumulated error neu1e is added to the input vectors of the
        context words the reference updates: its hidden -> in loop runs over window slots
        [b, window_size] only, i.e. the LEFT part of the bag."""
        D = syn0.shape[1]
        cen, ctx, left = [], [], []
        for s in ids:
            if ss > 0 and len(s):
                f = counts[s] / total
                keep = (np.sqrt(f / ss) + 1) * ss / f
                s = s[rng.random(len(s)) < keep]
            n = len(s)
            if n < 2:
                continue
            b = rng.integers(0, win, n)
            pos = np.arange(n)
            X = np.full((n, 2 * win), -1, dtype=np.int64)
            Lm = np.zeros((n, 2 * win), dtype=bool)
            col = 0
            for off in range(-win, win + 1):
                if off == 0:
                    continue
                ok = (np.abs(off) <= win - b) & (pos + off >= 0) & (pos + off < n)
                X[ok, col] = s[pos[ok] + off]
                Lm[ok, col] = off < 0
                col += 1
            has = (X >= 0).any(1)
            cen.append(s[has])
            ctx.append(X[has])
            left.append(Lm[has])
        if not cen:
            return step, n_steps_est
        c = torch.from_numpy(np.concatenate(cen)).to(dev)
        X = torch.from_numpy(np.concatenate(ctx)).to(dev)
        Lm = torch.from_numpy(np.concatenate(left)).to(dev)
        perm = torch.randperm(c.numel(), generator=gen).to(dev)
        c, X, Lm = c[perm], X[perm], Lm[perm]
        if n_steps_est is None:
            n_steps_est = epochs * ((c.numel() + B - 1) // B)
        for s0 in range(0, c.numel(), B):
            cb, xb, lb = c[s0:s0 + B], X[s0:s0 + B], Lm[s0:s0 + B]
            lr = max(lr0 * (1 - step / max(n_steps_est, 1)), lr0 * 1e-4)
            step += 1
            valid = xb >= 0
            cnt = valid.sum(1).clamp(min=1).to(syn0.dtype)
            h = (syn0[xb.clamp(min=0)] * valid[:, :, None]).sum(1) / cnt[:, None]      # neu1 [b, D]
            nodes = P_idx[cb]
            u = syn1[nodes]                                                              # [b, L, D]
            dot = (u * h[:, None, :]).sum(-1)
            live = (dot > -MAX_EXP) & (dot < MAX_EXP)
            g = (1 - P_code[cb] - torch.sigmoid(dot)) * P_mask[cb] * live * lr
            neu1e = (g[:, :, None] * u).sum(1)
            syn1.index_add_(0, nodes.reshape(-1), (g[:, :, None] * h[:, None, :]).reshape(-1, D))
            upd = lb & valid
            rows = torch.nonzero(upd, as_tuple=True)
            syn0.index_add_(0, xb[rows], neu1e[rows[0]])
        return step, n_steps_est

    def fit(self, X, y, w, offset, info: DataInfo, valid=None, model_key=None):
        if self.strings is None:
            raise ValueError("word2vec trains from a string column (use the estimator API)")
        return self.fit_strings(self.strings, info, model_key, X.device)

    def fit_strings(self, toks, info, model_key=None, device=None):
        from .shared_tree import resolve_seed
        t0 = time.time()
        p = self.p
        dev = device or torch.device("cpu")
        seed = resolve_seed(p["seed"])
        rng = np.random.default_rng(seed & 0xFFFFFFFF)
        sents, cur = [], []
        for t in toks:
            if t is None or (isinstance(t, float) and math.isnan(t)):
                if cur:
                    sents.append(cur)
                cur = []
            else:
                cur.append(str(t))
        if cur:
            sents.append(cur)
        cnt = Counter(w for s in sents for w in s)
        from ..parallel import collectives as coll
        dist = coll.is_dist()
        if dist:
            # row-sharded text (WordVectorTrainer's MRTask over chunks): the vocabulary is the merged word
            # count of every rank (a summary bounded by the vocabulary, not the rows)
            merged = Counter()
            for c in coll.all_gather_object(dict(cnt)):
                merged.update(c)
            cnt = merged
        words = sorted([w for w, c in cnt.items() if c >= int(p["min_word_freq"])], key=lambda w: (-cnt[w], w))
        vocab = {w: i for i, w in enumerate(words)}
        V, D = len(words), int(p["vec_size"])
        if V < 2:
            raise ValueError("vocabulary too small (check min_word_freq)")
        counts = np.array([cnt[w] for w in words], dtype=np.float64)
        paths, codes, n_inner = huffman(counts)
        L = max(len(x) for x in paths)
        P_idx = torch.zeros(V, L, dtype=torch.long)
        P_code = torch.zeros(V, L)
        P_mask = torch.zeros(V, L)
        for i, (pth, cd) in enumerate(zip(paths, codes)):
            P_idx[i, :len(pth)] = torch.tensor(pth)
            P_code[i, :len(cd)] = torch.tensor(cd, dtype=torch.float32)
            P_mask[i, :len(pth)] = 1
        P_idx, P_code, P_mask = P_idx.to(dev), P_code.to(dev), P_mask.to(dev)
        gen = torch.Generator().manual_seed(seed & 0x7FFFFFFF)
        syn0 = ((torch.rand(V, D, generator=gen) - 0.5) / D).to(dev)
        syn1 = torch.zeros(n_inner, D, device=dev)
        total = counts.sum()
        ss = float(p["sent_sample_rate"])
        ids = [np.array([vocab[w] for w in s if w in vocab], dtype=np.int64) for s in sents]
        epochs = int(p["epochs"])
        lr0 = float(p["init_learning_rate"])
        win = int(p["window_size"])
        B = int(p["batch_pairs"])
        step, n_steps_est = 0, None
        cbow = str(p.get("word_model") or "SkipGram").lower() == "cbow"
        if str(p.get("word_model") or "SkipGram").lower() not in ("skipgram", "cbow"):
            raise ValueError(f"word_model must be SkipGram or CBOW, got {p.get('word_model')!r}")
        def sync():
            # WordVectorTrainer.reduce / postGlobal: each rank trained its own sentences this epoch; the
            # model is the average of the ranks' weights
            if dist:
                for t in (syn0, syn1):
                    t.copy_(coll.all_reduce_(t.contiguous().to(coll.comm_device())).to(t.device) / coll.world())
        for ep in range(epochs):
            if cbow:
                step, n_steps_est = self._cbow_epoch(ids, counts, total, ss, win, rng, gen, syn0, syn1, P_idx, P_code,
                                                     P_mask, lr0, B, step, n_steps_est, epochs, dev)
                sync()
                if self.job is not None:
                    self.job.set_progress((ep + 1) / epochs)
                continue
            centers, ctxs = [], []
            for s in ids:
                if ss > 0 and len(s):
                    f = counts[s] / total
                    keep = (np.sqrt(f / ss) + 1) * ss / f
                    s = s[rng.random(len(s)) < keep]
                n = len(s)
                if n < 2:
                    continue
                b = rng.integers(0, win, n)
                for off in range(-win, win + 1):
                    if off == 0:
                        continue
                    pos = np.arange(n)
                    ok = (np.abs(off) <= win - b) & (pos + off >= 0) & (pos + off < n)
                    centers.append(s[pos[ok]])
                    ctxs.append(s[pos[ok] + off])
            if not centers:
                sync()
                continue
            c = torch.from_numpy(np.concatenate(centers)).to(dev)
            x = torch.from_numpy(np.concatenate(ctxs)).to(dev)
            perm = torch.randperm(c.numel(), generator=gen).to(dev)
            c, x = c[perm], x[perm]
            if n_steps_est is None:
                n_steps_est = epochs * ((c.numel() + B - 1) // B)
            for s0 in range(0, c.numel(), B):
                cb, xb = c[s0:s0 + B], x[s0:s0 + B]
                lr = max(lr0 * (1 - step / max(n_steps_est, 1)), lr0 * 1e-4)
                step += 1
                h = syn0[xb]                                   # [b, D] context (input) vectors
                nodes = P_idx[cb]                              # [b, L]
                u = syn1[nodes]                                # [b, L, D]
                f = torch.sigmoid((u * h[:, None, :]).sum(-1))
                g = (1 - P_code[cb] - f) * P_mask[cb] * lr     # word2vec.c: g = (1 - code - f) * alpha
                dh = (g[:, :, None] * u).sum(1)
                du = g[:, :, None] * h[:, None, :]
                syn1.index_add_(0, nodes.reshape(-1), du.reshape(-1, D))
                syn0.index_add_(0, xb, dh)
            sync()
            if self.job is not None:
                self.job.set_progress((ep + 1) / epochs)
        model = Word2VecModel(model_key or make_key("word2vec"), p, info)
        model.device = dev
        model.words = words
        model.vocab = vocab
        model.vectors = syn0
        model.output.update(vocab_size=V, vec_size=D, epochs=epochs, word_model="CBOW" if cbow else "SkipGram")
        model.output["run_time_ms"] = int((time.time() - t0) * 1000)
        return model
