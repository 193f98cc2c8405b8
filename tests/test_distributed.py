"""Multi-process (gloo, world_size=2) tests of the row-sharded distributed paths: histogram trees,
GLM Gram all-reduce, KMeans centroid all-reduce, DeepLearning gradient all-reduce. Each rank holds
half of the rows; the sharded model must equal the single-process model on the full data."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _data(N=3000, F=5, seed=0):
    g = torch.Generator().manual_seed(seed)
    X = torch.randn(F, N, generator=g)
    y = (torch.rand(N, generator=g) < torch.sigmoid(2 * X[0] - X[1] + 0.5 * X[2] * X[3])).float()
    return X, y


def _info(F):
    from llama_github_io_amd.models.base import DataInfo
    return DataInfo([f"x{i}" for i in range(F)], np.zeros(F, np.int32), [None] * F, "y", ["0", "1"])


def _train(algo, X, y, info):
    if algo == "gbm":
        from llama_github_io_amd.models.gbm import GBMTrainer
        m = GBMTrainer(dict(ntrees=4, max_depth=3, seed=7)).fit(X, y, None, None, info)
        return m.forest.predict_raw(_data()[0].to(X.device))[:, 0]
    if algo == "glm":
        from llama_github_io_amd.models.glm import GLMTrainer
        m = GLMTrainer(dict(family="binomial", lambda_=0.0)).fit(X, y, None, None, info)
        return m.beta[0].float()
    if algo == "kmeans":
        from llama_github_io_amd.models.base import DataInfo
        from llama_github_io_amd.models.kmeans import KMeansTrainer
        inf = DataInfo(info.x, info.iscat, info.domains, None, None)
        tr = KMeansTrainer(dict(k=3, seed=3, init="User", standardize=False,
                                user_points=np.array([[1, 0, 0, 0, 0], [-1, 0, 0, 0, 0], [0, 1, 0, 0, 0]], np.float32)))
        m = tr.fit(X, None, None, None, inf)
        return m.centers_std.flatten()
    raise ValueError(algo)


def _worker(rank, world, port, algo, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      H2O_AMD_DEVICE="cpu")
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        X, y = _data()
        N = X.shape[1]
        sl = slice(rank * N // world, (rank + 1) * N // world)
        out = _train(algo, X[:, sl].contiguous(), y[sl].contiguous(), _info(X.shape[0]))
        if rank == 0:
            q.put(out.numpy())
    finally:
        dist.destroy_process_group()


def _run(algo, world=2):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, algo, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return res


@pytest.mark.parametrize("algo", ["gbm", "glm", "kmeans"])
def test_sharded_equals_single(algo):
    X, y = _data()
    single = _train(algo, X, y, _info(X.shape[0])).numpy()
    sharded = _run(algo)
    tol = 1e-4 if algo != "glm" else 1e-5
    assert np.allclose(single, sharded, atol=tol, rtol=1e-4), (single[:5], sharded[:5])


def _hb_worker(rank, world, port, q):
    import time as _t
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      H2O_AMD_DEVICE="cpu", H2O_HEARTBEAT_S="0.1", H2O_HB_TIMEOUT_S="1.0")
    sys.path.insert(0, ROOT)
    from llama_github_io_amd.core import runtime
    from llama_github_io_amd.parallel import cluster
    runtime.init()
    _t.sleep(0.5)
    ok_before = cluster.healthy()
    if rank == 1:
        cluster.stop()          # rank 1 goes silent (simulated node loss)
        _t.sleep(3)
        q.put(("r1", True))
        return
    _t.sleep(2.5)
    q.put(("r0", (ok_before, cluster.healthy(), cluster.status()["dead"])))


def test_heartbeat_failure_detection():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_hb_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(30)
        if p.is_alive():
            p.kill()
    ok_before, ok_after, dead = res["r0"]
    assert ok_before and not ok_after and dead == [1]


def _oom_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      H2O_AMD_DEVICE="cpu")
    sys.path.insert(0, ROOT)
    import time as _t
    import torch.distributed as dist
    from llama_github_io_amd.parallel import collectives as coll
    from llama_github_io_amd.utils import memory
    dist.init_process_group("gloo", rank=rank, world_size=world)

    def build():
        if rank == 1:                       # one rank runs out of device memory inside the sharded build
            _t.sleep(0.5)
            raise torch.cuda.OutOfMemoryError("simulated: HIP out of memory")
        t = torch.ones(8)
        coll.all_reduce_(t)                 # its peer is waiting in the build's next collective
        return t
    t0 = _t.time()
    try:
        memory.with_backpressure(build)
        q.put((rank, "returned", _t.time() - t0))
    except Exception as e:  # noqa: BLE001
        q.put((rank, type(e).__name__, _t.time() - t0))


def test_oom_in_sharded_build_fails_every_rank_fast():
    """utils/memory.with_backpressure under row sharding: an OOM on one rank aborts the process group,
    so its peer leaves the pending collective with an error instead of hanging (no one-sided retry)."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_oom_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(30)
    assert res[0][1] != "returned" and res[1][1] == "RuntimeError", res
    assert all(r[2] < 30 for r in res), res


def _metrics_inputs(n=5000, seed=5):
    g = torch.Generator().manual_seed(seed)
    yb = (torch.rand(n, generator=g) < 0.4).double()
    p1 = torch.sigmoid(2 * yb - 1 + torch.randn(n, generator=g))
    w = torch.rand(n, generator=g) + 0.5
    yr = torch.randn(n, generator=g) * 3
    pr = yr + torch.randn(n, generator=g)
    K = 4
    y3 = torch.randint(0, K, (n,), generator=g)
    logits = torch.randn(n, K, generator=g) + 1.5 * torch.nn.functional.one_hot(y3, K)
    probs = torch.softmax(logits, 1).double()
    score = torch.rand(n, generator=g)
    return yb, p1, w, yr, pr, y3, probs, score


def _all_metrics(sl):
    from llama_github_io_amd import metrics as M
    yb, p1, w, yr, pr, y3, probs, score = (t[sl] for t in _metrics_inputs())
    b = M.binomial_metrics(yb, p1, w)
    r = M.regression_metrics(yr, pr, w)
    m = M.multinomial_metrics(y3, probs, w, domain=["a", "b", "c", "d"])
    a = M.anomaly_metrics(score)
    return dict(auc=b["AUC"], aucpr=b["pr_auc"], logloss=b["logloss"], mse=b["MSE"], mpce=b["mean_per_class_error"],
                thr=[r_["threshold"] for r_ in b["thresholds_and_metric_scores"]],
                lift=[g_["cumulative_lift"] for g_ in b["gains_lift_table"]],
                rmse=r["RMSE"], mae=r["mae"], r2=r["r2"], rmsle=r["rmsle"], mlogloss=m["logloss"], mauc=m["AUC"],
                mpce3=m["mean_per_class_error"], hits=m["hit_ratio_table"], cm=m["cm"]["table"],
                ascore=a["mean_score"], n=b["nobs"])


def _metrics_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from llama_github_io_amd.parallel import collectives as coll
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        n = _metrics_inputs()[0].numel()
        coll.stats(reset=True)
        out = _all_metrics(slice(rank * n // world, (rank + 1) * n // world))
        out["row_gathers"] = coll.stats()["row_gathers"]
        if rank == 0:
            q.put(out)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_metrics_merge_without_row_gathers(world):
    """Metrics of row-sharded predictions merge per-rank sufficient statistics (AUC2-style fixed score
    lattice, weighted sums, confusion matrix) — no collective ever gathers a row tensor — and match the
    single-process metrics (AUC within the lattice resolution)."""
    import socket
    single = _all_metrics(slice(None))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_metrics_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert out.pop("row_gathers") == 0
    for k in ("auc", "aucpr", "mauc"):
        assert abs(out[k] - single[k]) < 2e-5, (k, out[k], single[k])
    for k in ("logloss", "mse", "mpce", "rmse", "mae", "r2", "rmsle", "mlogloss", "mpce3", "ascore"):
        assert (out[k] != out[k] and single[k] != single[k]) or \
            abs(out[k] - single[k]) <= 1e-12 * max(1.0, abs(single[k])), (k, out[k], single[k])
    assert out["n"] == single["n"]
    assert np.allclose(out["thr"], single["thr"], rtol=0, atol=0) and np.allclose(out["lift"], single["lift"], rtol=1e-12)
    assert np.allclose(out["hits"], single["hits"], rtol=1e-12) and np.allclose(out["cm"], single["cm"], rtol=1e-12)


def _w2v_tokens():
    rng = np.random.default_rng(0)
    A, B = ["cat", "dog", "cow", "pig"], ["one", "two", "six", "ten"]
    words = []
    for i in range(1600):
        words += list(rng.choice(A if i % 2 else B, 6)) + [None]
    return words, A, B


def _w2v_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from llama_github_io_amd.models.base import DataInfo
    from llama_github_io_amd.models.word2vec import Word2VecTrainer
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        words, A, B = _w2v_tokens()
        n = len(words)
        local = words[rank * n // world:(rank + 1) * n // world]
        tr = Word2VecTrainer(dict(vec_size=10, min_word_freq=1, epochs=5, seed=1, sent_sample_rate=0, window_size=3))
        m = tr.fit_strings(np.array(local, dtype=object), DataInfo(["w"], np.zeros(1, np.int32), [None], None, None))
        vec = {w: m.vectors[i].double().numpy() for w, i in m.vocab.items()}
        cos = lambda a, b: float(vec[a] @ vec[b] / np.linalg.norm(vec[a]) / np.linalg.norm(vec[b]))  # noqa: E731
        within = np.mean([cos(a, b) for g in (A, B) for a in g for b in g if a < b])
        across = np.mean([cos(a, b) for a in A for b in B])
        q.put((rank, sorted(m.vocab), within, across, float(m.vectors.sum())))
    finally:
        dist.destroy_process_group()


def test_word2vec_sharded_text_trains_one_model():
    """Word2Vec over row-sharded text (WordVectorTrainer MRTask): merged vocabulary, per-epoch model
    averaging; every rank ends with the same vectors, and co-occurring words are nearer."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_w2v_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(2)])
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    (_, v0, w0, a0, s0), (_, v1, w1, a1, s1) = out
    assert v0 == v1 and abs(s0 - s1) < 1e-6
    assert w0 > a0 + 0.3, (w0, a0)


def _x2_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch
    import torch.distributed as dist
    from llama_github_io_amd.parallel import collectives as coll
    from llama_github_io_amd.parallel.order_stats import order_statistics
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(rank)
        n = 50 + 37 * rank                             # uneven shards
        v = torch.randn(n, generator=g, dtype=torch.float64)
        ids = torch.arange(n, dtype=torch.float64) + 1000 * rank
        # range partition by exact splitters (the isotonic / concordance pattern)
        tot = int(coll.all_reduce_(torch.tensor([float(n)], dtype=torch.float64)).item())
        spl = torch.tensor(order_statistics(v, [k * tot // world + 1 for k in range(1, world)]), dtype=torch.float64)
        dest = torch.searchsorted(spl, v.contiguous(), right=True)
        got = coll.exchange_rows(torch.stack([v, ids], 1), dest)
        parts = coll.all_gather_object(got.tolist())
        if rank == 0:
            q.put(dict(parts=parts, spl=spl.tolist()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_rows_range_partition(world):
    """collectives.exchange_rows (variable all-to-all): each row moves once, to the rank owning its key range;
    rows arrive grouped by source rank in their original order; nothing is lost or duplicated."""
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_x2_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    parts, spl = out["parts"], out["spl"]
    allrows = [r for part in parts for r in part]
    assert len(allrows) == sum(50 + 37 * r for r in range(world))
    assert len({r[1] for r in allrows}) == len(allrows)
    for k, part in enumerate(parts):                   # rank k holds exactly the keys of range k
        lo = -np.inf if k == 0 else spl[k - 1]
        hi = np.inf if k == world - 1 else spl[k]
        assert all(lo <= r[0] < hi for r in part)
        src = [int(r[1]) // 1000 for r in part]
        assert src == sorted(src)                       # grouped by source rank
        for sr in set(src):
            ids = [r[1] for r in part if int(r[1]) // 1000 == sr]
            assert ids == sorted(ids)                   # source order kept


def _impute_worker(rank, world, port, csv, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), H2O_AMD_DEVICE="cpu", OMP_NUM_THREADS="1")
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import h2o
    import torch.distributed as dist
    h2o.init()
    try:
        fr = h2o.import_file(csv)
        assert fr._shard is not None
        fr.impute("x", "mean", by=["g", "h"])
        fr.impute("e", "mode", by=["h"])
        df = fr.as_data_frame()
        if rank == 0:
            q.put(dict(x=df["x"].tolist(), e=df["e"].astype(str).tolist()))
    finally:
        if dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()


def test_sharded_group_impute_equals_single(tmp_path):
    """h2o.impute with groupByCols on a row-sharded frame (gloo world 2): the key / target columns are gathered,
    aggregated once, and each rank fills its own rows — equal to the single-process result."""
    import socket
    import pandas as pd
    rng = np.random.default_rng(11)
    n = 2000
    df = pd.DataFrame({"g": rng.choice(["a", "b", "c"], n), "h": rng.integers(0, 3, n),
                       "x": rng.normal(size=n).round(4), "e": rng.choice(["u", "v", "w"], n)})
    df.loc[rng.random(n) < 0.2, "x"] = np.nan
    df.loc[rng.random(n) < 0.2, "e"] = None
    csv = tmp_path / "imp.csv"
    df.to_csv(csv, index=False)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_impute_worker, args=(r, 2, port, str(csv), q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=300)
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    from llama_github_io_amd.frame import H2OFrame
    single = H2OFrame(pd.read_csv(csv), destination_frame="imp_single")
    single["g"] = single["g"].asfactor() if single.type("g") != "enum" else single["g"]
    single.impute("x", "mean", by=["g", "h"])
    single.impute("e", "mode", by=["h"])
    sd = single.as_data_frame()
    np.testing.assert_allclose(np.asarray(out["x"], dtype=float), sd["x"].to_numpy(dtype=float), rtol=1e-12)
    assert out["e"] == sd["e"].astype(str).tolist()
