"""Data-parallel correctness on CPU ranks (gloo), SURVEY.md §7.5 "Distributed".

The DP pipeline (sharded rows; all-reduced scaler sums C1, all-gathered minority rows C3,
all-reduced Newton gradient/Hessian C5, gathered test scores for the exact AUC) must match the
single-process computation on the concatenated data."""
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir, smote, scope="global", zero_min_rank=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FDX_COMM_TRACE="1")
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig, evaluate
    from fraud_detection_amd.parallel.comm import Communicator

    comm = Communicator(backend="gloo")
    X, y = separable(24_000, fraud_rate=0.02, seed=100)
    Xt, yt = separable(8_000, fraud_rate=0.02, seed=200)
    sh = slice(rank * len(X) // world, (rank + 1) * len(X) // world)
    sht = slice(rank * len(Xt) // world, (rank + 1) * len(Xt) // world)
    cfg = TrainConfig(smote=smote, tol=1e-8, init_std=0.0, smote_scope=scope)
    Xs, ys = X[sh], y[sh]
    if rank == zero_min_rank:  # a shard without minority rows
        Xs, ys = Xs[ys == 0], ys[ys == 0]
    res = DevicePipeline(cfg, comm).fit(Xs.contiguous(), ys.contiguous())
    ev = evaluate(res, Xt[sht].contiguous(), yt[sht].contiguous(), comm)
    mean, var, scale = res.scaler.numpy()
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), w=res.w, mean=mean, var=var, auc=ev["auc"],
             n_train=res.n_train_rows, trace=np.array([f"{op}|{path}" for op, path, _ in comm.trace]),
             stats=np.array(json.dumps(comm.collective_summary())))
    comm.barrier()
    comm.close()


def _run(world, smote, tmp_path, scope="global", zero_min_rank=None):
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, str(tmp_path), smote, scope, zero_min_rank), nprocs=world,
                       start_method="spawn")
    return [dict(np.load(os.path.join(tmp_path, f"r{r}.npz"))) for r in range(world)]


@pytest.mark.parametrize("world", [2, 4])
def test_dp_matches_single_process_without_smote(tmp_path, world):
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig, evaluate

    outs = _run(world, False, tmp_path)
    X, y = separable(24_000, fraud_rate=0.02, seed=100)
    Xt, yt = separable(8_000, fraud_rate=0.02, seed=200)
    ref = DevicePipeline(TrainConfig(smote=False, tol=1e-8, init_std=0.0)).fit(X, y)
    ev = evaluate(ref, Xt, yt)
    for o in outs:  # every rank holds the same global model
        np.testing.assert_allclose(o["mean"], ref.scaler.numpy()[0], rtol=1e-10, atol=1e-9)
        np.testing.assert_allclose(o["var"], ref.scaler.numpy()[1], rtol=1e-8)
        np.testing.assert_allclose(o["w"], ref.w, atol=1e-7)
        assert float(o["auc"]) == pytest.approx(ev["auc"], abs=1e-6)
    assert np.array_equal(outs[0]["w"], outs[-1]["w"])


def test_dp_with_smote_balances_globally(tmp_path):
    outs = _run(2, True, tmp_path)
    assert np.array_equal(outs[0]["w"], outs[1]["w"])
    assert float(outs[0]["auc"]) > 0.9
    # the ranks together hold exactly the one-process post-SMOTE table: 2 * n_majority rows
    from fraud_detection_amd.data.synthetic import separable

    _, y = separable(24_000, fraud_rate=0.02, seed=100)
    assert sum(int(o["n_train"]) for o in outs) == 2 * int((y == 0).sum())


@pytest.mark.parametrize("world", [3, 8])
def test_dp_global_smote_equals_single_process(tmp_path, world):
    """8-rank readiness: the full pipeline with smote_scope="global" under DP equals
    the single-process fit -- identical synthetic rows (one global Philox draw sequence, sliced at
    128-aligned boundaries), so the weights agree up to the all-reduce summation order."""
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig, evaluate

    outs = _run(world, True, tmp_path)
    X, y = separable(24_000, fraud_rate=0.02, seed=100)
    Xt, yt = separable(8_000, fraud_rate=0.02, seed=200)
    ref = DevicePipeline(TrainConfig(smote=True, tol=1e-8, init_std=0.0)).fit(X, y)
    ev = evaluate(ref, Xt, yt)
    assert sum(int(o["n_train"]) for o in outs) == ref.n_train_rows
    for o in outs:
        np.testing.assert_allclose(o["w"], ref.w, atol=1e-7)
        assert float(o["auc"]) == pytest.approx(ev["auc"], abs=1e-6)


@pytest.mark.parametrize("ranks", [
    [[37, 5000], [0, 4000], [90, 6100], [12, 333], [5, 9000], [64, 4096], [1, 10], [40, 7777]],
    [[0, 10000], [10, 100]],          # the zero-minority rank used to overflow rank 1
    [[10, 100], [0, 10000]],
    [[500, 1000], [0, 3], [0, 0], [1, 129]],
])
def test_global_smote_slices_cover_the_quota(ranks):
    from fraud_detection_amd.models.pipeline import global_smote_slices

    ratio = 1.0
    quota = lambda n, m: max(0, int(round((n - m) * ratio)) - m) if m > 0 else 0  # noqa: E731
    per, offs = zip(*[global_smote_slices(ranks, quota, r) for r in range(len(ranks))])
    per = per[0]
    total = quota(sum(r[1] for r in ranks), sum(r[0] for r in ranks))
    assert sum(per) == total and all(p >= 0 for p in per)
    assert all(o % 128 == 0 for o in offs) and list(offs) == [sum(per[:r]) for r in range(len(ranks))]
    # every slice fits the training buffer the rank sized before the exchange (pipeline.fit: cap)
    for p, (_, n) in zip(per, ranks):
        assert p <= int(np.ceil(n * max(ratio, 1.0))) + 128
    # boundaries sit within 64 rows of the row-proportional cumulative shares
    n_g = sum(r[1] for r in ranks)
    cum = [total * int(c) // n_g for c in np.cumsum([r[1] for r in ranks])[:-1]]
    assert all(abs(o - c) <= 64 for o, c in zip(offs[1:], cum))


@pytest.mark.parametrize("scope", ["shard", "global"])
def test_dp_rank_without_minority_rows(tmp_path, scope):
    """a shard with no minority rows must neither raise nor hang its peers (shard
    scope: it skips SMOTE; global scope: it takes a slice of the global draw sequence)."""
    outs = _run(2, True, tmp_path, scope=scope, zero_min_rank=1)
    assert np.array_equal(outs[0]["w"], outs[1]["w"])
    assert float(outs[0]["auc"]) > 0.9
    if scope == "global":
        from fraud_detection_amd.data.synthetic import separable
        from fraud_detection_amd.models.pipeline import DevicePipeline, TrainConfig

        X, y = separable(24_000, fraud_rate=0.02, seed=100)
        h = len(X) // 2
        keep = torch.ones(len(X), dtype=torch.bool)
        keep[h:] = y[h:] == 0
        ref = DevicePipeline(TrainConfig(smote=True, tol=1e-8, init_std=0.0)).fit(X[keep].contiguous(),
                                                                                y[keep].contiguous())
        assert sum(int(o["n_train"]) for o in outs) == ref.n_train_rows
        np.testing.assert_allclose(outs[0]["w"], ref.w, atol=1e-7)


def _knn_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from fraud_detection_amd.ops import knn as K
    from fraud_detection_amd.parallel.comm import Communicator

    comm = Communicator(backend="gloo")
    rng = np.random.default_rng(0)
    C = np.zeros((90, 32), np.float32)
    C[:, :30] = rng.normal(size=(90, 30))
    mine = torch.from_numpy(C[rank * 30:(rank + 1) * 30])
    allc, counts = comm.all_gather_rows(mine)
    off = int(sum(counts[:rank]))
    nbr = K.knn_topk(mine, allc, k=5, self_offset=off)
    np.save(os.path.join(out_dir, f"knn{rank}.npy"), nbr.numpy())
    comm.close()


def test_dp_knn_equals_global(tmp_path):
    port = _free_port()
    mp.start_processes(_knn_worker, args=(3, port, str(tmp_path)), nprocs=3, start_method="spawn")
    from fraud_detection_amd.ops import reference as ref

    rng = np.random.default_rng(0)
    C = np.zeros((90, 32), np.float32)
    C[:, :30] = rng.normal(size=(90, 30))
    full, _ = ref.knn_topk(C, C, 5, 0)
    got = np.concatenate([np.load(os.path.join(tmp_path, f"knn{r}.npy")) for r in range(3)])
    assert np.array_equal(got, full)


def _gbdt_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from fraud_detection_amd.ops import gbdt as gb
    from fraud_detection_amd.parallel.comm import Communicator

    comm = Communicator(backend="gloo")
    X, y, cuts = _gbdt_data()
    sh = slice(rank * len(X) // world, (rank + 1) * len(X) // world)
    ens = gb.fit(torch.from_numpy(X[sh].copy()), torch.from_numpy(y[sh].copy()),
                 gb.GBDTParams(n_estimators=4, max_depth=3), comm=comm, cuts=cuts)
    np.savez(os.path.join(out_dir, f"g{rank}.npz"), feat=ens.feat, bin=ens.bin, leaf=ens.leaf)
    comm.close()


def _gbdt_data():
    from fraud_detection_amd.ops import reference_gbdt as R

    rng = np.random.default_rng(11)
    X = rng.normal(size=(3000, 5)).astype(np.float32)
    y = (X[:, 0] + 0.5 * X[:, 1] ** 2 + rng.normal(size=3000) > 1.2).astype(np.uint8)
    return X, y, R.quantile_cuts(X, 64)


def test_dp_gbdt_equals_single_process(tmp_path):
    """Histogram all-reduce (int64, exact) makes the DP trees bit-identical to one process."""
    port = _free_port()
    mp.start_processes(_gbdt_worker, args=(2, port, str(tmp_path)), nprocs=2, start_method="spawn")
    from fraud_detection_amd.ops import gbdt as gb

    X, y, cuts = _gbdt_data()
    ref = gb.fit(torch.from_numpy(X), torch.from_numpy(y), gb.GBDTParams(n_estimators=4, max_depth=3), cuts=cuts)
    for r in range(2):
        o = np.load(os.path.join(tmp_path, f"g{r}.npz"))
        assert np.array_equal(o["feat"], ref.feat) and np.array_equal(o["bin"], ref.bin)
        assert np.array_equal(o["leaf"], ref.leaf)


def _train_worker(rank, world, port, out_dir, csv):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DATA_CSV=csv, MLFLOW_TRACKING_URI=os.path.join(out_dir, "mlruns"),
                      MLFLOW_AUC_THRESHOLD="0.5", FDX_DEVICE="cpu")
    from fraud_detection_amd import train
    from fraud_detection_amd.config import Settings
    from fraud_detection_amd.parallel.comm import Communicator

    comm = Communicator(backend="gloo")
    out = train.run(Settings.load(), cv_folds=2, model_dir=os.path.join(out_dir, "models"), verbose=False, comm=comm)
    np.save(os.path.join(out_dir, f"auc{rank}.npy"), np.array([out["test_auc"]] + list(out["cv_scores"])))
    comm.close()


def test_dp_train_entry_point(tmp_path, monkeypatch):
    """torchrun-style DP training: both ranks report the same (global) AUCs, rank 0 alone writes
    artifacts, and the result matches single-process training to SMOTE sampling noise."""
    from fraud_detection_amd import train
    from fraud_detection_amd.config import Settings
    from fraud_detection_amd.data.synthetic import separable_frame

    csv = str(tmp_path / "cc.csv")
    separable_frame(30_000, fraud_rate=0.02, seed=8).to_csv(csv, index=False)
    port = _free_port()
    mp.start_processes(_train_worker, args=(2, port, str(tmp_path), csv), nprocs=2, start_method="spawn")
    a0, a1 = np.load(tmp_path / "auc0.npy"), np.load(tmp_path / "auc1.npy")
    assert np.array_equal(a0, a1)
    assert os.path.exists(tmp_path / "models" / "logistic_model.joblib")
    monkeypatch.setenv("DATA_CSV", csv)
    single = train.run(Settings.load(), cv_folds=2, model_dir=str(tmp_path / "single"), verbose=False)
    assert abs(single["test_auc"] - a0[0]) < 0.01
    # small folds run fold-parallel (whole folds per rank): CV scores equal the single-process ones
    assert np.allclose(a0[1:], single["cv_scores"], rtol=0, atol=1e-12)


def test_dp_shard_scope_smote(tmp_path):
    """Per-partition SMOTE (neighbours within each rank's minority rows): same balance and row
    counts as the global scope, one model on all ranks, comparable AUC."""
    outs = _run(2, True, tmp_path, scope="shard")
    assert np.array_equal(outs[0]["w"], outs[1]["w"])
    assert float(outs[0]["auc"]) > 0.9
    from fraud_detection_amd.data.synthetic import separable

    _, y = separable(24_000, fraud_rate=0.02, seed=100)
    n_maj = [int((y[r * 12000:(r + 1) * 12000] == 0).sum()) for r in range(2)]
    assert [int(o["n_train"]) for o in outs] == [2 * m for m in n_maj]   # per-partition quotas


def test_collective_order_is_identical_on_every_rank(tmp_path):
    """The ordering contract of parallel/comm.py: every rank issues the same collective sequence
    (op, communicator path) -- the property that rules out cross-communicator deadlock -- and
    every collective is timed (fdx_allreduce_seconds / collective_summary)."""
    outs = _run(4, True, tmp_path)
    seqs = [list(o["trace"]) for o in outs]
    assert len(seqs[0]) > 5 and all(sq == seqs[0] for sq in seqs)
    st = json.loads(str(outs[0]["stats"]))
    assert st["all_reduce_sum"]["count"] >= 2 and st["all_gather_rows"]["count"] >= 2
    assert all(v["total_ms"] >= 0 for v in st.values())


def test_lost_rank_fails_the_whole_job(tmp_path):
    """A rank raising mid-fit (between collectives) makes torchrun tear the job down: the launcher
    exits non-zero well within the store timeout instead of leaving the survivors blocked."""
    from fraud_detection_amd.data.synthetic import separable_frame

    csv = str(tmp_path / "cc.csv")
    separable_frame(8_000, fraud_rate=0.02, seed=3).to_csv(csv, index=False)
    env = dict(os.environ, DATA_CSV=csv, FDX_DEVICE="cpu", FDX_FAULT="dp_rank_crash:1", FDX_DIST_TIMEOUT="300",
               MLFLOW_TRACKING_URI=str(tmp_path / "mlruns"), PYTHONPATH=os.path.dirname(os.path.dirname(__file__)))
    t0 = time.time()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={_free_port()}", "train_model.py"],
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), env=env,
                       capture_output=True, text=True, timeout=240)
    dt = time.time() - t0
    assert r.returncode != 0
    assert "simulated crash of rank 1" in (r.stdout + r.stderr)
    assert dt < 200, f"job took {dt:.0f}s to fail"


def _host_pg_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), FDX_HOST_PG="force")
    from fraud_detection_amd.parallel.comm import Communicator

    comm = Communicator(backend="gloo")
    assert comm._host_pg is not None
    got = comm.all_gather_ints([rank, 10 * rank + 1])
    s = comm.all_reduce_scalar(float(rank + 1))
    mx = comm.max_over_ranks(float(rank))
    mn = comm.all_reduce_scalar(float(rank + 5), op="min")
    np.savez(os.path.join(out_dir, f"h{rank}.npz"), got=np.array(got), s=s, mx=mx, mn=mn,
             stats=np.array(json.dumps(comm.collective_summary())))
    comm.barrier()
    comm.close()


def test_host_value_exchanges_use_the_cpu_group(tmp_path):
    """all_gather_ints / all_reduce_scalar over the CPU-only gloo group (the path DP fits take
    under RCCL, so the row/minority-count exchange never waits for the device stream)."""
    world = 3
    port = _free_port()
    mp.start_processes(_host_pg_worker, args=(world, port, str(tmp_path)), nprocs=world, start_method="spawn")
    for r in range(world):
        d = dict(np.load(os.path.join(tmp_path, f"h{r}.npz")))
        assert d["got"].tolist() == [[q, 10 * q + 1] for q in range(world)]
        assert float(d["s"]) == 6.0 and float(d["mx"]) == 2.0 and float(d["mn"]) == 5.0
        assert "all_gather_ints" in json.loads(str(d["stats"]))


def _sgd_rows():
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.ops import scaler as S

    X, y = separable(30_000, fraud_rate=0.1, seed=77)
    st = S.scaler_fit(X)
    return S.scale_cast(X, st, labels=y, out_dtype="f32")


def _sgd_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.parallel.comm import Communicator

    comm = Communicator(backend="gloo")
    R = _sgd_rows()
    n = R.shape[0]
    sh = slice(rank * n // world, (rank + 1) * n // world)
    f = L.sgd_fit(R[sh].contiguous(), batches=4, epochs=2, tol=0.0, comm=comm, subsample=None, extra_epochs=1)
    np.savez(os.path.join(out_dir, f"s{rank}.npz"), w=f.w, n_iter=f.n_iter, obj=f.objective, gmax=f.grad_max)
    comm.barrier()
    comm.close()


@pytest.mark.parametrize("world", [2, 3])
def test_dp_sgd_global_minibatch_is_the_union_of_shard_minibatches(tmp_path, world):
    """Data-parallel SGD: every step's minibatch is the union of the ranks' local minibatch b (their
    own strided row tiles), its sums all-reduced -- so all ranks hold one model, equal to the fp64
    mirror run over those unions (extra epochs included: tol 0 never converges)."""
    from fraud_detection_amd.ops import logreg as L
    from fraud_detection_amd.ops import reference as ref
    from fraud_detection_amd.ops.layout import LABEL_COL

    port = _free_port()
    mp.start_processes(_sgd_worker, args=(world, port, str(tmp_path)), nprocs=world, start_method="spawn")
    outs = [dict(np.load(os.path.join(tmp_path, f"s{r}.npz"))) for r in range(world)]
    for o in outs[1:]:
        assert np.array_equal(o["w"], outs[0]["w"])
    R = _sgd_rows().double().numpy()
    n, nb, epochs = R.shape[0], 4, 3
    parts = []
    for r in range(world):
        lo, hi = r * n // world, (r + 1) * n // world
        parts.append((lo, ref.sgd_row_batches(hi - lo, nb, ref.sgd_grid_blocks(hi - lo, nb, ref.SGD_FULL_BLOCKS))))
    st = ref.SgdStateRef(np.zeros(32))
    for ep in range(epochs):
        for b in range(nb):
            red = np.zeros(36)
            for lo, bt in parts:
                Rb = R[lo + np.nonzero(bt == b)[0]]
                g, loss, wsum, _ = ref.logreg_pass(Rb, st.w, (1.0, 1.0), False)
                X = Rb.copy()
                X[:, LABEL_COL] = 0.0
                wv = st.w.copy()
                wv[LABEL_COL] = 0.0
                p = ref.sigmoid(X @ wv)
                red += np.concatenate([g, [loss, wsum, 0.0, float(np.sum(p * (1 - p)))]])
            st.step(red[:32], red[32], red[33], red[35], 30, 1.0, L._epoch_lr(L.SGD_LR, ep), L.SGD_MOMENTUM, nb,
                    ep >= 1, b == nb - 1, 0.0)
    assert int(outs[0]["n_iter"]) == epochs * nb == st.iter
    w = st.w.copy()
    w[LABEL_COL] = 0.0
    np.testing.assert_allclose(outs[0]["w"], w, rtol=1e-9, atol=1e-12)
