"""The serving process model: one GPU-owner process, N
front-end workers forwarding through the shared-memory ring (csrc/serve/shm_ring.cpp), and the
small-batch host routing.  CPU here (the owner runs the exact fp64 engine); the GPU variants at
the bottom run the owner on the MI355X."""
import concurrent.futures as cf
import json
import os
import signal
import socket
import subprocess
import sys
import time
import urllib.request

import numpy as np
import pytest

from _models import kaggle_like_rows
from test_api_contract import GOLDEN_SAMPLE

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _engine(device="cpu"):
    from fraud_detection_amd.serve.engine import InferenceEngine

    return InferenceEngine.from_paths(device=device)


def test_ring_roundtrip_matches_engine_under_concurrency():
    from fraud_detection_amd.serve.gpu_owner import Dispatcher, GpuOwner, RingClient

    eng = _engine()
    owner = GpuOwner(eng, "", max_batch=512).start()
    try:
        cli = RingClient(owner.ring)
        disp = Dispatcher(eng, cli, host_max_rows=0)  # force every request through the ring
        rows = kaggle_like_rows(400, seed=11)
        ref_p, ref_z = eng.predict_proba(rows)

        def one(i):
            n = 1 + (i % 7) * 37  # 1..223 rows: single-slot and multi-slot requests
            j = (i * 13) % (len(rows) - n)
            p, z = disp.predict_proba(rows[j:j + n])
            return j, n, p, z

        with cf.ThreadPoolExecutor(16) as ex:
            for j, n, p, z in ex.map(one, range(300)):
                # the ring carries float32 results of the fp64 host computation
                np.testing.assert_allclose(p, ref_p[j:j + n], rtol=1e-6, atol=1e-12)
                np.testing.assert_allclose(z, ref_z[j:j + n], rtol=1e-6, atol=1e-5)
        p, z, phi = cli.predict_explain(rows[:70])
        rp, rz, rphi = eng.predict_explain(rows[:70])
        np.testing.assert_allclose(phi, rphi, rtol=1e-5, atol=1e-6)
        st = cli.stats()
        assert st["rows"] >= 300 and st["queued_tickets"] == 0
        assert owner.batches < st["slots"]  # several requests shared a batch
    finally:
        owner.stop()


def test_dispatcher_routes_small_batches_to_host():
    from fraud_detection_amd.obs.metrics import api_metrics
    from fraud_detection_amd.serve.gpu_owner import Dispatcher, GpuOwner, RingClient

    eng = _engine()
    owner = GpuOwner(eng, "").start()
    try:
        m = api_metrics()
        disp = Dispatcher(eng, RingClient(owner.ring), host_max_rows=8, metrics=m)
        x = np.asarray([GOLDEN_SAMPLE], np.float32)
        p, _ = disp.predict_one(x[0])
        assert p == pytest.approx(0.011905, abs=5e-7)
        assert owner.rows == 0  # host path
        disp.predict_proba(np.repeat(x, 9, 0))
        assert owner.rows == 9  # above the threshold: the owner
    finally:
        owner.stop()


def test_dispatcher_explain_splits_big_batches_and_falls_back():
    """/predict/batch with explain=true through a GPU owner must explain any batch size
    (split into ring-sized requests) and degrade to the front-end's own engine when the owner is
    down -- never an HTTP 500."""
    from fraud_detection_amd.serve.gpu_owner import Dispatcher, GpuOwner, RingClient

    eng = _engine()
    owner = GpuOwner(eng, "", max_batch=64, nslots=4, slot_rows=8).start()  # ring: 32 rows
    try:
        cli = RingClient(owner.ring, timeout_ms=3000.0)
        disp = Dispatcher(eng, cli, host_max_rows=0)  # a front-end: the owner lives elsewhere
        rows = kaggle_like_rows(150, seed=3)
        ex = eng.explain(rows, "linear")
        p, phi = disp.explain(rows, "linear")
        np.testing.assert_allclose(p, ex.prob, rtol=1e-6, atol=1e-12)
        np.testing.assert_allclose(phi, ex.phi, rtol=1e-5, atol=1e-6)
        assert owner.rows >= 150
    finally:
        owner.stop()
    p2, phi2 = disp.explain(rows, "linear")  # owner stopped: this process's engine answers
    np.testing.assert_allclose(phi2, ex.phi, rtol=1e-12, atol=1e-12)


def test_ring_fails_requests_when_owner_stops():
    from fraud_detection_amd import _fdx_ring as R

    r = R.Ring("", 8, 30, 4, 32)
    r.owner_state = R.OWNER_STOPPED
    with pytest.raises(RuntimeError):
        r.request(np.zeros((1, 30), np.float32), 0, 2000.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _get(url, timeout=5.0):
    with urllib.request.urlopen(url, timeout=timeout) as r:
        return r.status, r.read()


def _post(url, body):
    req = urllib.request.Request(url, data=json.dumps(body).encode(), headers={"Content-Type": "application/json"})
    with urllib.request.urlopen(req, timeout=30) as r:
        return json.loads(r.read())


def _launch(tmp_path, owner_device, workers=2):
    port = _free_port()
    ring = f"/dev/shm/fdx_ring_test_{os.getpid()}_{port}"
    env = dict(os.environ, DATABASE_URL=f"sqlite:///{tmp_path}/svc.db", MLFLOW_TRACKING_URI=f"file:{tmp_path}/mlruns",
               FDX_DEVICE=owner_device, FDX_HOST_MAX_ROWS="0", PYTHONPATH=ROOT)
    p = subprocess.Popen([sys.executable, "-m", "fraud_detection_amd.serve.launch", "--workers", str(workers),
                          "--host", "127.0.0.1", "--port", str(port), "--ring", ring], cwd=ROOT, env=env,
                         stdout=subprocess.PIPE, stderr=subprocess.STDOUT, start_new_session=True)
    base = f"http://127.0.0.1:{port}"
    deadline = time.time() + 240
    while True:
        try:
            if _get(base + "/status")[0] == 200:
                break
        except OSError:
            pass
        if p.poll() is not None or time.time() > deadline:
            out = p.stdout.read().decode(errors="replace") if p.poll() is not None else ""
            os.killpg(p.pid, signal.SIGKILL) if p.poll() is None else None
            raise AssertionError(f"service did not come up (rc={p.poll()}):\n{out[-4000:]}")
        time.sleep(0.2)
    return p, base, ring


def _stop(p, ring):
    p.send_signal(signal.SIGTERM)
    try:
        rc = p.wait(timeout=30)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        raise
    assert not os.path.exists(ring)
    return rc


def _exercise(base):
    with cf.ThreadPoolExecutor(16) as ex:
        scores = list(ex.map(lambda i: _post(base + "/predict", {"features": GOLDEN_SAMPLE if i % 2 else [0.1] * 30})["score"],
                             range(48)))
    for i, s in enumerate(scores):
        assert s == pytest.approx(0.011905 if i % 2 else 0.000544, abs=5e-7)
    rows = kaggle_like_rows(300, seed=4)
    b = _post(base + "/predict/batch", {"rows": rows.tolist()})
    assert len(b["scores"]) == 300
    m = _get(base + "/metrics")[1].decode()
    owner_rows = [ln for ln in m.splitlines() if ln.startswith("fdx_gpu_owner_rows")]
    assert owner_rows and float(owner_rows[0].split()[-1]) >= 24  # this worker saw the owner's total
    return b


def test_multiworker_launcher_cpu_owner(tmp_path):
    p, base, ring = _launch(tmp_path, "cpu")
    try:
        b = _exercise(base)
        eng = _engine()
        np.testing.assert_allclose(b["scores"], eng.predict_proba(kaggle_like_rows(300, seed=4))[0], rtol=1e-6)
    finally:
        _stop(p, ring)


@pytest.mark.gpu
def test_multiworker_launcher_gpu_owner(dev, tmp_path):
    """Two HTTP workers (no HIP context) forwarding to one GPU-owner process on the MI355X."""
    p, base, ring = _launch(tmp_path, "cuda")
    try:
        b = _exercise(base)
        eng = _engine()
        np.testing.assert_allclose(b["scores"], eng.predict_proba(kaggle_like_rows(300, seed=4))[0], atol=2e-6)
    finally:
        _stop(p, ring)


@pytest.mark.gpu
@pytest.mark.parametrize("loop", ["native", "python"])
def test_gpu_owner_in_process_batches(dev, loop, monkeypatch):
    from fraud_detection_amd.serve.gpu_owner import Dispatcher, GpuOwner, RingClient

    monkeypatch.setenv("FDX_OWNER_LOOP", loop)
    eng = _engine("cuda")
    assert eng.calibration.get("source") in ("measured", "FDX_HOST_MAX_ROWS")
    # the launch path's batching (the persistent mailbox path answers single rows too fast to
    # batch them: test_native_owner_persistent_kernel).  A 200 us collection window makes the
    # coalescing of the 32 concurrent producers deterministic: with no window a fast owner can
    # drain the ring one request at a time (600 batches for 600 requests on one r4 box).
    owner = GpuOwner(eng, "", persist_rows=0, window_us=200.0).start()
    try:
        disp = Dispatcher(eng, RingClient(owner.ring), host_max_rows=0)
        rows = kaggle_like_rows(600, seed=12)
        cpu = _engine()
        rp, _ = cpu.predict_proba(rows)
        with cf.ThreadPoolExecutor(32) as ex:
            got = list(ex.map(lambda i: disp.predict_proba(rows[i:i + 1])[0][0], range(600)))
        np.testing.assert_allclose(got, rp, atol=2e-6)
        big, _ = disp.predict_proba(rows)  # > ZERO_COPY_ROWS: the H2D copy path (python loop)
        np.testing.assert_allclose(big, rp, atol=2e-6)
        p, z, phi = RingClient(owner.ring).predict_explain(rows[:100])  # LinearSHAP through the owner
        _, _, rphi = cpu.predict_explain(rows[:100])
        np.testing.assert_allclose(phi, rphi, rtol=1e-4, atol=1e-4)
        assert owner.native == (loop == "native")
        assert owner.batches < 600 and owner.rows >= 1300
    finally:
        owner.stop()


@pytest.mark.gpu
def test_native_owner_persistent_kernel(dev):
    """Small predict batches through the owner's persistent mailbox kernel: the same bits as the
    launch path, explain still served (launch path from the same staging), and the kernel is
    relaunched after its idle timeout."""
    from fraud_detection_amd.serve.gpu_owner import Dispatcher, GpuOwner, RingClient

    eng = _engine("cuda")
    rows = kaggle_like_rows(400, seed=14)
    got = {}
    for persist in (0, 256):
        owner = GpuOwner(eng, "", persist_rows=persist, persist_idle_ms=30.0).start()
        try:
            assert owner.native
            disp = Dispatcher(eng, RingClient(owner.ring), host_max_rows=0)
            p = np.array([disp.predict_proba(rows[i:i + 1])[0][0] for i in range(200)])
            with cf.ThreadPoolExecutor(16) as ex:  # concurrent producers: multi-row batches
                pc = np.array(list(ex.map(lambda i: disp.predict_proba(rows[i:i + 1])[0][0], range(200, 400))))
            time.sleep(0.1)  # > idle timeout: the persistent kernel exits ...
            p2, _ = disp.predict_proba(rows[:5])  # ... and is relaunched for this one
            _, _, phi = RingClient(owner.ring).predict_explain(rows[:40])
            got[persist] = (p, pc, p2, phi)
            st = owner.native_stats()
            if persist:
                assert st["persistent"] and st["persistent_batches"] >= 200, st
                assert st["persistent_launches"] >= 2, st
            else:
                assert not st["persistent"]
        finally:
            owner.stop()
    for a, b in zip(got[0], got[256]):
        assert np.array_equal(a, b)
    rp, _ = _engine().predict_proba(rows)
    np.testing.assert_allclose(got[256][0], rp[:200], atol=2e-6)
