"""Multi-worker serving launcher: one GPU-owner process + N HTTP front-end workers.

    python -m fraud_detection_amd.serve.launch --workers 2 --port 8000

replaces the reference's ``gunicorn -k uvicorn.workers.UvicornWorker api.app:app --workers 2``
(/root/reference/Dockerfile:21).  Start order: the owner (serve/gpu_owner.py) loads the production
model onto the GPU, calibrates the host/device threshold and publishes its request ring under
/dev/shm; then uvicorn starts the front-end workers with FDX_GPU_OWNER_RING pointing at that ring
and FDX_DEVICE=cpu, so no front-end ever creates a HIP context (their CPU model copy only serves
the small batches the owner's calibration assigns to the host).  If either side exits, the other
is stopped and the launcher exits non-zero; SIGTERM / SIGINT are forwarded.  Nothing here touches
the GPU and nothing is exec'ed: both sides are child processes.
"""
from __future__ import annotations

import argparse
import os
import signal
import socket
import subprocess
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--workers", type=int, default=int(os.getenv("FDX_API_WORKERS", "2")))
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--app", default="api.app:app")
    ap.add_argument("--ring", default=None, help="ring file (default /dev/shm/fdx_ring_<pid>)")
    ap.add_argument("--owner-timeout", type=float, default=300.0, help="seconds to wait for the owner's ring")
    a = ap.parse_args(argv)
    ring = a.ring or f"/dev/shm/fdx_ring_{os.getpid()}"
    if os.path.exists(ring):
        os.unlink(ring)
    owner = subprocess.Popen([sys.executable, "-m", "fraud_detection_amd.serve.gpu_owner", "--ring", ring])
    deadline = time.time() + a.owner_timeout
    while not os.path.exists(ring):
        if owner.poll() is not None:
            print(f"[launch] GPU owner exited with {owner.returncode} before publishing its ring", file=sys.stderr)
            return owner.returncode or 1
        if time.time() > deadline:
            owner.terminate()
            print("[launch] GPU owner did not publish its ring in time", file=sys.stderr)
            return 1
        time.sleep(0.05)
    env = dict(os.environ, FDX_GPU_OWNER_RING=ring, FDX_DEVICE="cpu")
    # The listening socket is made here with TCP_NODELAY set, so every accepted connection
    # inherits it (Linux copies it on accept): uvicorn's multi-worker mode shares a socket whose
    # accepted connections asyncio does NOT switch to NODELAY, and a response written in two
    # segments then waits for the client's delayed ACK (~40 ms per request, measured).
    lsock = socket.socket(socket.AF_INET6 if ":" in a.host else socket.AF_INET, socket.SOCK_STREAM)
    lsock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
    lsock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
    lsock.bind((a.host, a.port))
    lsock.listen(2048)
    lsock.set_inheritable(True)
    front = subprocess.Popen([sys.executable, "-m", "uvicorn", a.app, "--fd", str(lsock.fileno()),
                              "--workers", str(a.workers)], env=env, pass_fds=(lsock.fileno(),))
    procs = [owner, front]

    def _fwd(signum, _frame):
        for p in procs:
            if p.poll() is None:
                p.send_signal(signum)

    signal.signal(signal.SIGTERM, _fwd)
    signal.signal(signal.SIGINT, _fwd)
    rc = None
    while rc is None:
        for p in procs:
            r = p.poll()
            if r is not None:
                rc = r
                break
        else:
            time.sleep(0.2)
    for p in procs:  # one side ended: stop the other
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=15)
        except subprocess.TimeoutExpired:
            p.kill()
    if os.path.exists(ring):
        os.unlink(ring)
    return rc if rc else 0


if __name__ == "__main__":
    raise SystemExit(main())
