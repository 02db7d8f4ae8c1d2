"""Inference engines shared by the API, the XAI worker and the library predictors.

Two model families, one interface (``predict_proba`` / ``predict_explain`` / ``explain``):

* ``InferenceEngine`` -- the linear model (reference: models/logistic_model.joblib + scaler.joblib,
  api/app.py:34-48) with the StandardScaler folded into the weights (ops/predict.py fold_scaler),
  so a request's raw features are read exactly once by the fused predict + LinearSHAP kernel
  (K5/K6).
* ``TreeInferenceEngine`` -- the GBDT family (reference train_model.py:95-113 trains and dumps an
  XGBClassifier): scaler -> tree-ensemble predict kernel (K11), explained with the masked-row
  KernelSHAP tree kernel (K7 tree path).

Explanations (``explain``): ``method="linear"`` is LinearSHAP (shap.LinearExplainer semantics of
explain_model.py:24 / api/worker.py:53, log-odds space, background = the standardized training
mean); ``method="kernel"`` is KernelSHAP (shap.KernelExplainer semantics, probability space,
background = the <= 128 training rows stored next to the model as ``shap_background.npy``);
``"auto"`` picks kernel when a background is available.

Device policy: ``device="auto"`` uses the GPU when one is present; CPU execution is exact fp64
numpy (what the reference's sklearn path computes).  Host <-> device traffic goes through
persistent pinned staging buffers (one upload and one download per call, no per-request pinned
allocation).

Small-batch routing: a GPU launch + synchronise costs tens of microseconds whatever the batch, the
exact host fp64 path a few microseconds per row, so a GPU engine measures both at start-up
(``calibrate``) and sends batches of at most ``host_max_rows`` rows to the host path
(FDX_HOST_MAX_ROWS pins the threshold; 0 = always the device).  Explanations with KernelSHAP /
TreeSHAP always run on the device (their host paths are orders of magnitude slower).
"""
from __future__ import annotations

import json
import logging
import os
import threading
from dataclasses import dataclass

import numpy as np
import torch

from ..compat.sklearn_export import LinearArtifacts, load_artifacts
from ..ops import predict as P

logger = logging.getLogger(__name__)

BACKGROUND_FILE = "shap_background.npy"
MAX_BACKGROUND = 128


def _pick_device(device) -> torch.device:
    if isinstance(device, torch.device):
        return device
    if device == "auto":
        return torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    return torch.device(device)


def load_background(model_dir: str | None) -> np.ndarray | None:
    """The KernelSHAP background saved by training (float32 [<=128, d]; no pickle)."""
    if not model_dir:
        return None
    p = os.path.join(model_dir, BACKGROUND_FILE)
    if not os.path.exists(p):
        return None
    B = np.load(p, allow_pickle=False)
    if B.ndim != 2 or B.shape[0] < 1 or B.shape[0] > MAX_BACKGROUND or not np.all(np.isfinite(B)):
        raise ValueError(f"{p}: expected a finite [1..{MAX_BACKGROUND}, d] float array, got {B.shape}")
    return np.ascontiguousarray(B, dtype=np.float32)


def sample_background(X: np.ndarray, n: int = 100, seed: int = 42) -> np.ndarray:
    """shap.sample-style background: ``n`` training rows drawn without replacement."""
    X = np.asarray(X, dtype=np.float32)
    n = max(1, min(int(n), MAX_BACKGROUND, X.shape[0]))
    idx = np.sort(np.random.default_rng(seed).choice(X.shape[0], n, replace=False))
    return np.ascontiguousarray(X[idx])


def save_background(B: np.ndarray, model_dir: str) -> str:
    os.makedirs(model_dir, exist_ok=True)
    p = os.path.join(model_dir, BACKGROUND_FILE)
    np.save(p, np.ascontiguousarray(B, dtype=np.float32), allow_pickle=False)
    return p


@dataclass
class Explanation:
    prob: np.ndarray        # [B] P(fraud)
    logit: np.ndarray       # [B] model log-odds / margin
    phi: np.ndarray         # [B, d] attributions
    base_value: float       # E[f] over the background, in phi's space
    method: str             # "linear" | "kernel" | "tree"
    space: str              # "log-odds" | "probability"


class _KernelTimer:
    """HIP-event device time of a launch sequence on the current stream -> fdx_gpu_kernel_seconds
    {kernel}.  Read after the caller's synchronisation (no extra sync)."""

    def __init__(self, name: str):
        self.name = name
        self.t0 = torch.cuda.Event(enable_timing=True)
        self.t1 = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.t0.record()
        return self

    def __exit__(self, *exc):
        self.t1.record()
        return False

    def observe(self):
        try:
            from ..obs.metrics import gpu_kernel_histogram

            gpu_kernel_histogram().labels(self.name).observe(self.t0.elapsed_time(self.t1) / 1e3)
        except Exception:  # noqa: BLE001 - metrics are best effort
            pass


ZERO_COPY_ROWS = int(os.environ.get("FDX_ZERO_COPY_ROWS", "256"))
# Batches up to this many rows go to the owner's persistent kernel (mailbox, no launch); 0 = off
PERSIST_ROWS = int(os.environ.get("FDX_OWNER_PERSIST_ROWS", "256"))
H2H_CHUNK_ROWS = 131072  # host-to-host batch scoring: rows per H2D / kernel / D2H pipeline stage
CALIBRATION_SIZES = (1, 4, 16, 64, 256, 1024, 4096, 16384, 65536)


def _median_time(fn, reps: int = 5) -> float:
    import time

    fn()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts))


class _Staging:
    """Persistent pinned host buffers + device buffers for one engine (grown on demand).  Calls
    are serialised by the engine lock, so one set suffices.  Small batches (<= ZERO_COPY_ROWS)
    skip both memcpys: the kernel reads the request from, and writes the result to, the pinned
    buffers through their device mapping (hipHostGetDevicePointer) -- one launch + one sync."""

    def __init__(self, device: torch.device, d: int, n_out: int):
        self.device, self.d, self.n_out = device, d, n_out
        self.cap = 0
        self.in_map = self.out_map = 0

    def ensure(self, n: int):
        if n > self.cap:
            cap = max(n, 2 * self.cap, 256)
            self.hin = torch.empty((cap, self.d), dtype=torch.float32, pin_memory=True)
            self.din = torch.empty((cap, self.d), dtype=torch.float32, device=self.device)
            self.hout = torch.empty(cap * self.n_out, dtype=torch.float32, pin_memory=True)
            self.dout = torch.empty(cap * self.n_out, dtype=torch.float32, device=self.device)
            self.cap = cap
            from ..ops.native import native

            m = native()
            self.in_map = m.host_device_pointer(self.hin.data_ptr())
            self.out_map = m.host_device_pointer(self.hout.data_ptr())

    def zero_copy(self, n: int) -> bool:
        self.ensure(n)
        return n <= ZERO_COPY_ROWS and self.in_map != 0 and self.out_map != 0

    def upload(self, X: np.ndarray) -> torch.Tensor:
        n = X.shape[0]
        self.ensure(n)
        self.hin[:n].numpy()[...] = X
        xd = self.din[:n]
        xd.copy_(self.hin[:n], non_blocking=True)
        return xd

    def download(self, n_vals: int) -> np.ndarray:
        """Copy dout[:n_vals] to host (on the current stream) and wait for it."""
        self.hout[:n_vals].copy_(self.dout[:n_vals], non_blocking=True)
        torch.cuda.current_stream(self.device).synchronize()
        return self.hout[:n_vals].numpy()


class _EngineBase:
    kind = "?"

    def __init__(self, device, source: str, background: np.ndarray | None, kernel_nsamples: int = 0,
                 kernel_link: str = "identity"):
        self.device = _pick_device(device)
        self.source = source
        self.background = background
        self.kernel_nsamples = int(kernel_nsamples or 0)
        self.kernel_link = kernel_link
        self._lock = threading.Lock()
        self._kexpl = None
        self.host_max_rows = 0
        self.calibration: dict = {}
        self._owner_in = None
        self._ostream = None
        if self.device.type == "cuda":
            from ..ops.native import native

            native()  # fail loudly rather than serve through an eager fallback
            self._stream = torch.cuda.Stream(self.device)

    def _finish_init(self):
        """Subclasses call this once their buffers exist: the small-batch threshold."""
        if self.device.type != "cuda":
            self.host_max_rows = 1 << 62  # a CPU engine runs everything on the host
            return
        env = os.environ.get("FDX_HOST_MAX_ROWS", "").strip()
        if env and int(env) >= 0:
            self.host_max_rows = int(env)
            self.calibration = {"source": "FDX_HOST_MAX_ROWS"}
        else:
            self.calibrate()

    def calibrate(self, sizes=CALIBRATION_SIZES) -> int:
        """Largest batch size (of ``sizes``) at which the exact host path is no slower than the
        device path (upload + kernel + download + sync), measured on this machine."""
        rng = np.random.default_rng(0)
        thr, rows = 0, []
        for n in sizes:
            X = self._calibration_rows(rng, n)
            th = _median_time(lambda: self._predict_host(X))
            td = _median_time(lambda: self._predict_device(X))
            rows.append({"rows": n, "host_us": round(th * 1e6, 2), "device_us": round(td * 1e6, 2)})
            if th > td:
                break
            thr = n
        self.host_max_rows = thr
        self.calibration = {"source": "measured", "sizes": rows}
        logger.info("%s engine: batches <= %d rows take the host path (%s)", self.kind, thr, rows)
        return thr

    def _calibration_rows(self, rng, n: int) -> np.ndarray:
        X = rng.normal(0.0, 1.0, (n, self.d)).astype(np.float32)
        return X

    def _use_host(self, n: int) -> bool:
        return self.device.type != "cuda" or n == 0 or n <= self.host_max_rows

    # ---- GPU-owner API (serve/gpu_owner.py): rows land in a pinned staging buffer -------------
    # Two buffer sets: the owner gathers batch i+1 into one while batch i runs from the other.
    def owner_input(self, cap: int, set_: int = 0) -> int:
        """Address of pinned float32 [cap, d] buffer `set_` (0/1) the ring gathers rows into."""
        if getattr(self, "_owner_in", None) is None or self._owner_in[0].shape[0] < cap:
            pin = self.device.type == "cuda"
            self._owner_in = [torch.empty((cap, self.d), dtype=torch.float32, pin_memory=pin) for _ in range(2)]
            self._owner_out = [np.empty(cap * (self.d + 2), np.float32) for _ in range(2)]
            self._owner_map = [0, 0]
            if pin:
                from ..ops.native import native

                self._owner_map = [native().host_device_pointer(t.data_ptr()) for t in self._owner_in]
        return self._owner_in[set_].data_ptr()

    def run_staged_async(self, n: int, explain: bool, set_: int = 0):
        """Start scoring (and explaining) the n rows of buffer `set_`; -> a handle for
        wait_staged.  Generic path: computed right here through the public API (the handle is
        already complete); InferenceEngine launches on the device and returns at once."""
        X = self._owner_in[set_][:n].numpy()
        o = self._owner_out[set_]
        if explain:
            e = self.explain(X, os.environ.get("FDX_XAI_METHOD", "auto"))
            p, z, phi = e.prob, e.logit, e.phi
        else:
            p, z = self.predict_proba(X)
            phi = None
        o[:n] = p
        o[n:2 * n] = z
        base = o.ctypes.data
        if phi is None:
            return (base, base + 4 * n, 0, 0)
        o[2 * n:2 * n + n * self.d] = np.asarray(phi, np.float32).reshape(-1)
        return (base, base + 4 * n, base + 8 * n, self.d)

    def wait_staged(self, handle):
        """-> (prob, logit, phi, dphi) addresses of float32 column blocks of a started batch."""
        return handle

    def run_staged(self, n: int, explain: bool, set_: int = 0):
        return self.wait_staged(self.run_staged_async(n, explain, set_))

    # ---- shared API ------------------------------------------------------------------------
    @property
    def has_background(self) -> bool:
        return self.background is not None

    def predict(self, X: np.ndarray):
        p, _ = self.predict_proba(X)
        return (p > 0.5).astype(np.int64), p

    def _check(self, X) -> np.ndarray:
        X = np.ascontiguousarray(X, dtype=np.float32)
        if X.ndim != 2 or X.shape[1] != self.d:
            raise ValueError(f"expected [B, {self.d}] features, got {X.shape}")
        return X

    def resolve_method(self, method: str = "auto") -> str:
        """``auto``: the family's default -- LinearSHAP for the linear model (log-odds
        attributions, what the reference's worker computes: xai_tasks.py:103-115, api/worker.py:53);
        KernelSHAP (probability space) is opt-in with ``kernel`` / FDX_XAI_METHOD=kernel."""
        method = (method or "auto").lower()
        if method == "auto":
            method = self.default_method
        if method in ("kernel", "tree") and not self.has_background:
            raise ValueError(f"{method} SHAP needs a background (shap_background.npy next to the model)")
        if method not in self.methods:
            raise ValueError(f"{self.kind} model supports {self.methods}, not {method!r}")
        return method

    def kernel_explainer(self):
        if self._kexpl is None:
            if not self.has_background:
                raise ValueError("no background for KernelSHAP")
            self._kexpl = self._make_kernel_explainer()
        return self._kexpl

    def explain(self, X: np.ndarray, method: str = "auto") -> Explanation:
        X = self._check(X)
        m = self.resolve_method(method)
        if m == "tree":
            return self._explain_tree(X)
        if m == "linear":
            p, z, phi = self.predict_explain(X)
            return Explanation(p, z, phi, self.expected_value(), "linear", "log-odds")
        n, d = X.shape
        if n == 0:
            p, z = self.predict_proba(X)
            return Explanation(p, z, np.zeros((0, d)), 0.0, "kernel", "probability")
        ke = self.kernel_explainer()
        space = "log-odds" if ke.link == "logit_model" else "probability"
        if self.device.type != "cuda":
            p, z = self.predict_proba(X)
            phi, fx, f0 = ke.explain(X)
            return Explanation(p, z, np.asarray(phi, np.float64), float(f0), "kernel", space)
        # one upload, one launch sequence, one download: phi / f(x) / f0 land in a single staging
        # buffer; the score comes from the kernel's f(x) (identity link: the probability)
        with self._lock, torch.cuda.stream(self._stream):
            st = self._xstage
            xd = st.upload(X)
            o = st.dout
            outs = (o[: n * d].view(n, d), o[n * d: n * d + n], o[n * d + n: n * d + 2 * n])
            with _KernelTimer(f"kernelshap_{self.kind}") as kt:
                self._kernel_device(xd, ke, outs)
            h = st.download(n * d + 2 * n)
            kt.observe()
        phi = h[: n * d].reshape(n, d).astype(np.float64)
        fx = h[n * d: n * d + n].astype(np.float64)
        z = self._logit_host(X)
        p = fx if ke.link == "identity" else 1.0 / (1.0 + np.exp(-z))
        return Explanation(p, z, phi, float(h[n * d + n]), "kernel", space)


class InferenceEngine(_EngineBase):
    """Linear model + folded scaler (see module docstring)."""

    kind = "linear"
    methods = ("linear", "kernel")
    default_method = "linear"

    def __init__(self, artifacts: LinearArtifacts, device: str = "auto", bg_std: np.ndarray | None = None,
                 source: str = "local", background: np.ndarray | None = None, kernel_nsamples: int = 0,
                 kernel_link: str = "identity"):
        self.art = artifacts
        self.d = len(artifacts.mean)
        self.feature_names = list(artifacts.feature_names)
        self.a, self.c, self.bias = P.fold_scaler(artifacts.padded_weights(), artifacts.mean, artifacts.scale, bg_std)
        super().__init__(device, source, background, kernel_nsamples, kernel_link)
        if self.device.type == "cuda":
            # the fused kernel reads fp32 weights (the fold is computed in fp64, then rounded once)
            self._a = torch.from_numpy(self.a.astype(np.float32)).to(self.device)
            self._c = torch.from_numpy(self.c.astype(np.float32)).to(self.device)
            self._stage = _Staging(self.device, self.d, self.d + 2)
            self._xstage = _Staging(self.device, self.d, self.d + 2)
            self._ostage = _Staging(self.device, self.d, self.d + 2)
            self._h2d_stream = torch.cuda.Stream(self.device)
            self._d2h_stream = torch.cuda.Stream(self.device)
            self._h2h_cap = 0
        self._finish_init()

    @classmethod
    def from_paths(cls, model_path=None, scaler_path=None, features_path=None, device="auto",
                   source: str = "local", **kw) -> "_EngineBase":
        model_path = model_path or os.getenv("MODEL_PATH", "./models/logistic_model.joblib")
        if model_path.endswith(".json"):
            return TreeInferenceEngine.from_paths(model_path, scaler_path, features_path, device, source, **kw)
        scaler_path = scaler_path or os.getenv("SCALER_PATH") or os.path.join(os.path.dirname(model_path),
                                                                               "scaler.joblib")
        features_path = features_path or os.getenv("FEATURE_NAMES_PATH", "./models/feature_names.json")
        bg = load_background(os.path.dirname(os.path.abspath(model_path)))
        return cls(load_artifacts(model_path, scaler_path, features_path), device=device, source=source,
                   background=bg, **kw)

    # ---- core ------------------------------------------------------------------------------
    def _launch(self, xo: int, n: int, want_phi: bool, st: "_Staging", zero_copy: bool):
        """Fused folded-scaler predict (+ LinearSHAP) on device rows at ``xo``; results into
        the staging output ([prob n][logit n][phi n*d]); waits for them.  -> host view."""
        d = self.d
        dphi = d if want_phi else 0
        m = P.native()
        s = torch.cuda.current_stream(self.device).cuda_stream
        if zero_copy:
            oo = st.out_map
            with _KernelTimer("predict_shap" if want_phi else "predict") as kt:
                m.predict_shap(xo, 1, n, d, d, dphi, P.ptr(self._a), P.ptr(self._c), float(self.bias),
                               oo, oo + 4 * n, oo + 8 * n if want_phi else 0, dphi, s)
            torch.cuda.current_stream(self.device).synchronize()
            o = st.hout[: n * (2 + dphi)].numpy()
        else:
            out = st.dout
            prob, logit = out[:n], out[n:2 * n]
            phi = out[2 * n:2 * n + n * dphi].view(n, dphi) if want_phi else None
            with _KernelTimer("predict_shap" if want_phi else "predict") as kt:
                m.predict_shap(xo, 1, n, d, d, dphi, P.ptr(self._a), P.ptr(self._c), float(self.bias),
                               P.ptr(prob), P.ptr(logit), P.ptr(phi) if want_phi else 0, dphi, s)
            o = st.download(n * (2 + dphi))
        kt.observe()
        return o

    def _device_run(self, X: np.ndarray, want_phi: bool):
        n, d = X.shape
        dphi = d if want_phi else 0
        with self._lock, torch.cuda.stream(self._stream):
            st = self._stage
            if st.zero_copy(n):
                # request and result stay in pinned memory: no memcpy, one launch, one sync
                st.hin[:n].numpy()[...] = X
                o = self._launch(st.in_map, n, want_phi, st, True)
            else:
                xd = st.upload(X)
                o = self._launch(P.ptr(xd), n, want_phi, st, False)
        p = o[:n].astype(np.float64)
        z = o[n:2 * n].astype(np.float64)
        ph = o[2 * n:].reshape(n, dphi).astype(np.float64) if want_phi else None
        return p, z, ph

    def run_staged_async(self, n: int, explain: bool, set_: int = 0):
        """GPU-owner path: the ring gathered the rows straight into pinned buffer `set_`; the kernel
        reads them there through the device mapping and writes the results into mapped pinned
        memory (small batches: one launch, nothing copied), or after one H2D copy (large
        batches).  Returns at once; wait_staged waits on the batch's event with the GIL released.
        Owner thread only, on the owner's own stream."""
        if self.device.type != "cuda" or (explain and os.environ.get("FDX_XAI_METHOD", "auto") not in ("auto", "linear")):
            return super().run_staged_async(n, explain, set_)
        d = self.d
        dphi = d if explain else 0
        m = P.native()
        if self._ostream is None:
            self._ostream = torch.cuda.Stream(self.device)
            self._ostages = [_Staging(self.device, d, d + 2) for _ in range(2)]
            self._oevents = [m.event_create() for _ in range(2)]
        st = self._ostages[set_]
        st.ensure(self._owner_in[set_].shape[0])
        sh = self._ostream.cuda_stream
        if n <= ZERO_COPY_ROWS and self._owner_map[set_] and st.out_map:
            oo = st.out_map
            m.predict_shap(self._owner_map[set_], 1, n, d, d, dphi, P.ptr(self._a), P.ptr(self._c), float(self.bias),
                           oo, oo + 4 * n, oo + 8 * n if explain else 0, dphi, sh)
        else:
            with torch.cuda.stream(self._ostream):
                st.din[:n].copy_(self._owner_in[set_][:n], non_blocking=True)
                out = st.dout
                m.predict_shap(P.ptr(st.din), 1, n, d, d, dphi, P.ptr(self._a), P.ptr(self._c), float(self.bias),
                               P.ptr(out), P.ptr(out) + 4 * n, P.ptr(out) + 8 * n if explain else 0, dphi, sh)
                st.hout[: n * (2 + dphi)].copy_(out[: n * (2 + dphi)], non_blocking=True)
        m.event_record(self._oevents[set_], sh)
        base = st.hout.data_ptr()
        return ("dev", set_, (base, base + 4 * n, (base + 8 * n) if explain else 0, dphi))

    def wait_staged(self, handle):
        if handle[0] != "dev":
            return handle
        P.native().event_sync(self._oevents[handle[1]])
        return handle[2]

    def start_native_owner(self, ring, cap: int, window_us: float, pipe_rows: int = 8,
                           persist_rows: int = PERSIST_ROWS, idle_ms: float = 200.0, life_ms: float = 10000.0) -> int:
        """Start the C++ owner loop on this engine's folded weights (GPU only): two device-mapped
        pinned input buffers (owner_input) and two device-mapped pinned output buffers.
        ``persist_rows`` > 0: batches of up to that many rows (predict) go to a persistent
        one-workgroup kernel through a mailbox in coherent host memory -- no launch and no event
        per batch; it exits after ``idle_ms`` without requests or ``life_ms`` in total and is
        relaunched on demand (csrc/kernels/predict.hip predict_persistent_kernel)."""
        m = P.native()
        self.owner_input(cap)
        if not all(self._owner_map):
            raise RuntimeError("pinned owner buffers are not device-mapped")
        if self._ostream is None:
            self._ostream = torch.cuda.Stream(self.device)
        self._nout = [torch.empty(cap * (self.d + 2), dtype=torch.float32, pin_memory=True) for _ in range(2)]
        omap = [m.host_device_pointer(t.data_ptr()) for t in self._nout]
        if not all(omap):
            raise RuntimeError("pinned owner outputs are not device-mapped")
        return m.owner_start(ring.base_address, ring.total_bytes, P.ptr(self._a), P.ptr(self._c), float(self.bias),
                             self.d, int(cap), float(window_us), int(pipe_rows), self._ostream.cuda_stream,
                             self._owner_in[0].data_ptr(), self._owner_in[1].data_ptr(), self._owner_map[0],
                             self._owner_map[1], self._nout[0].data_ptr(), self._nout[1].data_ptr(), omap[0], omap[1],
                             int(persist_rows), float(idle_ms), float(life_ms))

    def native_owner_stats(self, handle) -> dict:
        b, launches, on = P.native().owner_persistent_stats(handle)
        return {"persistent": bool(on), "persistent_batches": int(b), "persistent_launches": int(launches)}

    def stop_native_owner(self, handle) -> int:
        return int(P.native().owner_stop(handle))

    def _predict_host(self, X: np.ndarray):
        return self._cpu(X, want_phi=False)

    def _predict_device(self, X: np.ndarray):
        if X.shape[0] > ZERO_COPY_ROWS:
            return self._device_h2h(X)
        return self._device_run(X, False)

    def _device_h2h(self, X: np.ndarray, out=None):
        """Large batches, host in -> host out (config 2): the caller's rows are page-locked in place
        and pipelined chunk by chunk (H2D | fused kernel | D2H on three streams); the kernel
        writes the fp64 results the caller gets, so nothing is staged or converted on the host."""
        n, d = X.shape
        p, z = (np.empty(n), np.empty(n)) if out is None else out
        if p.dtype != np.float64 or z.dtype != np.float64 or not (p.flags.c_contiguous and z.flags.c_contiguous) \
                or p.shape != (n,) or z.shape != (n,):
            raise ValueError("out must be two contiguous float64 [n] arrays")
        with self._lock:
            if n > self._h2h_cap:
                cap = max(n, 2 * self._h2h_cap)
                self._h2h_x = torch.empty((cap, d), dtype=torch.float32, device=self.device)
                self._h2h_o = torch.empty((2, cap), dtype=torch.float64, device=self.device)
                self._h2h_cap = cap
            P.native().predict_h2h(X.ctypes.data, n, d, d, P.ptr(self._a), float(self.bias), p.ctypes.data,
                                   z.ctypes.data, P.ptr(self._h2h_x), P.ptr(self._h2h_o[0]), P.ptr(self._h2h_o[1]),
                                   H2H_CHUNK_ROWS, self._h2d_stream.cuda_stream, self._stream.cuda_stream,
                                   self._d2h_stream.cuda_stream)
        return (p, z) if out is None else out

    def predict_explain(self, X: np.ndarray):
        """X raw features [B, d] -> (prob [B], logit [B], phi [B, d]) as numpy (LinearSHAP)."""
        X = self._check(X)
        if self._use_host(X.shape[0]):
            return self._cpu(X)
        return self._device_run(X, True)

    def predict_proba(self, X: np.ndarray, out=None):
        """-> (prob [B], logit [B]) float64.  ``out``: optional (prob, logit) float64 arrays to
        fill (a batch-scoring loop reuses them: no per-call allocation)."""
        X = self._check(X)
        if self._use_host(X.shape[0]):
            p, z, _ = self._cpu(X, want_phi=False)
        elif X.shape[0] > ZERO_COPY_ROWS:
            return self._device_h2h(X, out)
        else:
            p, z, _ = self._device_run(X, False)
        if out is not None:
            out[0][...] = p
            out[1][...] = z
            return out
        return p, z

    def _cpu(self, X: np.ndarray, want_phi: bool = True):
        Xd = X.astype(np.float64)
        z = Xd @ self.a[: self.d] + self.bias
        p = 1.0 / (1.0 + np.exp(-z))
        phi = self.a[None, : self.d] * (Xd - self.c[None, : self.d]) if want_phi else None
        return p, z, phi

    def _make_kernel_explainer(self):
        from ..models.explainers import KernelExplainer

        return KernelExplainer(self.a, self.bias, self.background, nsamples=self.kernel_nsamples or None,
                               link=self.kernel_link, device=str(self.device))

    def _kernel_device(self, xd, ke, out):
        from ..ops.kernelshap import kernelshap

        return kernelshap(xd, ke, sync=False, out=out)

    def _logit_host(self, X: np.ndarray) -> np.ndarray:
        return X.astype(np.float64) @ self.a[: self.d] + self.bias

    def expected_value(self) -> float:
        """Model output (log-odds) at the background point: logit(x = c) = sum a*c + bias."""
        return float(self.a[: self.d] @ self.c[: self.d] + self.bias)

    def health(self) -> bool:
        return bool(np.all(np.isfinite(self.a)) and np.isfinite(self.bias))


class TreeInferenceEngine(_EngineBase):
    """GBDT family: standardize -> tree ensemble (fdx-gbdt/1 JSON, no pickle)."""

    kind = "gbdt"
    methods = ("kernel", "tree")  # tree: interventional TreeSHAP of the margin (exact, log-odds)
    default_method = "kernel"

    def __init__(self, ensemble, mean, var, scale, feature_names, device: str = "auto", source: str = "local",
                 background: np.ndarray | None = None, kernel_nsamples: int = 0, kernel_link: str = "identity",
                 n_samples_seen: int = 0):
        from ..ops.scaler import stats_from_numpy

        self.ens = ensemble
        self.mean = np.asarray(mean, np.float64)
        self.var = np.asarray(var, np.float64)
        self.scale = np.asarray(scale, np.float64)
        self.d = len(self.mean)
        if ensemble.n_features != self.d:
            raise ValueError(f"ensemble has {ensemble.n_features} features, scaler {self.d}")
        self.feature_names = list(feature_names)
        self.n_samples_seen = n_samples_seen
        super().__init__(device, source, background, kernel_nsamples, kernel_link)
        self._stats = stats_from_numpy(self.mean, self.scale, device=self.device)
        if self.device.type == "cuda":
            from ..ops.gbdt import DeviceEnsemble

            self._dens = DeviceEnsemble(ensemble, self.device)
            self._stage = _Staging(self.device, self.d, 1)
            self._xstage = _Staging(self.device, self.d, self.d + 2)
        self._finish_init()

    @classmethod
    def from_paths(cls, model_path=None, scaler_path=None, features_path=None, device="auto", source="local",
                   **kw) -> "TreeInferenceEngine":
        import joblib

        from ..compat.sklearn_export import FEATURE_NAMES, _is_ours
        from ..compat import safe_joblib
        from ..ops.gbdt import TreeEnsemble

        model_path = model_path or os.getenv("MODEL_PATH", "./models/xgb_model.json")
        mdir = os.path.dirname(os.path.abspath(model_path))
        scaler_path = scaler_path or os.path.join(mdir, "scaler.joblib")
        features_path = features_path or os.path.join(mdir, "feature_names.json")
        with open(model_path) as f:
            o = json.load(f)
        ens = TreeEnsemble.from_dict(o)
        if _is_ours(mdir) or source == "mlflow":
            sc = joblib.load(scaler_path)
            mean, var, scale, nss = sc.mean_, sc.var_, sc.scale_, int(np.ravel(sc.n_samples_seen_)[0])
        else:
            s = safe_joblib.decode_scaler(scaler_path)
            mean, var, scale, nss = s["mean_"], s["var_"], s["scale_"], s["n_samples_seen"]
        names = o.get("feature_names")
        if not names and features_path and os.path.exists(features_path):
            with open(features_path) as f:
                names = json.load(f)
        return cls(ens, mean, var, scale, names or FEATURE_NAMES[: len(mean)], device=device, source=source,
                   background=load_background(mdir), n_samples_seen=nss, **kw)

    def predict_proba(self, X: np.ndarray):
        """-> (prob [B], margin [B])."""
        X = self._check(X)
        if self._use_host(X.shape[0]):
            return self._predict_host(X)
        return self._predict_device(X)

    def _predict_host(self, X: np.ndarray):
        from ..models.explainers import _standardize
        from ..ops import reference_gbdt as RG

        e = self.ens
        m = RG.predict_margin(_standardize(X, self.mean, self.scale), e.feat, e.thr, e.leaf, e.depth,
                              e.base_margin).astype(np.float64)
        return 1.0 / (1.0 + np.exp(-m)), m

    def _predict_device(self, X: np.ndarray):
        from ..ops import gbdt as gb
        from ..ops.scaler import scale_cast

        n = X.shape[0]
        with self._lock, torch.cuda.stream(self._stream):
            st = self._stage
            xd = st.upload(X)
            with _KernelTimer("gbdt_predict") as kt:
                rows = scale_cast(xd, self._stats, out_dtype="f32")
                margin = gb.predict_margin(rows[:, : self.d], self.ens, self._dens)
            st.dout[:n].copy_(margin)
            m = st.download(n).astype(np.float64)
            kt.observe()
        return 1.0 / (1.0 + np.exp(-m)), m

    def predict_explain(self, X: np.ndarray):
        """(prob, margin, phi) with KernelSHAP phi (the only explainer of a tree model here)."""
        e = self.explain(X, "kernel")
        return e.prob, e.logit, e.phi

    def tree_explainer(self):
        if getattr(self, "_texpl", None) is None:
            if not self.has_background:
                raise ValueError("TreeSHAP needs a background (shap_background.npy next to the model)")
            from ..models.explainers import TreeExplainer

            self._texpl = TreeExplainer(self.ens, self.mean, self.scale, self.background, device=str(self.device))
        return self._texpl

    def _explain_tree(self, X: np.ndarray) -> "Explanation":
        """Interventional TreeSHAP (log-odds): one staging upload, one launch sequence, one download."""
        te = self.tree_explainer()
        n, d = X.shape
        if self.device.type != "cuda" or n == 0:
            phi, fx, f0 = te.explain(X) if n else (np.zeros((0, d)), np.zeros(0), te.expected_value)
            return Explanation(1.0 / (1.0 + np.exp(-fx)), fx, np.asarray(phi, np.float64), float(f0), "tree",
                               "log-odds")
        from ..ops.treeshap import treeshap

        with self._lock, torch.cuda.stream(self._stream):
            st = self._xstage
            xd = st.upload(X)
            o = st.dout
            outs = (o[: n * d].view(n, d), o[n * d: n * d + n], o[n * d + n: n * d + 2 * n])
            with _KernelTimer("treeshap_gbdt") as kt:
                treeshap(xd, te, sync=False, out=outs)
            h = st.download(n * d + 2 * n)
            kt.observe()
        phi = h[: n * d].reshape(n, d).astype(np.float64)
        fx = h[n * d: n * d + n].astype(np.float64)
        return Explanation(1.0 / (1.0 + np.exp(-fx)), fx, phi, float(h[n * d + n]), "tree", "log-odds")

    def _make_kernel_explainer(self):
        from ..models.explainers import TreeKernelExplainer

        return TreeKernelExplainer(self.ens, self.mean, self.scale, self.background,
                                   nsamples=self.kernel_nsamples or None, link=self.kernel_link,
                                   device=str(self.device))

    def _kernel_device(self, xd, ke, out):
        from ..ops.kernelshap import kernelshap_tree

        return kernelshap_tree(xd, ke, sync=False, out=out)

    def _logit_host(self, X: np.ndarray) -> np.ndarray:
        from ..models.explainers import _standardize
        from ..ops import reference_gbdt as RG

        e = self.ens
        return RG.predict_margin(_standardize(X, self.mean, self.scale), e.feat, e.thr, e.leaf, e.depth,
                                 e.base_margin).astype(np.float64)

    def expected_value(self) -> float:
        return float(self.ens.base_margin)

    def health(self) -> bool:
        return bool(np.all(np.isfinite(self.ens.leaf)))


def load_engine_dir(model_dir: str, device="auto", source: str = "local", **kw) -> _EngineBase:
    """Engine for a model directory (local artifacts or a resolved MLflow model dir): GBDT when an
    fdx-gbdt JSON is present (xgb_model.json), else the linear joblib layout (model.pkl for
    MLflow's sklearn flavour, logistic_model.joblib locally)."""
    for name in ("xgb_model.json",):
        p = os.path.join(model_dir, name)
        if os.path.exists(p):
            return TreeInferenceEngine.from_paths(p, os.path.join(model_dir, "scaler.joblib"),
                                                  os.path.join(model_dir, "feature_names.json"), device, source, **kw)
    for name in ("model.pkl", "logistic_model.joblib"):
        p = os.path.join(model_dir, name)
        if os.path.exists(p):
            art = load_artifacts(p, os.path.join(model_dir, "scaler.joblib"),
                                 os.path.join(model_dir, "feature_names.json"),
                                 trusted=True if source == "mlflow" else None)
            return InferenceEngine(art, device=device, source=source, background=load_background(model_dir), **kw)
    raise FileNotFoundError(f"no model artifacts in {model_dir}")
