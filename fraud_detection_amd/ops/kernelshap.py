"""K7 KernelSHAP device wrappers (csrc/kernels/kernelshap.hip): the linear-model MFMA coalition
GEMM and the tree-ensemble masked-evaluation kernel, sharing the WLS projection.

Work is split into ``parts`` coalition ranges per explanation so that E x parts workgroups fill
the 256 CUs in whole dispatch rounds (a 512-explanation worker lease would otherwise leave half
the device idle, and 1100 explanations would run a second, mostly empty round).  Partials of an
explanation are summed in part order by the last part to arrive, so results do not depend on
scheduling (tests/test_kernelshap.py checks run-to-run bit identity per part count; different
part counts differ only in the fp32 summation order of the projection).
"""
from __future__ import annotations


import numpy as np
import torch

from .native import native, ptr, stream_of

_LINKS = {"identity": 0, "logit": 1, "logit_model": 2}
MAX_PARTS = 8


def choose_parts(n_expl: int, n_tiles: int, target_wgs: int) -> int:
    """Coalition parts per explanation: split only while E x P is below ``target_wgs`` (enough
    workgroups to keep every SIMD issuing).  A split costs each extra part its own U build / f0
    and an agent-coherent hand-off of its partial projection.  Round 6 replaced the hand-off's
    release fence (an L2 write-back per workgroup: P = 2 ran 2-4x slower than P = 1) with
    agent-scope stores/loads (profiles/r6_ks): P = 4 now wins for small batches (64 explanations
    13.6 vs 23.0 us, identity link) and P = 1 from ~512 explanations (33.6 vs 33.7 / 38.0 us)."""
    if n_expl <= 0:
        return 1
    return int(max(1, min(MAX_PARTS, max(1, n_tiles // 4), -(-target_wgs // n_expl))))


def _cu_count(dev) -> int:
    return int(native().device_info(dev.index or 0)["cu_count"])


class _Workspace:
    """Partial-projection workspace [E, 8, 32] f32 + arrival counters [E] u32 (kept zeroed by the
    kernel itself), grown on demand, one per device."""

    def __init__(self):
        self.ws = None
        self.cnt = None

    def get(self, E: int, dev):
        if self.ws is None or self.ws.shape[0] < E or self.ws.device != dev:
            cap = max(E, 1024)
            self.ws = torch.empty((cap, MAX_PARTS, 32), device=dev, dtype=torch.float32)
            self.cnt = torch.zeros(cap, device=dev, dtype=torch.int32)
        return self.ws, self.cnt


def _check_x(X, d):
    if X.dim() != 2 or X.dtype != torch.float32 or X.shape[1] != d or not X.is_contiguous():
        raise ValueError(f"X must be contiguous float32 [E, {d}]")


def complement_pairs(Z: np.ndarray):
    """Split a coalition design into (base [P], comp [P]) row indices with Z[comp[p]] = 1 - Z[base[p]]
    (comp = -1 where the complement is not in the design).  shap's sampler draws coalitions in
    complement pairs, so P is ~S/2 (2042 rows at M = 30 -> 1032 pairs)."""
    keys = {z.tobytes(): i for i, z in enumerate(Z)}
    used = np.zeros(len(Z), bool)
    base, comp = [], []
    for i, z in enumerate(Z):
        if used[i]:
            continue
        used[i] = True
        j = keys.get((1 - z).tobytes(), -1)
        if j >= 0 and not used[j]:
            used[j] = True
        else:
            j = -1
        base.append(i)
        comp.append(j)
    return np.asarray(base, np.int64), np.asarray(comp, np.int64)


def _paired_enabled(link: str, paired: bool | None = None) -> bool:
    """The complement-paired kernel runs for the log-odds link, the unpaired one for the sigmoid
    links (``paired`` forces one -- tests and tools/ks_check.py).  Measured on MI355X
    (profiles/r2_s5): with the sigmoid links both run ~55 us per 1k batch (bound by the sigmoid
    epilogue's issue rate); the log-odds link has no epilogue and the paired kernel's half MFMA
    work shows, 25.2 vs 34.4 us."""
    if paired is not None:
        return bool(paired)
    return link == "logit_model"


def _device_design(expl, dev, paired: bool | None = None):
    """Upload the linear explainer's design once: Z as bf16 [S_pad, 32] (col 31 = 1 folds the
    background intercepts into the GEMM), A [d-1, S_pad] (zero-padded), A z_M, the weighted
    background rows W and the background logits.

    Paired layout (kernelshap_paired_kernel): Z holds the Ppad base coalitions of the
    complement pairs and A [d-1, 2 Ppad] has the base columns first, then each base's complement
    (zero columns for padding and for complements the design does not contain: they carry no
    weight, so the WLS solution is unchanged)."""
    key = (str(dev), _paired_enabled(expl.link, paired))
    if expl._dev_cache is not None and expl._dev_cache[0] == key:
        return expl._dev_cache[1]
    d = expl.d
    S = expl.Z.shape[0]
    paired = key[1]
    if paired:
        base, comp = complement_pairs(expl.Z)
        Ppad = (len(base) + 31) // 32 * 32
        if 2 * Ppad > 4096:
            raise ValueError("at most 2048 coalition pairs per design on device")
        Zp = np.zeros((Ppad, 32), np.float32)
        Zp[: len(base), :d] = expl.Z[base]
        Ap = np.zeros((d - 1, 2 * Ppad), np.float32)
        Ap[:, : len(base)] = expl.A[:, base]
        has = comp >= 0
        Ap[:, Ppad + np.nonzero(has)[0]] = expl.A[:, comp[has]]
        S_pad = 2 * Ppad
    else:
        S_pad = (S + 31) // 32 * 32
        if S_pad > 4096:
            raise ValueError("at most 4096 coalitions per design on device")
        Zp = np.zeros((S_pad, 32), np.float32)
        Zp[:S, :d] = expl.Z
        Ap = np.zeros((d - 1, S_pad), np.float32)
        Ap[:, :S] = expl.A
        Zp[:, 30] = 1.0  # the epilogue's exp2 shift rides in U column 30 (kernelshap.hip kPairShift)
    Zp[:, 31] = 1.0
    a32 = np.zeros(32, np.float32)
    a32[:d] = expl.a[:d]
    cb = (expl.B.astype(np.float64) @ expl.a[:d] + expl.bias).astype(np.float32)
    # W = [a o B_b, 0.., -c_b]: u_b = a o x - W_b, with u_b[31] = c_b folding the intercepts
    W = np.zeros((expl.B.shape[0], 32), np.float32)
    W[:, :d] = (expl.B.astype(np.float32) * a32[:d][None, :]).astype(np.float32)
    W[:, 31] = -cb
    if paired:  # bitmasks: bit k = z_k, bit 31 = the intercept column
        Zb = (Zp[:, :31] > 0.5).astype(np.uint64) << np.arange(31, dtype=np.uint64)[None, :]
        # bit 30 = the epilogue's exp2 shift column (kernelshap.hip kPairShift)
        Zdev = torch.from_numpy((Zb.sum(1) | (1 << 30) | (1 << 31)).astype(np.uint32).view(np.int32)).to(dev)
    else:
        Zdev = torch.from_numpy(Zp).to(dev).to(torch.bfloat16).contiguous()
    t = {
        "Z": Zdev,
        "A": torch.from_numpy(Ap).to(dev).contiguous(),
        "Az": torch.from_numpy((expl.A @ expl.zM).astype(np.float32)).to(dev),
        "a": torch.from_numpy(a32).to(dev),
        "bg": torch.from_numpy(W).to(dev),
        "cb": torch.from_numpy(cb).to(dev),
        "S": S, "S_pad": S_pad, "paired": paired, "ws": _Workspace(),
    }
    expl._dev_cache = (key, t)
    return t


def _outputs(E, d, dev, out):
    if out is not None:
        phi, fx, f0 = out
        if phi.shape != (E, d) or fx.shape[0] != E or f0.shape[0] < E or not phi.is_contiguous():
            raise ValueError("out = (phi [E, d] contiguous, fx [E], f0 [E]) float32 device tensors")
        return phi, fx, f0
    return (torch.empty((E, d), device=dev, dtype=torch.float32), torch.empty(E, device=dev, dtype=torch.float32),
            torch.empty(E, device=dev, dtype=torch.float32))


def kernelshap(X: torch.Tensor, expl, sync: bool = True, stamps: torch.Tensor | None = None,
               parts: int | None = None, out=None, paired: bool | None = None):
    """Linear model.  X [E, d] raw fp32 on device -> (phi [E, d], fx [E], f0) (numpy if sync else
    device tensors).  ``stamps`` (int64 [E, 8], tools/kernelshap_stamps.py): per-explanation phase
    timestamps (forces parts = 1).  ``parts``: coalition parts per explanation (None = auto).
    ``out``: preallocated (phi, fx, f0) device tensors (e.g. views of one staging buffer).
    ``paired``: force the complement-paired (True) / unpaired (False) kernel (None: by link)."""
    _check_x(X, expl.d)
    m = native()
    dev = X.device
    t = _device_design(expl, dev, False if stamps is not None else paired)
    E = X.shape[0]
    # MFMA tiles of 32 coalitions (paired: 32 base coalitions, i.e. 64 with the complements)
    n_tiles = t["S_pad"] // (64 if t["paired"] else 32)
    if stamps is not None:
        if t["paired"]:
            raise ValueError("phase stamps exist only in the unpaired kernel")
        parts = 1
    elif parts is None:
        # E x P ~ 256 workgroups (profiles/r6_ks: 64 explanations run at P = 4, >= 512 at P = 1)
        parts = choose_parts(E, n_tiles, 256)
    parts = max(1, min(int(parts), MAX_PARTS, n_tiles))
    phi, fx, f0 = _outputs(E, expl.d, dev, out)
    ws, cnt = t["ws"].get(E, dev) if parts > 1 else (None, None)
    if t["paired"]:
        m.kernelshap_paired(ptr(X), E, expl.d, ptr(t["a"]), float(expl.bias), ptr(t["bg"]), ptr(t["cb"]),
                            expl.B.shape[0], ptr(t["Z"]), t["S_pad"] // 2, parts, ptr(t["A"]), ptr(t["Az"]),
                            _LINKS[expl.link], ptr(phi), ptr(fx), ptr(f0), ptr(ws), ptr(cnt), stream_of(X))
    else:
        m.kernelshap(ptr(X), E, expl.d, ptr(t["a"]), float(expl.bias), ptr(t["bg"]), ptr(t["cb"]), expl.B.shape[0],
                     ptr(t["Z"]), t["S"], t["S_pad"], parts, ptr(t["A"]), ptr(t["Az"]), _LINKS[expl.link], ptr(phi),
                     ptr(fx), ptr(f0), ptr(ws), ptr(cnt), stream_of(X), ptr(stamps))
    if not sync:
        return phi, fx, f0
    return phi.cpu().numpy().astype(np.float64), fx.cpu().numpy().astype(np.float64), float(f0[0].item()) if E else 0.0


def _tree_device_design(expl, dev):
    key = (str(dev),)
    if expl._dev_cache is not None and expl._dev_cache[0] == key:
        return expl._dev_cache[1]
    ens = expl.ens
    S = expl.Z.shape[0]
    S_pad = (S + 31) // 32 * 32
    if S_pad > 4096:
        raise ValueError("at most 4096 coalitions per design on device")
    Zm = np.zeros(S_pad, np.uint32)
    Zm[:S] = expl.zmasks
    Ap = np.zeros((expl.d - 1, S_pad), np.float32)
    Ap[:, :S] = expl.A
    from ..ops.scaler import stats_from_numpy

    t = {
        "feat": torch.from_numpy(np.ascontiguousarray(ens.feat, np.int32)).to(dev),
        "thr": torch.from_numpy(np.ascontiguousarray(ens.thr, np.float32)).to(dev),
        "leaf": torch.from_numpy(np.ascontiguousarray(ens.leaf, np.float32)).to(dev),
        "bw": torch.from_numpy(np.ascontiguousarray(expl.bw.view(np.int32))).to(dev),
        "Zm": torch.from_numpy(Zm.view(np.int32)).to(dev),
        "A": torch.from_numpy(Ap).to(dev).contiguous(),
        "Az": torch.from_numpy((expl.A @ expl.zM).astype(np.float32)).to(dev),
        "stats": stats_from_numpy(expl.mean, expl.scale, device=dev),
        "S": S, "S_pad": S_pad, "ws": _Workspace(),
    }
    expl._dev_cache = (key, t)
    return t


def kernelshap_tree(X: torch.Tensor, expl, sync: bool = True, parts: int | None = None, out=None):
    """Tree ensemble (models/explainers.TreeKernelExplainer).  X [E, d] RAW fp32 on device; the
    rows are standardized on device with the model's scaler (the same kernel as predict), then
    every (coalition, background row) masked row is walked through the ensemble in the kernel."""
    _check_x(X, expl.d)
    m = native()
    dev = X.device
    t = _tree_device_design(expl, dev)
    from ..ops.scaler import scale_cast

    E = X.shape[0]
    Xs = scale_cast(X, t["stats"], out_dtype="f32")  # [E, 32]
    n_tiles = t["S_pad"] // 32
    if parts is None:
        # a workgroup carries ms of work here: split until every CU holds 4 workgroups
        parts = choose_parts(E, n_tiles, 4 * _cu_count(dev))
    parts = max(1, min(int(parts), MAX_PARTS, n_tiles))
    ens = expl.ens
    phi, fx, f0 = _outputs(E, expl.d, dev, out)
    ws, cnt = t["ws"].get(E, dev) if parts > 1 else (None, None)
    m.kernelshap_tree(ptr(Xs), Xs.stride(0), E, expl.d, ptr(t["feat"]), ptr(t["thr"]), ptr(t["leaf"]), ens.n_trees,
                      ens.depth, float(ens.base_margin), ptr(t["bw"]), expl.bw.shape[1], expl.B.shape[0], ptr(t["Zm"]),
                      t["S"], t["S_pad"], parts, ptr(t["A"]), ptr(t["Az"]), _LINKS[expl.link], ptr(phi), ptr(fx),
                      ptr(f0), ptr(ws), ptr(cnt), stream_of(X))
    if not sync:
        return phi, fx, f0
    return phi.cpu().numpy().astype(np.float64), fx.cpu().numpy().astype(np.float64), float(f0[0].item()) if E else 0.0
