"""K11 GBDT ops: quantile binning, boosting rounds and inference (csrc/kernels/gbdt.hip).

Device path: one boosting round = gradient kernel -> per level (histogram, [RCCL all-reduce of the
int64 histograms and child counts under DP], split, stable partition) -> leaf values -> margin
update.  Nothing in a round synchronises with the host.  CPU tensors run the numpy oracle
(ops/reference_gbdt.py), which builds the same trees from the same quantised gradients.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np
import torch

from . import reference_gbdt as R
from .native import native, ptr, stream_of

MAX_BIN = R.MAX_BIN
MAX_FEAT = 30
HIST_ENTRIES = MAX_FEAT * MAX_BIN * 2
# partition grid (<= 4096): 2048 blocks of 256 -- count kernel 57.5 us vs 62.0 at 1024 per level at
# 16M rows, scatter unchanged; 4096 and 512 slower, and 8 rows per thread instead of 4 slowed both
# kernels (67-79 us) (profiles/r5_zp, r5_zq)
PART_BLOCKS = int(os.environ.get("FDX_GBDT_PART_BLOCKS", "2048"))


@dataclass
class GBDTParams:
    """xgboost.XGBClassifier parameter names and defaults used by train_model.py:69-80."""
    n_estimators: int = 100
    learning_rate: float = 0.1
    max_depth: int = 5
    reg_lambda: float = 1.0
    min_child_weight: float = 1.0
    gamma: float = 0.0
    max_bin: int = 256
    scale_pos_weight: float = 1.0
    base_score: float = 0.5
    cut_sample_rows: int = 1 << 20

    def validate(self):
        if not 1 <= self.max_depth <= 7:
            raise ValueError("max_depth must be in [1, 7] (node ids are stored in one byte)")
        if not 2 <= self.max_bin <= MAX_BIN:
            raise ValueError("max_bin must be in [2, 256]")
        if not 0.0 < self.base_score < 1.0:
            raise ValueError("base_score must be in (0, 1)")
        if self.n_estimators < 0 or self.learning_rate <= 0:
            raise ValueError("bad n_estimators / learning_rate")
        return self


@dataclass
class TreeEnsemble:
    depth: int
    feat: np.ndarray   # [T, 2^D - 1] int32 (-1 = pass-through)
    bin: np.ndarray    # [T, 2^D - 1] int32
    thr: np.ndarray    # [T, 2^D - 1] float32
    gain: np.ndarray   # [T, 2^D - 1] float64
    leaf: np.ndarray   # [T, 2^D] float32
    cuts: np.ndarray   # [d, 256] float32
    nbins: np.ndarray  # [d] int32
    base_score: float = 0.5
    params: dict = field(default_factory=dict)

    @property
    def n_trees(self) -> int:
        return int(self.feat.shape[0])

    @property
    def n_features(self) -> int:
        return int(self.nbins.shape[0])

    @property
    def base_margin(self) -> float:
        return float(np.log(self.base_score / (1.0 - self.base_score)))

    def feature_importance(self, kind: str = "gain") -> np.ndarray:
        """xgboost-style importances: "gain" (mean gain per split) or "weight" (split count)."""
        d = self.n_features
        cnt = np.zeros(d)
        tot = np.zeros(d)
        m = self.feat >= 0
        np.add.at(cnt, self.feat[m], 1.0)
        np.add.at(tot, self.feat[m], self.gain[m])
        if kind == "weight":
            return cnt
        return np.where(cnt > 0, tot / np.maximum(cnt, 1), 0.0)

    def to_dict(self) -> dict:
        return {"format": "fdx-gbdt/1", "depth": self.depth, "base_score": self.base_score,
                "params": self.params, "feat": self.feat.tolist(), "bin": self.bin.tolist(),
                "thr": [[float(v) if np.isfinite(v) else "inf" for v in row] for row in self.thr],
                "gain": self.gain.tolist(), "leaf": self.leaf.tolist(),
                "cuts": [[float(v) if np.isfinite(v) else "inf" for v in row[:nb]] for row, nb in zip(self.cuts, self.nbins)],
                "nbins": self.nbins.tolist()}

    @classmethod
    def from_dict(cls, o: dict) -> "TreeEnsemble":
        if o.get("format") != "fdx-gbdt/1":
            raise ValueError("not an fdx-gbdt/1 model")
        f = lambda v: np.inf if v == "inf" else float(v)  # noqa: E731
        depth = int(o["depth"])
        ni = (1 << depth) - 1
        nbins = np.asarray(o["nbins"], np.int32)
        cuts = np.full((len(nbins), MAX_BIN), np.inf, np.float32)
        for i, row in enumerate(o["cuts"]):
            cuts[i, : len(row)] = [f(v) for v in row]
        feat = np.asarray(o["feat"], np.int32).reshape(-1, ni)
        return cls(depth=depth, feat=feat, bin=np.asarray(o["bin"], np.int32).reshape(-1, ni),
                   thr=np.asarray([[f(v) for v in row] for row in o["thr"]], np.float32).reshape(-1, ni),
                   gain=np.asarray(o["gain"], np.float64).reshape(-1, ni),
                   leaf=np.asarray(o["leaf"], np.float32).reshape(-1, 1 << depth), cuts=cuts, nbins=nbins,
                   base_score=float(o["base_score"]), params=dict(o.get("params", {})))


# ---- binning ---------------------------------------------------------------------------------
def quantile_cuts(X: torch.Tensor, max_bin: int = MAX_BIN, sample_rows: int = 1 << 20, comm=None):
    """Per-feature quantile cuts from a deterministic strided row sample.  Under DP every rank
    contributes a sample and the cuts come from the gathered sample, so all ranks agree."""
    n, d = X.shape
    if d > MAX_FEAT:
        raise ValueError(f"at most {MAX_FEAT} features")
    world = comm.world_size if comm is not None else 1
    per = max(1, sample_rows // world)
    stride = max(1, n // per)
    if comm is not None and world > 1:
        samp, _ = comm.all_gather_rows(X[::stride][:per].contiguous())
        src, m, step = samp, samp.shape[0], 1
    else:
        src, m, step = X, min(per, (n + stride - 1) // stride), stride
    if not src.is_cuda:
        return R.quantile_cuts(src[::step][:m].float().numpy(), max_bin)
    # Exact order statistics by a native radix select (quantile.hip): the minimum and the max_bin - 1
    # quantile rows of the sample come back to the host, where deduplication is trivial.  Selection
    # is exact, so the cuts equal the CPU oracle's (np.sort) on the same sample.
    if src.dtype != torch.float32 or src.stride(1) != 1:
        src, step = src[::step][:m].float().contiguous(), 1
    nat = native()
    ws = torch.empty(nat.quantile_select_ws_bytes(m, d), dtype=torch.uint8, device=src.device)
    picks = torch.empty((max_bin, d), dtype=torch.float32, device=src.device)
    nat.quantile_select(ptr(src), m, step, src.stride(0), d, max_bin, ptr(ws), ptr(picks), stream_of(src))
    picks = picks.cpu().numpy()
    return R.cuts_from_sorted_picks(picks[1:], picks[0], max_bin)


def bin_rows(X: torch.Tensor, cuts: np.ndarray, nbins: np.ndarray, out: torch.Tensor | None = None) -> torch.Tensor:
    """u8 [n, 32] bins (features in bytes 0..d-1).  ``out``: a [n, 32] u8 view to write (e.g. the
    SMOTE tail of a binned table)."""
    n, d = X.shape
    if out is not None and (tuple(out.shape) != (n, R.ROW_BYTES) or out.dtype != torch.uint8
                            or not out.is_contiguous() or out.device != X.device):
        raise ValueError("out must be a contiguous u8 [n, 32] tensor on X's device")
    if not X.is_cuda:
        b = torch.from_numpy(R.bin_rows(X.numpy(), cuts, nbins))
        return out.copy_(b) if out is not None else b
    if X.dtype != torch.float32 or X.stride(1) != 1:
        raise ValueError("X must be float32 with unit column stride")
    m = native()
    out = out if out is not None else torch.empty((n, R.ROW_BYTES), dtype=torch.uint8, device=X.device)
    ct = torch.from_numpy(np.ascontiguousarray(cuts[:d])).to(X.device)
    nt = torch.from_numpy(np.ascontiguousarray(nbins[:d])).to(X.device)
    if n:
        m.gbdt_bin(ptr(X), n, X.stride(0), d, ptr(ct), ptr(nt), ptr(out), stream_of(X))
    return out


# ---- training --------------------------------------------------------------------------------
# Rows a histogram block accumulates in LDS between flushes to its slot (0: the kernel's bound,
# 2^16 -- packed (h, g) words stay exact); tests lower it to exercise the multi-flush path.
HIST_FLUSH_ROWS = 0


class _Workspace:
    def __init__(self, n: int, depth: int, dev: torch.device):
        nheap = (2 << depth) - 1
        self.gh = torch.empty((n, 2), dtype=torch.int16, device=dev)  # (g, h) packed in 4 bytes
        self.ridx = [torch.empty(n, dtype=torch.int32, device=dev) for _ in range(2)]
        self.nid = [torch.empty(n, dtype=torch.uint8, device=dev) for _ in range(2)]
        self.flag = torch.empty(max(n, 1), dtype=torch.uint8, device=dev)
        self.counts = torch.empty(PART_BLOCKS, dtype=torch.int64, device=dev)  # right rows per partition block
        self.seg = torch.zeros((nheap, 2), dtype=torch.int64, device=dev)
        self.node_r = torch.zeros(nheap, dtype=torch.int64, device=dev)  # right rows per node (zeroed per round)
        self.gcnt = torch.zeros(nheap, dtype=torch.int64, device=dev)
        self.hist = torch.zeros(((1 << depth) - 1) * HIST_ENTRIES, dtype=torch.int64, device=dev)
        # per-(node, block) histogram slots the histogram kernel writes without atomics
        self.slots = torch.empty(native().gbdt_hist_slot_words(), dtype=torch.int64, device=dev)
        self.ng = torch.zeros(nheap, dtype=torch.int64, device=dev)
        self.nh = torch.zeros(nheap, dtype=torch.int64, device=dev)


def _resume(checkpoint, sig, T):
    """Trees of a matching checkpoint (numpy arrays) and how many rounds they cover."""
    if checkpoint is None:
        return None, 0
    got = checkpoint.latest(sig)
    if got is None:
        return None, 0
    tensors, meta = got
    t0 = min(int(meta["trees_done"]), T)
    return {k: v.numpy()[:t0] for k, v in tensors.items()}, t0


def fit(X: torch.Tensor, y: torch.Tensor, params: GBDTParams | None = None, comm=None,
        cuts=None, sample_weight_pos: float | None = None, return_margin: bool = False,
        checkpoint=None, checkpoint_every: int = 10, use_graph: bool | None = None):
    """Boost `n_estimators` depth-D trees on standardized float32 rows X [n, d] with labels y.

    ``checkpoint``: a utils.checkpoint.CheckpointManager.  Every ``checkpoint_every`` rounds the
    trees so far are saved; a later call with the same data/config resumes after the last saved
    round.  Training margins are recomputed from the saved trees over the same bins, so a resumed
    fit is bit-identical to an uninterrupted one."""
    p = (params or GBDTParams()).validate()
    n, d = X.shape
    if d > MAX_FEAT:
        raise ValueError(f"at most {MAX_FEAT} features")
    if cuts is None:
        cuts = quantile_cuts(X, p.max_bin, p.cut_sample_rows, comm)
    bins = bin_rows(X, cuts[0], cuts[1])
    return fit_binned(bins, y, cuts, p, comm=comm, sample_weight_pos=sample_weight_pos, return_margin=return_margin,
                      checkpoint=checkpoint, checkpoint_every=checkpoint_every, use_graph=use_graph)


def fit_binned(bins: torch.Tensor, y: torch.Tensor, cuts, params: GBDTParams | None = None, comm=None,
               sample_weight_pos: float | None = None, return_margin: bool = False, checkpoint=None,
               checkpoint_every: int = 10, use_graph: bool | None = None, hole: tuple | None = None):
    """Boosting on already-binned rows (u8 [n, 32], bin_rows) with their cuts (cuts, nbins).

    ``hole``: (at, len) -- the fit's rows are the table without the block [at, at + len) (a
    cross-validation fold on the fold-sorted table: no per-fold copy).  The returned margin (with
    ``return_margin``) covers EVERY table row, so the block's margins are the fold's validation
    scores under the fitted ensemble."""
    p = (params or GBDTParams()).validate()
    cuts_np, nbins = cuts
    d = int(len(nbins))
    n = int(bins.shape[0])  # table rows (the margin walk covers all of them)
    if d > MAX_FEAT:
        raise ValueError(f"at most {MAX_FEAT} features")
    if y.dtype != torch.uint8 or y.shape[0] != n:
        raise ValueError("y must be uint8 [n] (one label per table row)")
    ha, hl = (int(hole[0]), int(hole[1])) if hole else (0, 0)
    if ha < 0 or hl < 0 or ha + hl > n:
        raise ValueError(f"hole {hole} outside the {n} table rows")
    n_fit = n - hl
    spw = float(p.scale_pos_weight if sample_weight_pos is None else sample_weight_pos)
    gscale, hscale = R.grad_scales(spw)
    D = p.max_depth
    ni, nl = (1 << D) - 1, 1 << D
    T = p.n_estimators
    base_margin = float(np.log(p.base_score / (1.0 - p.base_score)))
    ens_kw = dict(depth=D, cuts=cuts_np, nbins=nbins, base_score=p.base_score, params=dict(p.__dict__))
    sig = None
    if checkpoint is not None:
        from ..utils.checkpoint import config_signature

        n_all = int(comm.all_reduce_scalar(float(n_fit))) if (comm is not None and comm.world_size > 1) else n_fit
        sig = config_signature(params={k: v for k, v in p.__dict__.items() if k != "n_estimators"}, spw=spw,
                               cuts=cuts_np, nbins=nbins, n=n_all, d=d, **({"hole": [ha, hl]} if hl else {}))
    prev, t0 = _resume(checkpoint, sig, T)

    def _save(t_done, feat, binv, thr, gain, leaf):
        if checkpoint is not None and t_done > 0:
            checkpoint.save(t_done, {"feat": feat[:t_done], "bin": binv[:t_done], "thr": thr[:t_done],
                                     "gain": gain[:t_done], "leaf": leaf[:t_done]},
                            {"signature": sig, "trees_done": t_done, "kind": "gbdt"})
            fault = os.environ.get("FDX_FAULT", "")
            if fault.startswith("gbdt_crash_after_trees=") and t_done >= int(fault.split("=", 1)[1]):
                os._exit(17)  # simulated lost rank right after a checkpoint (resume tests)

    if not bins.is_cuda:
        feat = np.zeros((T, ni), np.int32); binv = np.zeros((T, ni), np.int32)
        thr = np.zeros((T, ni), np.float32); gain = np.zeros((T, ni)); leaf = np.zeros((T, nl), np.float32)
        b_all = bins.numpy()
        y_all = y.numpy()
        keep = np.r_[0:ha, ha + hl:n]
        b, yy = b_all[keep], y_all[keep]
        margin = np.full(n_fit, np.float32(base_margin), np.float32)
        if t0:
            feat[:t0], binv[:t0], thr[:t0], gain[:t0], leaf[:t0] = (prev[k] for k in ("feat", "bin", "thr", "gain", "leaf"))
            margin = R.predict_margin_bins(b, feat[:t0], binv[:t0], leaf[:t0], D, base_margin)
        for t in range(t0, T):
            q = R.gradients(margin, yy, spw, gscale, hscale)
            tr, node = R.build_tree(b, q, cuts_np, nbins, D, p.reg_lambda, p.min_child_weight, p.gamma,
                                    p.learning_rate, gscale, hscale, comm)
            feat[t], binv[t], thr[t], gain[t], leaf[t] = tr.feat, tr.bin, tr.thr, tr.gain, tr.leaf
            margin = (margin + tr.leaf[node]).astype(np.float32)
            if (t + 1) % max(1, checkpoint_every) == 0 or t + 1 == T:
                _save(t + 1, feat, binv, thr, gain, leaf)
        ens = TreeEnsemble(feat=feat, bin=binv, thr=thr, gain=gain, leaf=leaf, **ens_kw)
        if not return_margin:
            return ens
        full = np.empty(n, np.float32)
        full[keep] = margin
        if hl:
            full[ha:ha + hl] = R.predict_margin_bins(b_all[ha:ha + hl], feat, binv, leaf, D, base_margin)
        return ens, torch.from_numpy(full)

    m = native()
    dev = bins.device
    st0 = stream_of(bins)
    ws = _Workspace(n, D, dev)
    # feature-major copy of the bins for the partition's one-byte-per-row reads (gbdt.hip)
    ldt = max(4, (n + 255) // 256 * 256)
    binsT = torch.empty(d * ldt, dtype=torch.uint8, device=dev)
    if n:
        m.gbdt_transpose(ptr(bins), n, d, ptr(binsT), ldt, st0)
    dist = comm is not None and comm.world_size > 1
    n_global = int(comm.all_reduce_scalar(float(n_fit))) if dist else n_fit
    ct = torch.from_numpy(np.ascontiguousarray(cuts_np[:d])).to(dev)
    nt = torch.from_numpy(np.ascontiguousarray(nbins[:d])).to(dev)
    feat = torch.empty((T, ni), dtype=torch.int32, device=dev)
    binv = torch.empty((T, ni), dtype=torch.int32, device=dev)
    thr = torch.empty((T, ni), dtype=torch.float32, device=dev)
    gain = torch.empty((T, ni), dtype=torch.float64, device=dev)
    leaf = torch.empty((T, nl), dtype=torch.float32, device=dev)
    margin = torch.full((n,), base_margin, dtype=torch.float32, device=dev)
    if t0:
        for name, dst in (("feat", feat), ("bin", binv), ("thr", thr), ("gain", gain), ("leaf", leaf)):
            dst[:t0].copy_(torch.from_numpy(np.ascontiguousarray(prev[name])))
        for t in range(t0):  # the margins of the saved trees, by the round's own margin kernel
            m.gbdt_margin(ptr(binsT), ldt, n, ptr(feat[t]), ptr(binv[t]), ptr(leaf[t]), D, ptr(margin), ptr(y), spw,
                          gscale, hscale, 0, st0)
    lam, mcw, gam = float(p.reg_lambda), float(p.min_child_weight), float(p.gamma)
    ginv, hinv = 1.0 / gscale, 1.0 / hscale

    def round_body(o_feat, o_bin, o_thr, o_gain, o_leaf, grad_first=False, grad_next=True, prev=None,
                   defer_margin=False):
        """One boosting round: a fixed launch sequence with static pointers (graph-capturable).
        The gradients of a round come from the previous round's margin update (gbdt_margin with
        gh), so only the first round of a fit launches gbdt_grad.  ``prev`` (feat, bin, leaf of the
        previous tree, its margin walk deferred): level 0 runs that walk fused in front of its
        histogram (gbdt_hist_l0_fused).  ``defer_margin``: leave this tree's walk to the next round."""
        st = stream_of(bins)  # the capture stream while a hipGraph is being recorded
        if grad_first:
            m.gbdt_grad(ptr(margin), ptr(y), n, spw, gscale, hscale, ptr(ws.gh), st)
        # zero histograms and per-node counts, root segment + global count: one launch (level 0
        # reads rows in order, so ridx / nid need no iota / root fill)
        m.gbdt_round_init(ptr(ws.hist), ws.hist.numel(), ptr(ws.seg), ptr(ws.gcnt), n_fit, n_global, st,
                          ptr(ws.node_r), ws.node_r.numel())
        cur = 0
        for level in range(D):
            h0, nn = (1 << level) - 1, 1 << level
            if level == 0 and prev is not None:
                m.gbdt_hist_l0_fused(ptr(bins), ptr(ws.gh), ptr(ws.seg), ptr(ws.gcnt), d, ptr(ws.hist), ptr(ws.slots),
                                     st, HIST_FLUSH_ROWS, ha, hl, ptr(prev[0]), ptr(prev[1]), ptr(prev[2]), D,
                                     ptr(margin), ptr(y), spw, gscale, hscale)
            else:
                m.gbdt_hist(ptr(bins), ptr(ws.gh), ptr(ws.ridx[cur]), ptr(ws.seg), ptr(ws.gcnt), level, d,
                            ptr(ws.hist), ptr(ws.slots), st, HIST_FLUSH_ROWS, ha, hl)
            if dist:
                comm.all_reduce_(ws.hist[h0 * HIST_ENTRIES:(h0 + nn) * HIST_ENTRIES])
            m.gbdt_split(ptr(ws.hist), ptr(ws.gcnt), level, d, ptr(nt), ptr(ct), ginv, hinv, lam, mcw, gam,
                         ptr(o_feat), ptr(o_bin), ptr(o_thr), ptr(o_gain), ptr(ws.ng), ptr(ws.nh), st)
            if level == D - 1:
                break  # leaves: the margin walk and gbdt_leaf (split-kernel child sums) need no partition
            if n_fit:
                # count + scatter; the scatter also writes the children's segments and counts (gcnt)
                m.gbdt_partition(ptr(binsT), ldt, ptr(ws.ridx[cur]), ptr(ws.nid[cur]), n_fit, ptr(o_feat), ptr(o_bin),
                                 level, ptr(ws.flag), ptr(ws.counts), PART_BLOCKS, ptr(ws.seg), ptr(ws.node_r),
                                 ptr(ws.ridx[cur ^ 1]), ptr(ws.nid[cur ^ 1]), st, ptr(ws.gcnt), ha, hl)
            cur ^= 1
            c0 = 2 * h0 + 1
            if not n_fit:
                ws.seg[2 * h0 + 1:2 * (h0 + nn) + 1].zero_()
                ws.gcnt[c0:c0 + 2 * nn].zero_()
            if dist:
                comm.all_reduce_(ws.gcnt[c0:c0 + 2 * nn])
        m.gbdt_leaf(ptr(ws.ng), ptr(ws.nh), D, ginv, hinv, lam, mcw, float(p.learning_rate), ptr(o_leaf), st)
        if n and not defer_margin:
            m.gbdt_margin(ptr(binsT), ldt, n, ptr(o_feat), ptr(o_bin), ptr(o_leaf), D, ptr(margin), ptr(y), spw,
                          gscale, hscale, ptr(ws.gh) if grad_next else 0, st)

    def after_round(t):
        if checkpoint is not None and ((t + 1) % max(1, checkpoint_every) == 0 or t + 1 == T):
            _save(t + 1, feat, binv, thr, gain, leaf)  # device -> host copy: syncs every k rounds only

    # hipGraph: a round is ~5 + 6*D launches with static shapes, so after one eager round it is
    # recorded once and replayed (one graph launch per round instead of ~45 Python->HIP launches;
    # the per-round tree lands in a fixed record and is copied into its slot).  Not under DP,
    # where the round contains host-side collectives.  Opt-in (FDX_GBDT_GRAPH=1): eager launches
    # already run ahead of the GPU, and replay + record copies measured 0.61 vs 0.50 ms/tree at
    # 0.96M rows and 1.62 vs 1.54 at 6.4M (profiles/r1_s22).
    if use_graph is None:  # opt-in: measured slower than eager launches (profiles/r1_s22)
        use_graph = os.environ.get("FDX_GBDT_GRAPH", "0") == "1"
    graphable = use_graph and not dist and n > 0 and T - t0 >= 3
    fuse_margin = os.environ.get("FDX_GBDT_FUSE_MARGIN", "0") == "1" and not graphable
    graph = None
    for t in range(t0, T):
        if graphable and t == t0 + 1:  # round t0 ran eagerly: its kernels had to execute
            from ..runtime.graphs import capture

            rec = [torch.empty(ni, dtype=torch.int32, device=dev), torch.empty(ni, dtype=torch.int32, device=dev),
                   torch.empty(ni, dtype=torch.float32, device=dev), torch.empty(ni, dtype=torch.float64, device=dev),
                   torch.empty(nl, dtype=torch.float32, device=dev)]
            graph = capture(lambda: round_body(*rec))
        if graph is not None:
            graph.replay()
            for dst, src in zip((feat[t], binv[t], thr[t], gain[t], leaf[t]), rec):
                dst.copy_(src)
        else:
            # FDX_GBDT_FUSE_MARGIN=1: a round's margin walk runs fused into the next round's level-0
            # histogram pass (one pass over the table fewer) -- measured slower: 410 us for the fused
            # pass against 151 + 140 us (its per-row fp64 phase and the LANE phase alternate behind
            # block barriers, 64-VGPR budget, profiles/r6_gbdt), so opt-in
            fuse = fuse_margin and n_fit > 0
            round_body(feat[t], binv[t], thr[t], gain[t], leaf[t], grad_first=(t == t0), grad_next=(t + 1 < T),
                       prev=(feat[t - 1], binv[t - 1], leaf[t - 1]) if (fuse and t > t0) else None,
                       defer_margin=fuse and t + 1 < T)
        after_round(t)
    ens = TreeEnsemble(feat=feat.cpu().numpy(), bin=binv.cpu().numpy(), thr=thr.cpu().numpy(),
                       gain=gain.cpu().numpy(), leaf=leaf.cpu().numpy(), **ens_kw)
    return (ens, margin) if return_margin else ens


# ---- inference -------------------------------------------------------------------------------
class DeviceEnsemble:
    """Tree arrays resident on a device for repeated inference."""

    def __init__(self, ens: TreeEnsemble, device: torch.device):
        self.ens = ens
        self.device = device
        self.feat = torch.from_numpy(np.ascontiguousarray(ens.feat)).to(device)
        self.thr = torch.from_numpy(np.ascontiguousarray(ens.thr)).to(device)
        self.leaf = torch.from_numpy(np.ascontiguousarray(ens.leaf)).to(device)


def predict_margin(X: torch.Tensor, ens: TreeEnsemble, dens: DeviceEnsemble | None = None) -> torch.Tensor:
    """float32 margins of standardized rows X [n, d] (d <= 30, any row stride)."""
    n, d = X.shape
    if d != ens.n_features:
        raise ValueError(f"model has {ens.n_features} features, X has {d}")
    if not X.is_cuda:
        return torch.from_numpy(R.predict_margin(X.numpy(), ens.feat, ens.thr, ens.leaf, ens.depth, ens.base_margin))
    if X.dtype != torch.float32 or X.stride(1) != 1:
        raise ValueError("X must be float32 with unit column stride")
    dens = dens if dens is not None and dens.device == X.device else DeviceEnsemble(ens, X.device)
    out = torch.empty(n, dtype=torch.float32, device=X.device)
    if n:
        native().gbdt_predict(ptr(X), n, X.stride(0), d, ptr(dens.feat), ptr(dens.thr), ptr(dens.leaf), ens.n_trees,
                              ens.depth, ens.base_margin, ptr(out), stream_of(X))
    return out


def predict_proba(X: torch.Tensor, ens: TreeEnsemble, dens: DeviceEnsemble | None = None) -> torch.Tensor:
    return torch.sigmoid(predict_margin(X, ens, dens))
