#!/usr/bin/env python3
"""CPU (fp64) exploration of SGD schedules on the bench distribution: 8M raw training rows ->
~16M post-SMOTE rows, standardized, the device's minibatch partition (row tiles of the 512-block
SGD grid, pick tiles of 16).  For each schedule: epoch-gradient max-norm at the end (the device's
convergence test), the exact objective of the returned weights against the Newton optimum on the
same training set, and the bytes the fit streams (in units of one full epoch).

A schedule is a list of epochs (lr scalar, subsample s): an epoch visits nb minibatches over
1/s of the rows (fine partition of nb * s chunks, every s-th chunk).

    python tools/sgd_schedule_lab.py [--rows 8000000] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from fraud_detection_amd.ops import reference as ref  # noqa: E402

FINE = 64  # finest partition: tile mod 64, (pick // 16) mod 64


def build(rows: int, seed: int = 1000):
    from fraud_detection_amd.data.synthetic import separable

    X, y = separable(rows, seed=seed)
    X = X.numpy().astype(np.float64)
    y = y.numpy().astype(np.float64)
    mu, sd = X.mean(0), X.std(0)
    Xs = (X - mu) / sd
    n = Xs.shape[0]
    R = np.zeros((n, 32))
    R[:, :30] = Xs
    R[:, 30] = 1.0
    R[:, 31] = y
    R = R.astype(np.float32).astype(np.float64)  # like bf16-ish storage noise? keep fp32 rounding
    mins = np.nonzero(y > 0.5)[0]
    P = R[mins]
    k = 5
    F = P[:, :30]
    sq = (F * F).sum(1)
    idx = np.empty((len(P), k), dtype=np.int64)
    for i0 in range(0, len(P), 2048):
        d2 = sq[i0:i0 + 2048, None] + sq[None, :] - 2.0 * F[i0:i0 + 2048] @ F.T
        d2[np.arange(d2.shape[0]), i0 + np.arange(d2.shape[0])] = np.inf
        part = np.argpartition(d2, k, axis=1)[:, :k]
        order = np.take_along_axis(d2, part, 1).argsort(1)
        idx[i0:i0 + 2048] = np.take_along_axis(part, order, 1)
    n_new = int(n - 2 * len(mins))
    rng = np.random.default_rng(42)
    picks = rng.integers(0, len(mins) * k, n_new)
    lam = rng.random(n_new)
    a = P[picks // k]
    b = P[idx.reshape(-1)[picks]]
    S = a + lam[:, None] * (b - a)
    S[:, 31] = 1.0
    cr = (np.arange(n) // 64) % FINE
    cs = (picks // 16) % FINE
    chunks = []
    for c in range(FINE):
        chunks.append(np.concatenate([R[cr == c], S[cs == c]]))
    return chunks


def sums(Rb, w):
    X = Rb[:, :32].copy()
    y = X[:, 31].copy()
    X[:, 31] = 0.0
    z = X @ w
    p = 1.0 / (1.0 + np.exp(-z))
    g = X.T @ (p - y)
    loss = float(np.sum(np.logaddexp(0.0, z) - y * z))
    return g, loss, float(len(y)), float(np.sum(p * (1 - p)))


def full_objective(chunks, w, C=1.0):
    g = np.zeros(32)
    loss = 0.0
    S = 0.0
    for Rb in chunks:
        gg, ll, ss, _ = sums(Rb, w)
        g += gg
        loss += ll
        S += ss
    grad = g / S
    grad[:30] += w[:30] / (C * S)
    grad[31] = 0.0
    return loss / S + 0.5 * float(w[:30] @ w[:30]) / (C * S), float(np.abs(grad).max())


def newton(chunks, C=1.0, iters=12):
    w = np.zeros(32)
    for _ in range(iters):
        g = np.zeros(32)
        H = np.zeros((32, 32))
        S = 0.0
        for Rb in chunks:
            X = Rb.copy()
            y = X[:, 31].copy()
            X[:, 31] = 0.0
            p = 1.0 / (1.0 + np.exp(-(X @ w)))
            g += X.T @ (p - y)
            H += (X * (p * (1 - p))[:, None]).T @ X
            S += len(y)
        idx = list(range(31))
        gr = g[idx] / S
        gr[:30] += w[:30] / (C * S)
        A = H[np.ix_(idx, idx)] / S
        A[np.arange(30), np.arange(30)] += 1.0 / (C * S)
        w[idx] -= np.linalg.solve(A, gr)
    return w


def run_schedule(chunks, nb, epochs, mom=0.55, C=1.0, avg_from=None, tol=1e-3):
    """epochs: list of (c, s).  avg_from: epochs >= avg_from are Polyak-averaged (each returns its
    own average) and the fit stops at the first converged epoch end (ops/logreg.sgd_fit with
    extra_epochs); None: only the last epoch is averaged and every epoch runs."""
    st = ref.SgdStateRef(np.zeros(32))
    streamed = 0.0
    for ei, spec in enumerate(epochs):
        c, s = spec[0], spec[1]
        nbe = spec[2] if len(spec) > 2 else nb  # per-epoch minibatch count (optional)
        if avg_from is not None and st.done:
            break
        last_epoch = (ei == len(epochs) - 1) if avg_from is None else ei >= avg_from
        for b in range(nbe):
            fine = [ch for ch in range(FINE) if ch % (nbe * s) == b * s] if s > 1 else \
                   [ch for ch in range(FINE) if ch % nbe == b]
            g = np.zeros(32)
            loss = S = dsum = 0.0
            for ch in fine:
                gg, ll, ss, dd = sums(chunks[ch], st.w)
                g += gg
                loss += ll
                S += ss
                dsum += dd
            streamed += len(fine) / FINE
            red = np.concatenate([g, [loss, S, 0.0, dsum]])
            st.step(red[:32], red[32], red[33], red[35], 30, C, c, mom, nbe * s, last_epoch, b == nbe - 1,
                    -1.0 if s > 1 else (tol if avg_from is not None else 1e-3), True)
    w = st.w.copy()
    w[31] = 0.0
    return w, st.gmax, streamed


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8_000_000)
    ap.add_argument("--json", default="")
    ap.add_argument("--seed", type=int, default=1000)
    a = ap.parse_args()
    t0 = time.time()
    chunks = build(a.rows, a.seed)
    print(f"built {sum(len(c) for c in chunks)} rows in {time.time() - t0:.0f}s", flush=True)
    wn = newton(chunks)
    on, gn = full_objective(chunks, wn)
    print(f"newton objective {on:.9f} grad {gn:.2e}", flush=True)
    # (nb, epochs[, avg_from]): with avg_from the fit stops at its first converged epoch end
    scheds = {
        "sub4_c_x1": (8, [(0.4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 2),
        "sub4_c_x1lo": (8, [(0.4, 4), (0.7, 1), (0.8, 1), (0.4, 1)], 2),
        "sub4_lo3": (8, [(0.4, 4), (0.7, 1), (0.4, 1), (0.4, 1)], 2),
        "sub4_lo3b": (8, [(0.4, 4), (0.8, 1), (0.5, 1), (0.3, 1)], 2),
        "sub4_avg2": (8, [(0.4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "full_lo3": (8, [(0.4, 1), (0.7, 1), (0.4, 1), (0.4, 1)], 2),
        "sub4_avg1_b": (8, [(0.4, 4), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "sub4_avg1_c": (8, [(0.5, 4), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "sub4_avg1_d": (8, [(0.4, 4), (0.6, 1), (0.6, 1), (0.6, 1)], 1),
        "sub4_avg1_e": (8, [(0.4, 4), (0.7, 1), (0.6, 1), (0.5, 1)], 1),
        "sub4_avg1_f": (8, [(0.4, 4), (0.9, 1), (0.8, 1), (0.7, 1)], 1),
        "sub4_avg1_m45": (8, [(0.4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1, 0.45),
        "sub4_avg1_m65": (8, [(0.4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1, 0.65),
        "sub4_avg1_m75": (8, [(0.4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1, 0.75),
        "sub4_avg1_g": (8, [(0.4, 4), (0.7, 1), (0.9, 1), (0.9, 1)], 1),
        "sub4_avg1_h": (8, [(0.3, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub2_avg1": (8, [(0.4, 2), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "nb6_avg1": (6, [(0.4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "nb4_avg1": (4, [(0.4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub4nb4_avg1": (8, [(0.4, 4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub4nb4_avg1_b": (8, [(0.5, 4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub4nb4_avg1_c": (8, [(0.6, 4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub8nb4_avg1": (8, [(0.5, 8, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub8nb4_avg1_b": (8, [(0.4, 8, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub8nb4_avg1_c": (8, [(0.6, 8, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "full6_avg1": (8, [(0.4, 4), (0.7, 1, 6), (0.8, 1, 6), (0.8, 1, 6)], 1),
        "full6_avg1_b": (8, [(0.4, 4), (0.8, 1, 6), (0.9, 1, 6), (0.9, 1, 6)], 1),
        "full6_avg1_c": (8, [(0.4, 4), (0.6, 1, 6), (0.7, 1, 6), (0.7, 1, 6)], 1),
        "full4_avg1": (8, [(0.4, 4), (0.7, 1, 4), (0.8, 1, 4), (0.8, 1, 4)], 1),
        "full4_avg1_b": (8, [(0.4, 4), (0.9, 1, 4), (1.0, 1, 4), (1.0, 1, 4)], 1),
        "sub6_full6": (8, [(0.4, 4, 6), (0.7, 1, 6), (0.8, 1, 6), (0.8, 1, 6)], 1),
        "full8_6": (8, [(0.4, 4), (0.7, 1), (0.8, 1, 6), (0.8, 1, 6)], 1),
        "s4n4_a": (8, [(0.5, 4, 4), (0.6, 1), (0.8, 1), (0.8, 1)], 1),
        "s4n4_b": (8, [(0.6, 4, 4), (0.6, 1), (0.8, 1), (0.8, 1)], 1),
        "s4n4_c": (8, [(0.7, 4, 4), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "s4n4_d": (8, [(0.6, 4, 4), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "s4n4_e": (8, [(0.6, 4, 4), (0.7, 1), (0.7, 1), (0.7, 1)], 1),
        "s4n4_f": (8, [(0.6, 4, 4), (0.7, 1), (0.9, 1), (0.9, 1)], 1),
        "s4n6_a": (8, [(0.5, 4, 6), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "s4n6_b": (8, [(0.4, 4, 6), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "d86": (8, [(0.6, 4, 4), (0.8, 1, 8), (0.8, 1, 6), (0.8, 1, 6)], 1),
        "d66": (8, [(0.6, 4, 4), (0.8, 1, 6), (0.8, 1, 6), (0.8, 1, 6)], 1),
        # round 6: the same 16 steps with a smaller last-epoch step (iterate noise at <= 0.8x rows)
        "d66lo": (8, [(0.6, 4, 4), (0.8, 1, 6), (0.5, 1, 6), (0.5, 1, 6)], 1),
        "d66lo6": (8, [(0.6, 4, 4), (0.8, 1, 6), (0.6, 1, 6), (0.6, 1, 6)], 1),
        "d66lo4": (8, [(0.6, 4, 4), (0.8, 1, 6), (0.4, 1, 6), (0.4, 1, 6)], 1),
        "d76lo": (8, [(0.6, 4, 4), (0.7, 1, 6), (0.5, 1, 6), (0.5, 1, 6)], 1),
        "d96lo": (8, [(0.6, 4, 4), (0.9, 1, 6), (0.5, 1, 6), (0.5, 1, 6)], 1),
        "d3": (8, [(0.6, 4, 3), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "d2": (8, [(0.7, 4, 2), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "d48": (8, [(0.6, 8, 4), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "d816": (8, [(0.6, 16, 4), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "sub8_avg1": (8, [(0.4, 8), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub8_avg1_b": (8, [(0.5, 8), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "sub4x2_avg2": (8, [(0.4, 4), (0.5, 2), (0.8, 1), (0.8, 1)], 2),
        "nb4_avg1_b": (4, [(0.4, 8), (0.7, 1), (0.8, 1), (0.8, 1)], 1),
        "nb6_avg1_b": (6, [(0.5, 4), (0.8, 1), (0.8, 1), (0.8, 1)], 1),
        "nb4_avg1_c": (4, [(0.5, 4), (0.8, 1), (0.9, 1), (0.9, 1)], 1),
        "sub8_8x3": (8, [(0.4, 8), (0.6, 1), (0.8, 1)]),
        "sub4_8x3_b": (8, [(0.5, 4), (0.6, 1), (0.8, 1)]),
        "sub4_8x3_c": (8, [(0.4, 4), (0.7, 1), (0.8, 1)]),
        "sub4_8x2p5": (8, [(0.4, 4), (0.6, 2), (0.8, 1)]),
        "sub4_8x2_d": (8, [(0.4, 4), (0.7, 1)]),
        "cur_8x3": (8, [(0.4, 1), (0.6, 1), (0.8, 1)]),
        "8x2_a": (8, [(0.5, 1), (0.8, 1)]),
        "8x2_b": (8, [(0.6, 1), (0.9, 1)]),
        "sub4_8x3": (8, [(0.4, 4), (0.6, 1), (0.8, 1)]),
        "sub2_8x3": (8, [(0.4, 2), (0.6, 1), (0.8, 1)]),
        "sub4_sub2_full": (8, [(0.4, 4), (0.6, 2), (0.8, 1)]),
        "4x3": (4, [(0.4, 1), (0.6, 1), (0.8, 1)]),
    }
    out = {"newton_objective": on}
    only = os.environ.get("LAB_ONLY", "")
    for name, spec in scheds.items():
        nb, ep = spec[0], spec[1]
        avg_from = spec[2] if len(spec) > 2 else None
        mom = spec[3] if len(spec) > 3 else 0.55
        if only and name not in only.split(","):
            continue
        if nb * max(e[1] for e in ep) > FINE:
            continue
        t1 = time.time()
        w, gmax, streamed = run_schedule(chunks, nb, ep, mom=mom, avg_from=avg_from)
        o, gfull = full_objective(chunks, w)
        gap = (o - on) / on
        out[name] = {"nb": nb, "epochs": ep, "steps": sum(e[2] if len(e) > 2 else nb for e in ep), "epoch_gmax": gmax, "full_grad": gfull,
                     "gap": gap, "epochs_streamed": streamed}
        print(f"{name:16s} steps {out[name]['steps']:3d} streamed {streamed:.2f} ep_gmax {gmax:.2e} "
              f"full_grad {gfull:.2e} gap {gap:.2e} ({time.time() - t1:.0f}s)", flush=True)
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
