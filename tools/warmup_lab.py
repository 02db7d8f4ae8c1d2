#!/usr/bin/env python3
"""CPU (fp64) lab: can the Newton warm-up run on the REAL rows only, concurrently with the k-NN and
the SMOTE bucket sort, without costing full-data iterations?

For the bench distribution (scaled down: --rows raw training rows, SMOTE to balance, k = 5) it
counts the full-data Newton iterations (lazy Hessian: fresh every 4th, as ops/logreg.newton_fit)
needed to reach max|grad| <= tol from the end point of each warm-up:
  A  today's warm-up: Newton steps on uniform sub-samples of the post-SMOTE rows (1/16 x3, 1/8, 1/4)
  B  the same schedule on the real rows only, positives weighted (n_min + n_new) / n_min
  C  B's exact fixed point (the best any real-rows-only warm-up can give)
  D  real rows + one midpoint row per (parent, neighbour) pick, weighted by its expected sample
     count (a mean-field SMOTE that needs the neighbour lists but not the bucket sort)

    python tools/warmup_lab.py [--rows 2000000] [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402


def sigmoid(z):
    return 0.5 * (1.0 + np.tanh(0.5 * z))


def grad_hess(X, y, sw, w, C, S_total, hess=True):
    """Mean objective over the weighted rows (weights sw), L2 on the feature columns (not the last)."""
    z = X @ w
    p = sigmoid(z)
    S = float(sw.sum())
    g = X.T @ (sw * (p - y)) / S
    reg = np.ones(X.shape[1]) / (C * S)
    reg[-1] = 0.0
    g = g + reg * w
    H = None
    if hess:
        d = sw * p * (1 - p)
        H = (X * d[:, None]).T @ X / S + np.diag(reg)
    return g, H


def newton_steps(X, y, sw, w, C, iters):
    for _ in range(iters):
        g, H = grad_hess(X, y, sw, w, C, None)
        w = w - np.linalg.solve(H, g)
    return w


def full_phase(X, y, sw, w, C, tol, refresh=4, max_iter=25):
    """Iterations (each one pass) until max|grad| <= tol at the start of an iteration."""
    H = None
    for it in range(max_iter):
        fresh = it % refresh == 0
        g, Hn = grad_hess(X, y, sw, w, C, None, hess=fresh)
        if fresh:
            H = Hn
        if np.abs(g).max() <= tol:
            return it + 1, w  # the checking pass counts (the device runs it)
        w = w - np.linalg.solve(H, g)
    return max_iter, w


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=2_000_000)
    ap.add_argument("--seeds", default="1000,1001")
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    from fraud_detection_amd.data.synthetic import separable

    out = {"rows": a.rows, "tol": a.tol, "runs": []}
    for seed in [int(s) for s in a.seeds.split(",")]:
        X, y = separable(a.rows, seed=seed)
        X = X.numpy().astype(np.float64)
        y = y.numpy().astype(np.float64)
        X = (X - X.mean(0)) / X.std(0)
        R = np.concatenate([X, np.ones((len(X), 1))], 1)
        mins = np.nonzero(y > 0.5)[0]
        M = R[mins]
        k = 5
        F = M[:, :-1]
        sq = (F * F).sum(1)
        d2 = sq[:, None] + sq[None, :] - 2.0 * F @ F.T
        np.fill_diagonal(d2, np.inf)
        nbr = np.argsort(d2, 1)[:, :k]
        n_min = len(mins)
        n_new = (len(R) - n_min) - n_min
        rng = np.random.default_rng(seed)
        picks = rng.integers(0, n_min * k, n_new)
        lam = rng.random(n_new)
        A_ = M[picks // k]
        S = A_ + lam[:, None] * (M[nbr.reshape(-1)[picks]] - A_)
        XF = np.concatenate([R, S])
        yF = np.concatenate([y, np.ones(n_new)])
        swF = np.ones(len(XF))
        C = 1.0
        w0 = np.zeros(R.shape[1])
        sched = [(16, 3), (8, 1), (4, 1)]

        def warm(Xw, yw, sww):
            w = w0.copy()
            r = np.random.default_rng(7)
            for sub, iters in sched:
                idx = r.permutation(len(Xw))[: len(Xw) // sub]
                w = newton_steps(Xw[idx], yw[idx], sww[idx], w, C, iters)
            return w

        wA = warm(XF, yF, swF)
        om = (n_min + n_new) / n_min
        swB = np.where(y > 0.5, om, 1.0)
        wB = warm(R, y, swB)
        wC = newton_steps(R, y, swB, w0.copy(), C, 12)
        mid = 0.5 * (M[np.repeat(np.arange(n_min), k)] + M[nbr.reshape(-1)])
        XD = np.concatenate([R, mid])
        yD = np.concatenate([y, np.ones(len(mid))])
        swD = np.concatenate([np.ones(len(R)), np.full(len(mid), n_new / (n_min * k))])
        wD = warm(XD, yD, swD)
        wstar = newton_steps(XF, yF, swF, w0.copy(), C, 12)
        run = {"seed": seed, "n_min": int(n_min), "n_new": int(n_new)}
        for name, w in (("A_today", wA), ("B_real_weighted", wB), ("C_real_weighted_opt", wC),
                        ("D_real_plus_midpoints", wD)):
            it, _ = full_phase(XF, yF, swF, w, C, a.tol)
            g, _ = grad_hess(XF, yF, swF, w, C, None, hess=False)
            run[name] = {"full_iters": it, "start_gmax": float(np.abs(g).max()),
                         "dist_to_opt": float(np.abs(w - wstar).max())}
        print(json.dumps(run), flush=True)
        out["runs"].append(run)
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
