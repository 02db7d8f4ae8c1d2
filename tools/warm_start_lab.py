#!/usr/bin/env python3
"""fp64 CPU lab: does a warm start from the REAL rows (positives weighted to the post-SMOTE class
mass) save the Newton warm-up?  Builds the bench distribution (tools/sgd_schedule_lab.build), runs
the device's progressive warm-up schedule [(16, 3), (8, 1), (4, 1)] on the post-SMOTE rows, and
weighted Newton on real-row subsets, then counts the full-data Newton steps each start needs to reach
a gradient max-norm of 1e-8.  Round 5 (8M raw rows): progressive 3 steps, every real-row start 4.

    python tools/warm_start_lab.py [rows] [seed]
"""
import os, sys
import numpy as np
_R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, _R); sys.path.insert(0, os.path.join(_R, 'tools'))
import sgd_schedule_lab as L
from fraud_detection_amd.data.synthetic import separable
rows = int(sys.argv[1]); seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
chunks = L.build(rows, seed)
# real rows / synthetic rows split: synthetic rows have col 31 == 1 AND were appended after R rows in each chunk;
# rebuild real rows separately
X, y = separable(rows, seed=seed)
X = X.numpy().astype(np.float64); y = y.numpy().astype(np.float64)
mu, sd = X.mean(0), X.std(0)
R = np.zeros((len(y), 32)); R[:, :30] = (X - mu) / sd; R[:, 30] = 1.0; R[:, 31] = y
npos = y.sum(); ntot = sum(len(c) for c in chunks); wpos = (ntot - (len(y) - npos)) / npos
print("n_real", len(y), "pos", int(npos), "post-smote", ntot, "wpos", round(wpos, 1))

def grad_hess(Rb, w, wp=1.0):
    Xb = Rb.copy(); yb = Xb[:, 31].copy(); Xb[:, 31] = 0.0
    s = np.where(yb > 0.5, wp, 1.0)
    p = 1 / (1 + np.exp(-(Xb @ w)))
    return Xb.T @ ((p - yb) * s), (Xb * (s * p * (1 - p))[:, None]).T @ Xb, s.sum()

def newton_step(parts, w, C=1.0, wp=1.0):
    g = np.zeros(32); H = np.zeros((32, 32)); S = 0.0
    for Rb in parts:
        gg, hh, ss = grad_hess(Rb, w, wp); g += gg; H += hh; S += ss
    idx = list(range(31)); gr = g[idx] / S; gr[:30] += w[:30] / (C * S)
    A = H[np.ix_(idx, idx)] / S; A[np.arange(30), np.arange(30)] += 1 / (C * S)
    w = w.copy(); w[idx] -= np.linalg.solve(A, gr); return w, np.abs(gr).max()

def full_iters(w, tol=1e-8, maxit=10):
    for it in range(maxit):
        w2, gm = newton_step(chunks, w)
        if gm < tol: return it, gm
        w = w2
    return maxit, gm

# progressive: (16,3),(8,1),(4,1) on post-smote chunks (FINE=64 partition: 1/16 = every 16th chunk... use chunk subsets)
w = np.zeros(32)
for sub, its in [(16, 3), (8, 1), (4, 1)]:
    part = [chunks[c] for c in range(0, L.FINE, sub)]
    for _ in range(its): w, _ = newton_step(part, w)
print("progressive: full iters to 1e-8 =", full_iters(w))
rng = np.random.default_rng(0)
for sub_sched in ([(4, 3)], [(2, 3)], [(1, 4)], [(16, 3), (8, 1), (4, 1)]):
    w = np.zeros(32)
    for sub, its in sub_sched:
        sel = (np.arange(len(y)) // 64) % sub == 0
        part = [R[sel]]
        for _ in range(its): w, _ = newton_step(part, w, wp=wpos)
    print("real-row weighted", sub_sched, "-> full iters", full_iters(w))
