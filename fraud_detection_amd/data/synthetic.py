"""Credit-card-shaped synthetic data (Kaggle creditcard schema: Time, V1..V28, Amount, Class).

Two generators:

* ``reference_frame`` reproduces scripts/generate_synthetic_data.py:6-27 of the reference
  exactly (same numpy RandomState(42) draw sequence): Time ~ U(0, 172800) sorted, V ~ N(0, 1),
  Amount = exp(N(3, 1)), and labels chosen at random (1%), i.e. INDEPENDENT of the features, so
  any model scores AUC ~ 0.5 on it.  Kept for contract parity (CI).
* ``separable`` is the benchmark distribution: legit V ~ N(0, I), fraud V ~
  N(delta * u, I) for a fixed unit direction u, so the Bayes AUC is Phi(delta / sqrt(2))
  (0.970 at delta = 2.66, matching the reference's published 0.9710).  Generated directly on the
  target device with torch's counter-based generator; rows are row-major fp32 [n, 30].
"""
from __future__ import annotations

import math

import numpy as np
import pandas as pd
import torch

FEATURES = ["Time"] + [f"V{i}" for i in range(1, 29)] + ["Amount"]
COLUMNS = FEATURES + ["Class"]
DEFAULT_FRAUD_RATE = 0.0017   # Kaggle creditcard: 492 / 284,807
DEFAULT_DELTA = 2.66          # Mahalanobis separation -> Bayes AUC ~ 0.970


def reference_frame(n_samples: int = 1000, n_features: int = 30, fraud_ratio: float = 0.01,
                    seed: int = 42) -> pd.DataFrame:
    rs = np.random.RandomState(seed)
    v = rs.randn(n_samples, n_features - 2)
    t = np.sort(rs.uniform(0, 172800, n_samples))
    amount = np.exp(rs.normal(3, 1, n_samples))
    y = np.zeros(n_samples)
    y[rs.choice(n_samples, int(n_samples * fraud_ratio), replace=False)] = 1
    data = np.column_stack([t, v, amount, y])
    return pd.DataFrame(data, columns=COLUMNS[: n_features] + ["Class"] if n_features == 30 else
                        ["Time"] + [f"V{i}" for i in range(1, n_features - 1)] + ["Amount", "Class"])


def fraud_direction(n_v: int = 28) -> np.ndarray:
    """Fixed unit direction of the fraud shift, loosely shaped like the Kaggle signal
    (strong on V14/V17/V12/V10 negative, V4/V11 positive), deterministic."""
    u = np.zeros(n_v)
    pattern = {14: -1.0, 17: -0.9, 12: -0.85, 10: -0.8, 16: -0.6, 3: -0.55, 7: -0.5, 4: 0.75,
               11: 0.6, 2: 0.4, 9: -0.45, 18: -0.35, 1: -0.3, 5: -0.25, 6: -0.2, 21: 0.2}
    for k, v in pattern.items():
        if k <= n_v:
            u[k - 1] = v
    return u / np.linalg.norm(u)


def bayes_auc(delta: float = DEFAULT_DELTA) -> float:
    return 0.5 * (1.0 + math.erf(delta / 2.0))  # Phi(delta / sqrt(2))


def separable(n: int, fraud_rate: float = DEFAULT_FRAUD_RATE, delta: float = DEFAULT_DELTA, seed: int = 0,
              device="cpu", n_features: int = 30, exact_count: bool = True):
    """Return (X fp32 [n, n_features], y uint8 [n]) on ``device``."""
    dev = torch.device(device)
    g = torch.Generator(device=dev)
    g.manual_seed(int(seed))
    n_v = n_features - 2
    X = torch.empty((n, n_features), device=dev, dtype=torch.float32)
    X[:, 1:1 + n_v] = torch.randn((n, n_v), device=dev, generator=g)
    t = torch.rand(n, device=dev, generator=g) * 172800.0
    X[:, 0] = torch.sort(t).values
    X[:, n_features - 1] = torch.exp(torch.randn(n, device=dev, generator=g) + 3.0)
    if exact_count:
        n_fraud = int(round(n * fraud_rate))
        perm = torch.randperm(n, device=dev, generator=g)[:n_fraud]
        y = torch.zeros(n, device=dev, dtype=torch.uint8)
        y[perm] = 1
    else:
        y = (torch.rand(n, device=dev, generator=g) < fraud_rate).to(torch.uint8)
    u = torch.from_numpy(fraud_direction(n_v) * delta).to(dev, torch.float32)
    X[:, 1:1 + n_v] += y.to(torch.float32)[:, None] * u[None, :]
    return X, y


def separable_frame(n: int, fraud_rate: float = DEFAULT_FRAUD_RATE, delta: float = DEFAULT_DELTA,
                    seed: int = 0) -> pd.DataFrame:
    X, y = separable(n, fraud_rate, delta, seed, "cpu")
    df = pd.DataFrame(X.numpy().astype(np.float64), columns=FEATURES)
    df["Class"] = y.numpy().astype(np.float64)
    return df
