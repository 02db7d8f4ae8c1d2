"""Dataset I/O for the creditcard schema (reference: train_model.py:22-29, preprocess.py:21-29,
load_data.py:4-15).  CSV parsing runs in the native reader (csrc/io/csv_reader.cpp: mmap +
threads + from_chars) with a pandas fallback; splits are stratified exactly like the reference's
sklearn calls (test_size=0.2, random_state=42; StratifiedKFold(5, shuffle=True, 42))."""
from __future__ import annotations

import importlib

import numpy as np

from .synthetic import FEATURES


def read_table(path: str, label: str = "Class"):
    """-> (X float32 [n, d], y uint8 [n] or None, feature_names)."""
    try:
        io = importlib.import_module("fraud_detection_amd._fdx_io")
        arr, header = io.read_csv(path)
        header = [h.strip() for h in header]
    except ImportError:
        import pandas as pd

        df = pd.read_csv(path)
        arr, header = df.to_numpy(dtype=np.float32), list(df.columns)
    if label in header:
        j = header.index(label)
        y = arr[:, j]
        if np.isnan(y).any():
            raise ValueError(f"missing values in label column {label!r}")
        X = np.ascontiguousarray(np.delete(arr, j, axis=1))
        names = [h for h in header if h != label]
        return X, y.astype(np.uint8), names
    return np.ascontiguousarray(arr), None, header


def missing_report(X: np.ndarray, names) -> dict:
    return {n: int(c) for n, c in zip(names, np.isnan(X).sum(0))}


def stratified_split(y: np.ndarray, test_size: float = 0.2, seed: int = 42):
    """Indices (train, test), identical to sklearn.model_selection.train_test_split(stratify=y)."""
    from sklearn.model_selection import train_test_split

    idx = np.arange(len(y))
    tr, te = train_test_split(idx, test_size=test_size, random_state=seed, stratify=y)
    return tr, te


def stratified_folds(y: np.ndarray, n_splits: int = 5, seed: int = 42):
    from sklearn.model_selection import StratifiedKFold

    return list(StratifiedKFold(n_splits=n_splits, shuffle=True, random_state=seed).split(np.zeros(len(y)), y))


__all__ = ["read_table", "stratified_split", "stratified_folds", "missing_report", "FEATURES"]
