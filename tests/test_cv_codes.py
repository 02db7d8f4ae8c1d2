"""Fold-code plumbing of the device CV jobs (models/cv.py): sklearn StratifiedKFold splits ->
per-row codes, and the checks on caller-supplied codes (CPU)."""
import numpy as np
import pytest
import torch

from fraud_detection_amd.models.cv import fold_codes_from_splits, resolve_fold_codes


def test_codes_from_sklearn_splits():
    from sklearn.model_selection import StratifiedKFold

    rng = np.random.default_rng(0)
    y = (rng.random(5000) < 0.05).astype(np.uint8)
    sk = list(StratifiedKFold(n_splits=5, shuffle=True, random_state=42).split(np.zeros(len(y)), y))
    c = fold_codes_from_splits(sk, len(y))
    assert c.dtype == np.uint8 and set(np.unique(c)) == set(range(5))
    for k, (tr, va) in enumerate(sk):
        assert np.array_equal(np.nonzero(c == k)[0], np.sort(va))
        assert np.array_equal(np.nonzero(c != k)[0], np.sort(tr))


def test_codes_checked():
    y = torch.zeros(10, dtype=torch.uint8)
    with pytest.raises(ValueError):
        fold_codes_from_splits([(np.arange(5, 10), np.arange(5))], 10)  # rows 5..9 validate nowhere
    with pytest.raises(ValueError):
        resolve_fold_codes(y, 5, 42, np.zeros(9, np.uint8))
    with pytest.raises(ValueError):
        resolve_fold_codes(y, 5, 42, np.full(10, 5, np.uint8))
    c = resolve_fold_codes(y, 5, 42, np.arange(10) % 5)
    assert c.dtype == torch.uint8 and c.tolist() == [0, 1, 2, 3, 4] * 2
    assert resolve_fold_codes(y, 5, 42).shape == (10,)  # the Feistel codes
