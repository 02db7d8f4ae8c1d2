"""Checkpoint/resume: atomic safetensors files, keep-N rotation, signature
matching, and bit-identical resumed GBDT / SGD fits (CPU oracles; the device paths share the
resume logic and are covered in tests/test_gbdt_gpu.py)."""
import os

import numpy as np
import pytest
import torch

from fraud_detection_amd.ops import gbdt as gb
from fraud_detection_amd.ops import logreg as L
from fraud_detection_amd.ops import scaler as S
from fraud_detection_amd.utils.checkpoint import CheckpointManager, load_checkpoint, save_checkpoint


def test_roundtrip_and_rotation(tmp_path):
    p = save_checkpoint(str(tmp_path / "a.safetensors"), {"w": np.arange(4.0), "t": torch.ones(2, 3)}, {"step": 3})
    t, meta = load_checkpoint(p)
    assert meta == {"step": 3} and torch.equal(t["w"], torch.arange(4.0, dtype=torch.float64))
    mgr = CheckpointManager(str(tmp_path / "m"), keep=2)
    for step in range(1, 6):
        mgr.save(step, {"x": np.full(3, step)}, {"signature": "A" if step < 5 else "B"})
    files = sorted(os.listdir(tmp_path / "m"))
    assert files == ["ckpt-4.safetensors", "ckpt-5.safetensors"]
    assert mgr.latest("A")[1]["step"] == 4 and mgr.latest("B")[1]["step"] == 5
    assert mgr.latest("C") is None
    assert not [f for f in files if f.startswith(".ckpt_")]  # no temp files left behind


def test_non_lead_rank_does_not_write(tmp_path):
    mgr = CheckpointManager(str(tmp_path), rank=1)
    assert mgr.save(1, {"x": np.zeros(1)}, {}) is None and not os.listdir(tmp_path)


def _gbdt_data():
    rng = np.random.default_rng(3)
    X = rng.normal(size=(3000, 6)).astype(np.float32)
    y = (X[:, 0] - X[:, 1] ** 2 + rng.normal(size=3000) > 0.5).astype(np.uint8)
    return torch.from_numpy(X), torch.from_numpy(y)


def test_gbdt_resume_is_bit_identical(tmp_path):
    X, y = _gbdt_data()
    full = gb.fit(X, y, gb.GBDTParams(n_estimators=10, max_depth=3))
    mgr = CheckpointManager(str(tmp_path), prefix="gbdt")
    gb.fit(X, y, gb.GBDTParams(n_estimators=6, max_depth=3), checkpoint=mgr, checkpoint_every=2)  # "crash" at 6
    assert mgr.latest()[1]["trees_done"] == 6
    resumed = gb.fit(X, y, gb.GBDTParams(n_estimators=10, max_depth=3), checkpoint=mgr, checkpoint_every=2)
    for k in ("feat", "bin", "thr", "gain", "leaf"):
        assert np.array_equal(getattr(resumed, k), getattr(full, k)), k
    # a different config must not resume from these trees
    other = gb.fit(X, y, gb.GBDTParams(n_estimators=2, max_depth=3, learning_rate=0.3), checkpoint=mgr)
    assert not np.array_equal(other.leaf, full.leaf[:2])


def test_sgd_resume_is_bit_identical(tmp_path):
    from fraud_detection_amd.data.synthetic import separable

    X, y = separable(6000, fraud_rate=0.1, seed=4)
    rows = S.scale_cast(X, S.scaler_fit(X), labels=y)
    kw = dict(epochs=3, batches=6)
    full = L.sgd_fit(rows, **kw)
    mgr = CheckpointManager(str(tmp_path), prefix="sgd", keep=3)
    L.sgd_fit(rows, **kw, checkpoint=mgr, checkpoint_every=4, max_steps=12)  # "crash" after 2 epochs
    got = mgr.latest()
    assert got[1]["epoch"] == 2 and got[1]["batch"] == 0
    resumed = L.sgd_fit(rows, **kw, checkpoint=mgr, checkpoint_every=4)
    assert np.array_equal(resumed.w, full.w) and resumed.n_iter == full.n_iter
    # mid-epoch interruption (step 9 of 18: epoch 1, minibatch 3) resumes to the same model too
    mgr2 = CheckpointManager(str(tmp_path / "mid"), prefix="sgd", keep=3)
    L.sgd_fit(rows, **kw, checkpoint=mgr2, checkpoint_every=3, max_steps=9)
    assert mgr2.latest()[1]["epoch"] == 1 and mgr2.latest()[1]["batch"] == 3
    again = L.sgd_fit(rows, **kw, checkpoint=mgr2, checkpoint_every=3)
    assert np.array_equal(again.w, full.w)


def test_gbdt_resume_mid_epoch_checkpoint_every(tmp_path):
    X, y = _gbdt_data()
    mgr = CheckpointManager(str(tmp_path), prefix="g2", keep=1)
    gb.fit(X, y, gb.GBDTParams(n_estimators=5, max_depth=2), checkpoint=mgr, checkpoint_every=3)
    assert mgr.latest()[1]["trees_done"] == 5  # final round always saved
