"""K3 stratified split oracle (ops/split.py): per-class test share, fold balance, permutation."""
import numpy as np
import pytest

from fraud_detection_amd.ops import split as SP


@pytest.mark.parametrize("n,rate,k", [(1000, 0.01, 5), (12345, 0.2, 5), (77, 0.5, 3), (5000, 0.002, 1)])
def test_codes_stratified_and_balanced(n, rate, k):
    rng = np.random.default_rng(n)
    y = (rng.random(n) < rate).astype(np.uint8)
    c = SP.assign_numpy(y, 0.2, k, 42)
    for cls in (0, 1):
        cc = c[y == cls]
        n_c = cc.shape[0]
        ntest = min(int(np.floor(0.2 * n_c + 0.5)), n_c)
        assert int((cc == SP.TEST).sum()) == ntest
        tr = cc[cc != SP.TEST]
        if k > 1:
            sizes = np.bincount(tr, minlength=k)
            assert sizes.shape[0] == k and sizes.max() - sizes.min() <= 1 and sizes.sum() == n_c - ntest
        else:
            assert np.all(tr == 0)


def test_permutation_is_a_shuffle():
    n = 100_000
    y = np.zeros(n, np.uint8)
    c = SP.assign_numpy(y, 0.2, 5, 7)
    te = np.flatnonzero(c == SP.TEST)
    # a shuffled test set is spread over the table, not a prefix/suffix block
    assert te.shape[0] == 20_000
    hist = np.histogram(te, bins=10, range=(0, n))[0]
    assert hist.min() > 1700 and hist.max() < 2300
    # another seed gives another split
    c2 = SP.assign_numpy(y, 0.2, 5, 8)
    assert (c2 != c).mean() > 0.3


def test_cpu_tensor_path_and_indices():
    import torch

    y = torch.from_numpy((np.random.default_rng(3).random(5000) < 0.1).astype(np.uint8))
    c = SP.assign(y, 0.2, 5, 42)
    assert np.array_equal(c.numpy(), SP.assign_numpy(y.numpy(), 0.2, 5, 42))
    tr, te, folds = SP.split_indices(c, 5)
    assert tr.shape[0] + te.shape[0] == 5000
    assert len(folds) == 5
    allval = torch.cat([v for _, v in folds]).sort().values
    assert torch.equal(allval, tr)
    for ftr, fva in folds:
        assert ftr.shape[0] + fva.shape[0] == tr.shape[0]


def test_train_entry_point_device_split(tmp_path, monkeypatch):
    from fraud_detection_amd import train
    from fraud_detection_amd.config import Settings
    from fraud_detection_amd.data.synthetic import reference_frame

    df = reference_frame(6000, seed=6)
    csv = tmp_path / "cc.csv"
    df.to_csv(csv, index=False)
    monkeypatch.setenv("DATA_CSV", str(csv))
    monkeypatch.setenv("MLFLOW_TRACKING_URI", str(tmp_path / "mlruns"))
    monkeypatch.setenv("FDX_SPLIT", "device")
    out = train.run(Settings.load(), cv_folds=3, model_dir=str(tmp_path / "models"), verbose=False)
    assert out["split"] == "device" and len(out["cv_scores"]) == 3
    y = df["Class"].to_numpy().astype(np.uint8)
    codes = SP.assign_numpy(y, 0.2, 3, 42)
    ev = out["eval"]
    assert ev["tn"] + ev["fp"] + ev["fn"] + ev["tp"] == int((codes == SP.TEST).sum())  # the K3 test set
