"""Reference entry scripts run end to end on a small preprocessed set (evaluate_model.py,
explain_model.py incl. the rank-sharded KernelSHAP under a 2-rank gloo job)."""
import os
import shutil
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture()
def workdir(tmp_path):
    shutil.copytree(os.path.join(ROOT, "models"), tmp_path / "models")
    os.makedirs(tmp_path / "data")
    rng = np.random.default_rng(0)
    X = rng.normal(0, 1, (3000, 30)).astype(np.float32)
    w = np.r_[rng.normal(0, 1, 30)]
    y = (X @ w + rng.normal(0, 1, 3000) > 2.5).astype(np.int64)
    np.savez_compressed(tmp_path / "data" / "preprocessed_data.npz", X_res=X, y_res=y, X_test=X, y_test=y)
    return tmp_path


def _run(args, cwd, env=None):
    e = dict(os.environ, PYTHONPATH=ROOT, MPLBACKEND="Agg", FDX_DEVICE="cpu", **(env or {}))
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=e, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return r.stdout


def test_evaluate_model_script(workdir):
    out = _run([os.path.join(ROOT, "evaluate_model.py")], workdir)
    assert "Confusion Matrix" in out and "AUC" in out
    assert (workdir / "plots" / "roc_curve.png").exists() and (workdir / "plots" / "confusion_matrix.png").exists()


def test_explain_model_kernel_sharded_over_two_ranks(workdir):
    _run([os.path.join(ROOT, "explain_model.py"), "--kernel", "--rows", "64"], workdir)
    single = np.load(workdir / "plots" / "kernelshap_values.npy")
    os.remove(workdir / "plots" / "kernelshap_values.npy")
    port = str(29500 + os.getpid() % 1000)
    _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr=127.0.0.1",
          f"--master-port={port}", os.path.join(ROOT, "explain_model.py"), "--kernel", "--rows", "64"], workdir)
    dp = np.load(workdir / "plots" / "kernelshap_values.npy")
    assert dp.shape == single.shape == (64, 30)
    np.testing.assert_allclose(dp, single, atol=1e-12)


def test_eda_script_on_generated_csv(tmp_path):
    """scripts/generate_synthetic_data.py -> eda.py: both plots and processed_data.csv (the
    2-column Amount/Time frame converts column-major; the scaler needs row-major rows)."""
    _run([os.path.join(ROOT, "scripts", "generate_synthetic_data.py"), "--separable", "--rows", "5000"], tmp_path)
    _run([os.path.join(ROOT, "eda.py")], tmp_path)
    assert (tmp_path / "plots" / "class_distribution.png").exists()
    assert (tmp_path / "plots" / "amount_distribution.png").exists()
    import pandas as pd

    df = pd.read_csv(tmp_path / "processed_data.csv")
    assert {"scaled_amount", "scaled_time", "Class"} <= set(df.columns)
    assert abs(df["scaled_amount"].mean()) < 1e-3 and abs(df["scaled_amount"].std(ddof=0) - 1) < 1e-3


def test_explain_model_tree_shap_of_a_gbdt(workdir):
    """explain_model.py --tree: interventional TreeSHAP of models/xgb_model.json on the test rows."""
    import json

    from test_treeshap import random_ensemble

    ens = random_ensemble(30, 4, 12, 5)
    with open(workdir / "models" / "xgb_model.json", "w") as f:
        json.dump(ens.to_dict(), f)
    out = _run([os.path.join(ROOT, "explain_model.py"), "--tree", "--rows", "50"], workdir)
    assert "treeshap_rows" in out
    phi = np.load(workdir / "plots" / "treeshap_values.npy")
    assert phi.shape == (50, 30) and (workdir / "plots" / "treeshap_summary.png").exists()
