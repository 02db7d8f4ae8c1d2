"""Model-directory builders shared by the serving / XAI tests: the reference's shipped linear
artifacts plus a KernelSHAP background, and a small GBDT registered under the MLflow alias (the
layouts train.py writes)."""
import os
import shutil

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kaggle_like_rows(n: int, seed: int = 0) -> np.ndarray:
    """Raw rows in the shipped scaler's range (Time, V1..V28, Amount)."""
    rng = np.random.default_rng(seed)
    X = rng.normal(0, 1.2, size=(n, 30)).astype(np.float32)
    X[:, 0] = rng.uniform(0, 172_800, n)
    X[:, 29] = np.exp(rng.normal(3, 1, n))
    return X


def linear_dir_with_background(tmp_path, n_bg: int = 100) -> str:
    """Copy of models/ (the reference's LR + scaler) with a shap_background.npy."""
    from fraud_detection_amd.serve.engine import save_background

    d = os.path.join(str(tmp_path), "models_bg")
    shutil.copytree(os.path.join(ROOT, "models"), d, dirs_exist_ok=True)
    save_background(kaggle_like_rows(n_bg, seed=1), d)
    return d


def gbdt_registered(tmp_path, trees: int = 12, depth: int = 5, n: int = 6000):
    """Train a small GBDT on synthetic credit-card rows, save it with a background, log it to a
    file MLflow store and point the 'production' alias at it.  Returns (settings kwargs, result)."""
    from fraud_detection_amd.compat import mlflow_compat as mlf
    from fraud_detection_amd.data.synthetic import separable
    from fraud_detection_amd.models.gbdt import GBDTPipeline
    from fraud_detection_amd.models.pipeline import TrainConfig
    from fraud_detection_amd.ops import gbdt as gb
    from fraud_detection_amd.serve.engine import sample_background, save_background

    X, y = separable(n, fraud_rate=0.05, seed=21)
    res = GBDTPipeline(TrainConfig(), params=gb.GBDTParams(n_estimators=trees, max_depth=depth)).fit(X, y)
    mdir = os.path.join(str(tmp_path), "gbdt_model")
    names = ["Time"] + [f"V{i}" for i in range(1, 29)] + ["Amount"]
    paths = res.save(mdir, names)
    paths["background"] = save_background(sample_background(X.numpy(), 64), mdir)
    uri = f"file:{tmp_path}/mlruns_gbdt"
    mlf.set_tracking_uri(uri)
    mlf.set_experiment("gbdt-test")
    with mlf.start_run():
        muri = res.log_model(mlf, paths)
    v = mlf.register_model(muri, "fraud-detection-model")
    mlf.set_registered_model_alias("fraud-detection-model", "production", v)
    return {"mlflow_tracking_uri": uri}, res, X


def torch_rows(X) -> torch.Tensor:
    return torch.from_numpy(np.ascontiguousarray(X, dtype=np.float32))
