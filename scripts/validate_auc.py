"""Model AUC gate (reference path scripts/validate_auc.py:1-40).

    python scripts/validate_auc.py [model_uri] [threshold]

Loads a registered model (``models:/<name>@<alias>``, ``models:/<name>/<version>`` or
``runs:/<id>/model``), scores it on credit_card-shaped synthetic data of the model's real width
(the reference used a 10-feature set against a 30-feature model), logs
metric ``auc_score`` and tag ``validation_pass`` to a tracking run, exits 0 if AUC >= threshold.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from fraud_detection_amd.compat import mlflow_compat as mlf  # noqa: E402
from fraud_detection_amd.compat.sklearn_export import load_artifacts  # noqa: E402
from fraud_detection_amd.data.synthetic import separable  # noqa: E402
from fraud_detection_amd.serve.engine import InferenceEngine  # noqa: E402


def load_synthetic_data(size=20000, seed=42):
    X, y = separable(size, fraud_rate=0.05, seed=seed)
    return X.numpy(), y.numpy()


def validate_auc(model_uri, threshold=0.95):
    from sklearn.metrics import roc_auc_score

    try:
        mlf.set_tracking_uri(os.getenv("MLFLOW_TRACKING_URI", "file:./mlruns"))
        mdir = mlf.resolve_model_dir(model_uri)
        art = load_artifacts(os.path.join(mdir, "model.pkl"), os.path.join(mdir, "scaler.joblib"),
                             os.path.join(mdir, "feature_names.json"), trusted=True)
        eng = InferenceEngine(art)
        X, y = load_synthetic_data()
        _, p = eng.predict(X)
        auc = float(roc_auc_score(y, p))
        mlf.set_experiment(os.getenv("MLFLOW_EXPERIMENT", "fraud-detection-ci"))
        with mlf.start_run():
            mlf.log_metric("auc_score", auc)
            mlf.set_tag("validation_pass", str(auc >= threshold))
        print("AUC validation complete: auc={}, threshold={}".format(auc, threshold))
        return [auc, bool(auc >= threshold)]
    except Exception as e:  # noqa: BLE001
        print("Error in validation: {}".format(e))
        return [0.0, False]


if __name__ == "__main__":
    uri = sys.argv[1] if len(sys.argv) > 1 else "models:/{}@{}".format(
        os.getenv("MLFLOW_MODEL_NAME", "fraud-detection-model"), os.getenv("MLFLOW_MODEL_STAGE", "production"))
    threshold = float(sys.argv[2]) if len(sys.argv) > 2 else 0.95
    auc, passed = validate_auc(uri, threshold)
    sys.exit(0 if passed else 1)
