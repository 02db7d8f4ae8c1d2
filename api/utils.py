"""Model loader utility (reference: api/utils.py:10-25)."""
import json
import logging
import os

from fraud_detection_amd.compat.sklearn_export import load_artifacts, make_logistic

logger = logging.getLogger(__name__)


def load_model_and_features(model_path: str | None = None, features_path: str | None = None):
    """Return (sklearn LogisticRegression, feature_names).  Files written by this framework are
    loaded with joblib; foreign pickles only through the non-executing decoder."""
    model_path = model_path or os.getenv("MODEL_PATH", "./models/logistic_model.joblib")
    features_path = features_path or os.getenv("FEATURE_NAMES_PATH", "./models/feature_names.json")
    if not os.path.exists(model_path):
        logger.error("Model file not found: %s", model_path)
        raise FileNotFoundError(f"Model not found at {model_path}")
    scaler_path = os.path.join(os.path.dirname(model_path), "scaler.joblib")
    art = load_artifacts(model_path, scaler_path, features_path if os.path.exists(features_path) else None)
    model = make_logistic(art.coef, art.intercept, art.n_iter, art.C)
    feature_names = []
    if os.path.exists(features_path):
        with open(features_path, "r", encoding="utf-8") as f:
            feature_names = json.load(f)
    return model, feature_names
