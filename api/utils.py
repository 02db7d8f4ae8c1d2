"""Model loader (reference contract: api/utils.py:10-25).

``load_model_and_features(model_path=None, features_path=None) -> (LogisticRegression, [names])``
with the reference's env defaults (MODEL_PATH, FEATURE_NAMES_PATH) and FileNotFoundError when the
model is absent.  The model object is rebuilt from the decoded artifact
(fraud_detection_amd.compat.sklearn_export): pickles this framework did not write are decoded
without executing them.
"""
import json
import logging
import os

from fraud_detection_amd.compat.sklearn_export import load_artifacts, make_logistic

log = logging.getLogger(__name__)
_DEFAULTS = {"MODEL_PATH": "./models/logistic_model.joblib",
             "FEATURE_NAMES_PATH": "./models/feature_names.json"}


def _resolve(explicit, env):
    return explicit or os.getenv(env, _DEFAULTS[env])


def load_model_and_features(model_path=None, features_path=None):
    mpath = _resolve(model_path, "MODEL_PATH")
    fpath = _resolve(features_path, "FEATURE_NAMES_PATH")
    if not os.path.isfile(mpath):
        log.error("Model file not found: %s", mpath)
        raise FileNotFoundError(f"Model not found at {mpath}")
    have_names = os.path.isfile(fpath)
    art = load_artifacts(mpath, os.path.join(os.path.dirname(mpath), "scaler.joblib"),
                         fpath if have_names else None)
    names = json.load(open(fpath, encoding="utf-8")) if have_names else []
    return make_logistic(art.coef, art.intercept, art.n_iter, art.C), names
