"""Offline preprocessing (reference path preprocess.py:1-59).

Reads data/creditcard.csv, fits the StandardScaler on the TRAIN split only (the reference fit it
on the full data before splitting -- a leak), stratified 80/20 split
(random_state=42), SMOTE on the training rows (MFMA k-NN + Philox interpolation on MI355X), and
writes data/preprocessed_data.npz (X_res, y_res, X_test, y_test: scaled features) plus
models/scaler.joblib, models/columns.joblib, models/feature_names.json.
"""
import json
import os

import joblib
import numpy as np
import torch

from fraud_detection_amd.compat.sklearn_export import make_scaler
from fraud_detection_amd.data.io import read_table, stratified_split
from fraud_detection_amd.models.smote import SMOTE
from fraud_detection_amd.ops import scaler as S

DATA_PATH = os.getenv("DATA_CSV", "data/creditcard.csv")
PROCESSED_DATA_PATH = "data/preprocessed_data.npz"
MODELS_DIR = "models"


def main():
    os.makedirs(MODELS_DIR, exist_ok=True)
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    print("Loading dataset...")
    X, y, feature_names = read_table(DATA_PATH)
    print("Checking missing values:", int(np.isnan(X).sum()))
    print("Splitting dataset (Train 80% / Test 20%)...")
    tr, te = stratified_split(y, 0.2, 42)
    Xtr = torch.from_numpy(X[tr]).to(dev)
    print("Scaling features (fit on the training split)...")
    stats = S.scaler_fit(Xtr)
    mean, var, scale = stats.numpy()
    X_train = ((X[tr] - mean) / scale)
    X_test = ((X[te] - mean) / scale)
    print("Class balance before SMOTE ->", np.bincount(y[tr]))
    X_res, y_res = SMOTE(random_state=42, device=str(dev)).fit_resample(X_train, y[tr])
    print("Class balance after SMOTE ->", np.bincount(y_res))
    np.savez_compressed(PROCESSED_DATA_PATH, X_res=X_res, y_res=y_res, X_test=X_test, y_test=y[te])
    joblib.dump(make_scaler(mean, var, scale, len(tr), feature_names), os.path.join(MODELS_DIR, "scaler.joblib"))
    joblib.dump(feature_names, os.path.join(MODELS_DIR, "columns.joblib"))
    with open(os.path.join(MODELS_DIR, "feature_names.json"), "w") as f:
        json.dump(feature_names, f)
    print("Preprocessing complete.")


if __name__ == "__main__":
    main()
