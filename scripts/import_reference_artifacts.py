#!/usr/bin/env python3
"""Re-export the reference's shipped LogisticRegression + StandardScaler as our own artifacts.

The reference's models/*.joblib are sklearn 1.6.1 pickles.  They are decoded
with the NON-executing decoder (fraud_detection_amd/compat/safe_joblib.py), and their fitted
parameters are written as fresh sklearn 1.7 objects plus a JSON fixture.  Nothing from the
reference's pickles is executed or loaded by pickle.

Usage: python scripts/import_reference_artifacts.py [--ref /root/reference] [--out models]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from fraud_detection_amd.compat import safe_joblib  # noqa: E402
from fraud_detection_amd.compat.sklearn_export import LinearArtifacts, save_artifacts  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--out", default="models")
    ap.add_argument("--fixture", default="tests/fixtures/reference_lr_params.json")
    a = ap.parse_args()
    m = safe_joblib.decode_logistic(os.path.join(a.ref, "models/logistic_model.joblib"))
    s = safe_joblib.decode_scaler(os.path.join(a.ref, "models/scaler.joblib"))
    cols = safe_joblib.decode_list(os.path.join(a.ref, "models/columns.joblib"))
    art = LinearArtifacts(coef=m["coef"][0], intercept=float(m["intercept"][0]), mean=s["mean_"], var=s["var_"],
                          scale=s["scale_"], n_samples_seen=s["n_samples_seen"], feature_names=cols,
                          n_iter=int(m["n_iter"][0]), C=m["C"])
    paths = save_artifacts(art, a.out)
    os.makedirs(os.path.dirname(a.fixture), exist_ok=True)
    with open(a.fixture, "w") as f:
        json.dump({"coef": art.coef.tolist(), "intercept": art.intercept, "mean": art.mean.tolist(),
                   "var": art.var.tolist(), "scale": art.scale.tolist(), "n_samples_seen": art.n_samples_seen,
                   "feature_names": cols, "n_iter": art.n_iter, "C": art.C,
                   "source": "reference models/*.joblib via safe_joblib (sklearn 1.6.1 pickles)"}, f, indent=1)
    print(json.dumps(paths, indent=1))


if __name__ == "__main__":
    main()
