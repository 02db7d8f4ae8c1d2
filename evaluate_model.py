"""Offline evaluation (reference path evaluate_model.py:1-63): confusion matrix, classification
report and ROC curve/AUC of models/logistic_model.joblib on data/preprocessed_data.npz, saved as
plots/confusion_matrix.png and plots/roc_curve.png.  Scores come from the device predict kernel
(K5) and the AUC from the exact device kernel (K10) when a GPU is present."""
import os

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402
import torch  # noqa: E402
from sklearn.metrics import classification_report, roc_curve  # noqa: E402

from fraud_detection_amd.compat.sklearn_export import load_artifacts  # noqa: E402
from fraud_detection_amd.ops import metrics as M  # noqa: E402
from fraud_detection_amd.ops import predict as P  # noqa: E402


def scores(X_test: np.ndarray, art, dev) -> torch.Tensor:
    """log-odds of the scaled test rows (the npz holds scaled features) from the fused predict
    kernel K5 (identity scaler: a = coef, c = 0); the CPU oracle without a GPU."""
    d = X_test.shape[1]
    a = np.zeros(32)
    a[:d] = art.coef
    Xt = torch.from_numpy(np.ascontiguousarray(X_test, np.float32)).to(dev)
    _, _, z = P.predict_shap_raw(Xt, torch.from_numpy(a), torch.zeros(32, dtype=torch.float64),
                                 float(art.intercept), dphi=0, want_logit=True)
    return z


def main():
    os.makedirs("plots", exist_ok=True)
    print("Loading model and test data...")
    art = load_artifacts("models/logistic_model.joblib", "models/scaler.joblib", "models/feature_names.json")
    data = np.load("data/preprocessed_data.npz")
    X_test, y_test = data["X_test"], data["y_test"].astype(np.uint8)
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    zt = scores(X_test, art, dev)
    yt = torch.from_numpy(y_test).to(dev)
    z = zt.cpu().numpy().astype(np.float64)
    y_pred = (z > 0).astype(int)
    y_proba = 1.0 / (1.0 + np.exp(-z))
    tn, fp, fn, tp = (int(v) for v in M.confusion_counts(zt, yt, 0.0))
    cm = np.array([[tn, fp], [fn, tp]])
    print("Confusion Matrix:")
    print(cm)
    fig, ax = plt.subplots(figsize=(6, 4))
    ax.imshow(cm, cmap="Blues")
    for (i, j), v in np.ndenumerate(cm):
        ax.text(j, i, str(v), ha="center", va="center", color="black")
    ax.set_xticks([0, 1], ["Non-Fraud", "Fraud"])
    ax.set_yticks([0, 1], ["Non-Fraud", "Fraud"])
    ax.set_title("Confusion Matrix")
    ax.set_xlabel("Predicted")
    ax.set_ylabel("Actual")
    fig.tight_layout()
    fig.savefig("plots/confusion_matrix.png")
    plt.close(fig)
    print("Classification Report:")
    print(classification_report(y_test, y_pred))
    roc_auc = M.roc_auc(zt, yt)
    fpr, tpr, _ = roc_curve(y_test, y_proba)
    fig, ax = plt.subplots(figsize=(6, 4))
    ax.plot(fpr, tpr, label=f"AUC = {roc_auc:.4f}")
    ax.plot([0, 1], [0, 1], "k--", label="Random Guess")
    ax.set_xlabel("False Positive Rate")
    ax.set_ylabel("True Positive Rate")
    ax.set_title("ROC Curve")
    ax.legend()
    fig.tight_layout()
    fig.savefig("plots/roc_curve.png")
    plt.close(fig)
    print(f"Evaluation complete (AUC {roc_auc:.4f}). Plots saved to 'plots/'.")
    return {"auc": roc_auc, "confusion": cm.tolist()}


if __name__ == "__main__":
    main()
