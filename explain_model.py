"""Batch explainability (reference path explain_model.py:1-49): LinearSHAP of the served model on
the (already scaled) test split, summary plot and dependence plots of the top-3 features by mean
|phi|, saved under plots/.  Fixes the reference's double scaling (explain_model.py:19; SURVEY.md
App. D item 3): the npz features are already standardized, so the explainer runs on them
directly, with the test set as background (LinearExplainer(model, X_test_scaled)).
``--kernel`` additionally runs KernelSHAP (MFMA coalition GEMM) on ``--n`` rows; under torchrun
(one rank per GPU) the rows are sharded across ranks (contiguous slices, collective C7 broadcast of
the design is implicit: every rank builds the same cached design) and the phi rows are gathered to
rank 0 (collective C8), which writes ``plots/kernelshap_values.npy``.  ``--tree``: when a GBDT was
trained (``train_model.py --model gbdt`` -> models/xgb_model.json), explain it with interventional
TreeSHAP (exact, margin space; shap.TreeExplainer(model, data=background) semantics) on --n rows:
plots/treeshap_summary.png and plots/treeshap_values.npy."""
import argparse
import os

import matplotlib

matplotlib.use("Agg")
import matplotlib.pyplot as plt  # noqa: E402
import numpy as np  # noqa: E402

from fraud_detection_amd.compat.sklearn_export import load_artifacts  # noqa: E402
from fraud_detection_amd.models.explainers import KernelExplainer, LinearExplainer  # noqa: E402


def summary_plot(phi, X, names, path):
    order = np.argsort(np.abs(phi).mean(0))[::-1][:20]
    fig, ax = plt.subplots(figsize=(12, 8))
    for row, j in enumerate(order[::-1]):
        v = X[:, j]
        lo, hi = np.percentile(v, [5, 95])
        col = np.clip((v - lo) / (hi - lo + 1e-12), 0, 1)
        jitter = (np.random.default_rng(j).random(len(v)) - 0.5) * 0.6
        ax.scatter(phi[:, j], row + jitter, c=col, cmap="coolwarm", s=4, alpha=0.6)
    ax.set_yticks(range(len(order)), [names[j] for j in order[::-1]])
    ax.set_xlabel("SHAP value (impact on log-odds)")
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def dependence_plot(j, phi, X, names, path):
    fig, ax = plt.subplots(figsize=(8, 6))
    ax.scatter(X[:, j], phi[:, j], s=4, alpha=0.5)
    ax.set_xlabel(names[j])
    ax.set_ylabel(f"SHAP value for {names[j]}")
    fig.tight_layout()
    fig.savefig(path)
    plt.close(fig)


def kernel_sharded(ke, X: np.ndarray, comm):
    """KernelSHAP of X split over the ranks of ``comm`` (None = this process): each rank explains
    its contiguous shard on its own device, rank 0 receives every row in order."""
    import torch

    rank, world = (comm.rank, comm.world_size) if comm is not None else (0, 1)
    lo, hi = rank * len(X) // world, (rank + 1) * len(X) // world
    phi, fx, f0 = ke.explain(X[lo:hi])
    if comm is None or world == 1:
        return phi, fx, f0
    part = torch.from_numpy(np.concatenate([phi, fx[:, None]], 1).astype(np.float64))
    if comm.backend == "nccl":
        part = part.to(torch.device("cuda", torch.cuda.current_device()))
    allp, _ = comm.all_gather_rows(part)
    allp = allp.cpu().numpy()
    return allp[:, :-1], allp[:, -1], f0


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", action="store_true", help="also run KernelSHAP on --n rows")
    ap.add_argument("--rows", "--n", dest="n", type=int, default=1000, help="KernelSHAP rows (alias --n)")
    ap.add_argument("--tree", action="store_true", help="TreeSHAP of the GBDT model (models/xgb_model.json)")
    a = ap.parse_args(argv)
    comm = None
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch

        from fraud_detection_amd.parallel.comm import Communicator

        if torch.cuda.is_available():
            torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        comm = Communicator()
    try:
        return _main(a, comm)
    finally:
        if comm is not None:
            comm.close()


def _main(a, comm):
    lead = comm is None or comm.rank == 0
    os.makedirs("plots", exist_ok=True)
    print("Loading model, scaler, and data...")
    art = load_artifacts("models/logistic_model.joblib", "models/scaler.joblib", "models/feature_names.json")
    data = np.load("data/preprocessed_data.npz")
    X_test = data["X_test"].astype(np.float32)
    d = X_test.shape[1]
    names = [f"Feature_{i}" for i in range(d)]
    # features are already standardized: identity scaler, background = test set
    expl = LinearExplainer(art.coef, art.intercept, np.zeros(d), np.ones(d), background=X_test)
    print("Computing SHAP values for the test set...")
    phi = expl.shap_values(X_test)
    top = np.argsort(np.abs(phi).mean(0))[-3:][::-1]
    if lead:
        summary_plot(phi, X_test, names, "plots/shap_summary.png")
        for j in top:
            dependence_plot(j, phi, X_test, names, f"plots/shap_dependence_feature_{j}.png")
    out = {"top_features": [int(j) for j in top], "expected_value": expl.expected_value}
    if a.kernel:
        w = np.zeros(32)
        w[:d] = art.coef
        bg = X_test[np.random.default_rng(0).choice(len(X_test), min(100, len(X_test)), replace=False)]
        dev = "auto"
        if comm is not None and comm.backend == "nccl":
            import torch

            dev = f"cuda:{torch.cuda.current_device()}"
        ke = KernelExplainer(w, art.intercept, bg, link="identity", device=dev)
        phik, fx, f0 = kernel_sharded(ke, X_test[: a.n], comm)
        out["kernelshap_rows"] = int(phik.shape[0])
        out["kernelshap_ranks"] = comm.world_size if comm is not None else 1
        out["kernelshap_efficiency_max_err"] = float(np.abs(phik.sum(1) - (fx - f0)).max())
        if lead:
            np.save("plots/kernelshap_values.npy", phik)
    if a.tree and lead:
        out.update(tree_explain(X_test, names, a.n))
    print("SHAP explainability completed. Plots saved in 'plots/'.", out)
    return out


def tree_explain(X_test, names, n) -> dict:
    """Interventional TreeSHAP of the GBDT on the (standardized) test rows, background = 100 test
    rows: the ensemble was trained on standardized rows, so the explainer's scaler is identity."""
    import json

    from fraud_detection_amd.models.explainers import TreeExplainer
    from fraud_detection_amd.models.gbdt import MODEL_FILE
    from fraud_detection_amd.ops.gbdt import TreeEnsemble

    path = os.path.join("models", MODEL_FILE)
    if not os.path.exists(path):
        raise SystemExit(f"--tree needs a GBDT model at {path} (train_model.py --model gbdt)")
    with open(path) as f:
        ens = TreeEnsemble.from_dict(json.load(f))
    d = X_test.shape[1]
    bg = X_test[np.random.default_rng(1).choice(len(X_test), min(100, len(X_test)), replace=False)]
    te = TreeExplainer(ens, np.zeros(d), np.ones(d), bg)
    rows = X_test[:n]
    phi, fx, f0 = te.explain(rows)
    summary_plot(phi, rows, names, "plots/treeshap_summary.png")
    np.save("plots/treeshap_values.npy", phi)
    return {"treeshap_rows": int(phi.shape[0]), "treeshap_expected_value": float(f0),
            "treeshap_efficiency_max_err": float(np.abs(phi.sum(1) - (fx - f0)).max())}


if __name__ == "__main__":
    main()
