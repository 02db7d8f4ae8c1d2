"""Training script (reference path train_model.py).  Env: DATA_CSV, MLFLOW_TRACKING_URI,
MLFLOW_EXPERIMENT, MLFLOW_MODEL_NAME, MLFLOW_AUC_THRESHOLD, MLFLOW_MODEL_STAGE (+ FDX_* knobs).
Runs on the MI355X kernels when a GPU is present, the CPU oracles otherwise.
Implementation: fraud_detection_amd/train.py."""
import sys

from fraud_detection_amd.train import main, run  # noqa: F401

if __name__ == "__main__":
    sys.exit(main())
