"""Typed configuration: defaults -> optional YAML file (FDX_CONFIG) -> environment (the reference's
variable names) -> explicit overrides / CLI flags.
"""
from __future__ import annotations

import os
from dataclasses import asdict, dataclass, field, fields

import yaml

# env var -> attribute (reference names first)
ENV_MAP = {
    "DATA_CSV": "data_csv",
    "MLFLOW_TRACKING_URI": "mlflow_tracking_uri",
    "MLFLOW_EXPERIMENT": "mlflow_experiment",
    "MLFLOW_MODEL_NAME": "mlflow_model_name",
    "MLFLOW_AUC_THRESHOLD": "mlflow_auc_threshold",
    "MLFLOW_MODEL_STAGE": "mlflow_model_stage",
    "DATABASE_URL": "database_url",
    "CELERY_BROKER_URL": "celery_broker_url",
    "MODEL_PATH": "model_path",
    "FEATURE_NAMES_PATH": "feature_names_path",
    "SCALER_PATH": "scaler_path",
    "OTEL_EXPORTER_OTLP_ENDPOINT": "otel_endpoint",
    "OTEL_SERVICE_NAME": "otel_service_name",
    "FDX_DEVICE": "device",
    "FDX_DTYPE": "dtype",
    "FDX_SOLVER": "solver",
    "FDX_MICROBATCH_US": "microbatch_us",
    "FDX_MICROBATCH_MAX": "microbatch_max",
    "FDX_GPU_OWNER_RING": "gpu_owner_ring",
    "FDX_QUEUE_URL": "queue_url",
    "FDX_XAI_BATCH": "xai_batch",
    "FDX_KERNELSHAP_NSAMPLES": "kernelshap_nsamples",
    "FDX_KERNELSHAP_BACKGROUND": "kernelshap_background",
    "FDX_KERNELSHAP_LINK": "kernelshap_link",
    "FDX_XAI_METHOD": "xai_method",
    "FDX_SMOTE_K": "smote_k",
    "FDX_SEED": "seed",
    "FDX_SPLIT": "split",
    "FDX_CV_PARALLEL": "cv_parallel",
    "FDX_CHECKPOINT_DIR": "checkpoint_dir",
}


@dataclass
class Settings:
    data_csv: str = "data/creditcard.csv"
    mlflow_tracking_uri: str = "file:./mlruns"
    mlflow_experiment: str = "fraud-detection-ci"
    mlflow_model_name: str = "fraud-detection-model"
    mlflow_auc_threshold: float = 0.95
    mlflow_model_stage: str = "production"
    database_url: str = "sqlite:///./fraud.db"
    celery_broker_url: str = "sql"
    queue_url: str = ""
    model_path: str = "./models/logistic_model.joblib"
    scaler_path: str = "./models/scaler.joblib"
    feature_names_path: str = "./models/feature_names.json"
    otel_endpoint: str = "http://otel-collector:4318/v1/traces"
    otel_service_name: str = "fraud-api"
    device: str = "auto"           # auto | cuda | cpu
    dtype: str = "bf16"            # bf16 | fp8 (training row storage)
    solver: str = "newton"         # newton | sgd
    microbatch_us: int = 0         # GPU owner: extra wait for more rows (0 = continuous batching)
    microbatch_max: int = 8192
    gpu_owner_ring: str = ""       # multi-worker serving: the GPU-owner process's ring (serve/launch.py)
    xai_batch: int = 512
    kernelshap_nsamples: int = 0   # 0 -> shap default 2*M + 2048
    kernelshap_background: int = 100   # rows saved with the model (shap_background.npy)
    kernelshap_link: str = "identity"  # identity (probabilities) | logit | logit_model
    xai_method: str = "auto"           # auto (the family default: linear | GBDT kernel) | linear | kernel | tree
    smote_k: int = 5
    seed: int = 42
    split: str = "auto"            # sklearn (reference-exact) | device (K3 kernel) | auto
    cv_parallel: str = "auto"      # dp (each fold over all ranks) | fold (whole folds per rank) | auto
    checkpoint_dir: str = ""       # job resume: completed CV folds + GBDT tree checkpoints
    extra: dict = field(default_factory=dict)

    @classmethod
    def load(cls, path: str | None = None, env: dict | None = None, **overrides) -> "Settings":
        s = cls()
        path = path or os.getenv("FDX_CONFIG")
        if path and os.path.exists(path):
            with open(path) as f:
                data = yaml.safe_load(f) or {}
            s._apply(data)
        env = os.environ if env is None else env
        s._apply({attr: env[k] for k, attr in ENV_MAP.items() if k in env})
        s._apply(overrides)
        return s

    def _apply(self, data: dict):
        types = {f.name: f.type for f in fields(self)}
        for k, v in data.items():
            if k not in types:
                self.extra[k] = v
                continue
            cur = getattr(self, k)
            if isinstance(cur, bool):
                v = str(v).lower() in ("1", "true", "yes")
            elif isinstance(cur, int):
                v = int(v)
            elif isinstance(cur, float):
                v = float(v)
            setattr(self, k, v)

    def as_dict(self) -> dict:
        return asdict(self)


def get_settings(**overrides) -> Settings:
    return Settings.load(**overrides)
