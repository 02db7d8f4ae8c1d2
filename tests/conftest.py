import os
import sys
import tempfile

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Hermetic service state for the whole test session (set before any api/db module import).
_TMP = tempfile.mkdtemp(prefix="fdx_tests_")
os.environ.setdefault("DATABASE_URL", f"sqlite:///{_TMP}/fraud.db")
os.environ.setdefault("MLFLOW_TRACKING_URI", f"file:{_TMP}/mlruns")
os.environ.setdefault("MODEL_PATH", os.path.join(ROOT, "models", "logistic_model.joblib"))
os.environ.setdefault("FEATURE_NAMES_PATH", os.path.join(ROOT, "models", "feature_names.json"))
os.environ.setdefault("FDX_DEVICE", "cpu")
os.chdir(ROOT)

import torch  # noqa: E402  (before any extension import)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP extension")
    config.addinivalue_line("markers", "slow: long-running test")


def pytest_collection_modifyitems(config, items):
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from fraud_detection_amd.ops.native import native

    native()  # GPU tests must exercise the HIP kernels, never a fallback
    return torch.device("cuda", 0)
