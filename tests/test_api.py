"""The reference's two API smoke checks (reference tests/test_api.py:1-13), kept as a contract:
a client built at import time, i.e. WITHOUT running the lifespan, must still answer /status and
accept a 30-feature /predict.  The full contract (lifespan, queue, /explain) is in
tests/test_api_contract.py."""
import pytest
from fastapi.testclient import TestClient

from api.app import app

CLIENT = TestClient(app)          # deliberately not a context manager


def test_status():
    body = CLIENT.get("/status")
    assert (body.status_code, body.json()["status"] in {"UP", "OK"}) == (200, True)


@pytest.mark.parametrize("features", [[0.1] * 30])
def test_predict_minimal(features):
    assert CLIENT.post("/predict", json={"features": features}).status_code in {200, 201, 202}
