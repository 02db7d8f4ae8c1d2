"""Pydantic schemas (reference path api/schemas.py)."""
from fraud_detection_amd.serve.schemas import (  # noqa: F401
    BatchIn, BatchOut, PredictAccepted, PredictionOut, PredictResponse, TransactionFeatures, TransactionIn)
