"""Pydantic request/response models (reference: api/app.py:110-119, api/schemas.py:5-23)."""
from __future__ import annotations

import uuid
from typing import Dict, List, Optional

from pydantic import BaseModel, Field


class TransactionIn(BaseModel):
    transaction_id: str = Field(default_factory=lambda: str(uuid.uuid4()))
    features: list


class PredictionOut(BaseModel):
    transaction_id: str
    prediction: int
    score: float
    correlation_id: str
    explanation_status: str


class TransactionFeatures(BaseModel):
    """Feature name -> value mapping (api/schemas.py:5-11)."""

    features: Dict[str, float] = Field(..., description="Feature name -> numeric value mapping")


class PredictAccepted(BaseModel):
    transaction_id: str = Field(..., description="UUID identifying the queued transaction")
    status: str = Field("PENDING", description="Initial status")


class PredictResponse(BaseModel):
    transaction_id: str
    status: str
    prediction_score: Optional[float] = None
    detail: Optional[str] = None


class BatchIn(BaseModel):
    rows: List[List[float]]
    explain: bool = False


class BatchOut(BaseModel):
    predictions: List[int]
    scores: List[float]
    shap_values: Optional[List[List[float]]] = None
