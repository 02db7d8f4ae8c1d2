"""ORM models (reference path db/models.py)."""
from fraud_detection_amd.store.models import Base, ShapExplanation, StatusEnum, TaskRecord, TransactionResult  # noqa: F401
