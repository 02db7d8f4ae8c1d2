"""ORM schema (reference: db/models.py:11-24, alembic/versions/0001_initial_transaction_results.py:17-31,
api/app.py:49-63 raw DDL for shap_explanations).

Dialect-portable: JSON is JSONB on PostgreSQL, TEXT-backed JSON on SQLite; UUIDs use the
SQLAlchemy 2 ``Uuid`` type.  Timestamps come from the database (``CURRENT_TIMESTAMP``) -- the
reference's ``default=datetime`` made every ORM insert raise.
Also holds the durable task-queue table that replaces the Redis/Celery broker.
"""
from __future__ import annotations

import enum
import uuid

from sqlalchemy import JSON, DateTime, Float, Index, Integer, String, Text, Uuid, func
from sqlalchemy.dialects.postgresql import JSONB
from sqlalchemy.orm import DeclarativeBase, Mapped, mapped_column

JSONType = JSON().with_variant(JSONB(), "postgresql")


class Base(DeclarativeBase):
    pass


class StatusEnum(str, enum.Enum):
    PENDING = "PENDING"
    COMPLETED = "COMPLETED"
    FAILED = "FAILED"


class TransactionResult(Base):
    __tablename__ = "transaction_results"
    id: Mapped[uuid.UUID] = mapped_column(Uuid(as_uuid=True), primary_key=True, default=uuid.uuid4)
    input_data: Mapped[dict] = mapped_column(JSONType, nullable=False)
    shap_values: Mapped[dict | None] = mapped_column(JSONType, nullable=True)
    prediction_score: Mapped[float | None] = mapped_column(Float, nullable=True)
    status: Mapped[str] = mapped_column(String(50), nullable=False, default=StatusEnum.PENDING.value)
    created_at = mapped_column(DateTime(timezone=True), server_default=func.current_timestamp())
    updated_at = mapped_column(DateTime(timezone=True), server_default=func.current_timestamp(),
                               onupdate=func.current_timestamp())


class ShapExplanation(Base):
    __tablename__ = "shap_explanations"
    transaction_id: Mapped[str] = mapped_column(String(255), primary_key=True)
    correlation_id: Mapped[str | None] = mapped_column(String(255), nullable=True)
    shap_values: Mapped[dict] = mapped_column(JSONType, nullable=False)
    feature_names: Mapped[list | None] = mapped_column(JSONType, nullable=True)
    explainer: Mapped[str | None] = mapped_column(String(32), nullable=True)   # linear | kernel (fdx_0005)
    base_value: Mapped[float | None] = mapped_column(Float, nullable=True)     # E[f] over the background
    created_at = mapped_column(DateTime(timezone=True), server_default=func.current_timestamp())


class TaskRecord(Base):
    """Durable queue row (replaces the Redis list ``celery``)."""

    __tablename__ = "fdx_task_queue"
    id: Mapped[str] = mapped_column(String(36), primary_key=True)
    name: Mapped[str] = mapped_column(String(255), nullable=False)
    args: Mapped[list] = mapped_column(JSONType, nullable=False)
    kwargs: Mapped[dict] = mapped_column(JSONType, nullable=False)
    headers: Mapped[dict] = mapped_column(JSONType, nullable=False)
    status: Mapped[str] = mapped_column(String(16), nullable=False, default="QUEUED")
    attempts: Mapped[int] = mapped_column(Integer, nullable=False, default=0)
    max_retries: Mapped[int] = mapped_column(Integer, nullable=False, default=5)
    eta: Mapped[float] = mapped_column(Float, nullable=False)
    lease_until: Mapped[float] = mapped_column(Float, nullable=False, default=0.0)
    worker: Mapped[str | None] = mapped_column(String(128), nullable=True)
    result: Mapped[dict | None] = mapped_column(JSONType, nullable=True)
    error: Mapped[str | None] = mapped_column(Text, nullable=True)
    created_at: Mapped[float] = mapped_column(Float, nullable=False)
    updated_at: Mapped[float] = mapped_column(Float, nullable=False)

    __table_args__ = (Index("ix_fdx_task_queue_status_eta", "status", "eta"),)


class SchemaVersion(Base):
    __tablename__ = "fdx_schema_version"
    revision: Mapped[str] = mapped_column(String(64), primary_key=True)
    applied_at = mapped_column(DateTime(timezone=True), server_default=func.current_timestamp())
