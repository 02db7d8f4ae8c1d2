"""durable task queue (replaces the Redis list used by Celery)."""
from alembic import op

from fraud_detection_amd.store.models import TaskRecord

revision = "fdx_0004"
down_revision = "fbae492048d4"
branch_labels = None
depends_on = None


def upgrade() -> None:
    TaskRecord.__table__.create(bind=op.get_bind(), checkfirst=True)


def downgrade() -> None:
    op.drop_table(TaskRecord.__tablename__)
