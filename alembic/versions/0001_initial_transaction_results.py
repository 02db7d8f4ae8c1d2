"""transaction_results (same revision id as the reference chain)."""
from alembic import op

from fraud_detection_amd.store.models import TransactionResult

revision = "0001_initial_transaction_results"
down_revision = None
branch_labels = None
depends_on = None


def upgrade() -> None:
    TransactionResult.__table__.create(bind=op.get_bind(), checkfirst=True)


def downgrade() -> None:
    op.drop_table(TransactionResult.__tablename__)
