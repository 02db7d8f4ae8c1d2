"""shap_explanations table (created by raw DDL at API startup in the reference)."""
from alembic import op

from fraud_detection_amd.store.models import ShapExplanation

revision = "fbae492048d4"
down_revision = "291cc0eb137d"
branch_labels = None
depends_on = None


def upgrade() -> None:
    ShapExplanation.__table__.create(bind=op.get_bind(), checkfirst=True)


def downgrade() -> None:
    op.drop_table(ShapExplanation.__tablename__)
