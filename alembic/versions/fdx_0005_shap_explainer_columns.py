"""shap_explanations: which explainer produced the row (linear | kernel) and its base value."""
import sqlalchemy as sa
from alembic import op

revision = "fdx_0005"
down_revision = "fdx_0004"
branch_labels = None
depends_on = None


def upgrade() -> None:
    cols = {c["name"] for c in sa.inspect(op.get_bind()).get_columns("shap_explanations")}
    if "explainer" not in cols:
        op.add_column("shap_explanations", sa.Column("explainer", sa.String(32), nullable=True))
    if "base_value" not in cols:
        op.add_column("shap_explanations", sa.Column("base_value", sa.Float(), nullable=True))


def downgrade() -> None:
    op.drop_column("shap_explanations", "base_value")
    op.drop_column("shap_explanations", "explainer")
