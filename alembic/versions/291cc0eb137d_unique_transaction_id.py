"""unique transaction id: already guaranteed by the primary key (no-op, keeps the chain)."""
revision = "291cc0eb137d"
down_revision = "0001_initial_transaction_results"
branch_labels = None
depends_on = None


def upgrade() -> None:
    pass


def downgrade() -> None:
    pass
