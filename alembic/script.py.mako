## Template for `alembic revision`: every revision in this repo carries the same four
## identifiers the built-in runner (fraud_detection_amd/store/migrations.py) reads.
<%text># -*- revision -*-</%text>
"""${message}

revision ${up_revision} (parent: ${down_revision | comma,n}), generated ${create_date}
"""
import sqlalchemy as sa
from alembic import op
${imports if imports else ""}

revision, down_revision = ${repr(up_revision)}, ${repr(down_revision)}
branch_labels, depends_on = ${repr(branch_labels)}, ${repr(depends_on)}


def upgrade() -> None:
    """Forward DDL for this revision."""
    ${upgrades if upgrades else "return None"}


def downgrade() -> None:
    """Inverse of upgrade()."""
    ${downgrades if downgrades else "return None"}
