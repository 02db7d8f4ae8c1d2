"""Versioned schema migrations (alembic is not installed in this image; this runner keeps the
reference's revision chain: alembic/versions/0001_initial_transaction_results.py ->
2025116_291cc0eb137d (unique constraint, empty upstream) -> 2025116_fbae492048d4
(shap_explanations, empty upstream; the table was created by raw DDL in api/app.py:49-63)).

    python -m fraud_detection_amd.store.migrations upgrade [head]
    python -m fraud_detection_amd.store.migrations current
"""
from __future__ import annotations

import argparse
import logging

from sqlalchemy import inspect, select, text
from sqlalchemy.engine import Engine

from .db import make_engine
from .models import Base, SchemaVersion, ShapExplanation, TaskRecord, TransactionResult

logger = logging.getLogger(__name__)


def _create(*tables):
    def op(engine: Engine):
        Base.metadata.create_all(bind=engine, tables=[t.__table__ for t in tables])
    return op


def _noop(engine: Engine):
    return None


def _add_columns(table, cols):
    """ALTER TABLE ADD COLUMN for the ones a database created before this revision lacks (a table
    created fresh from the current models already has them)."""
    def op(engine: Engine):
        have = {c["name"] for c in inspect(engine).get_columns(table.__tablename__)}
        with engine.begin() as c:
            for name in cols:
                if name not in have:
                    col = table.__table__.c[name]
                    c.execute(text(f"ALTER TABLE {table.__tablename__} ADD COLUMN {name} "
                                   f"{col.type.compile(dialect=engine.dialect)}"))
    return op


REVISIONS = [
    ("0001", "initial transaction_results", _create(TransactionResult)),
    ("291cc0eb137d", "unique constraint on transaction id (primary key already unique)", _noop),
    ("fbae492048d4", "shap_explanations table", _create(ShapExplanation)),
    ("fdx_0004", "durable task queue", _create(TaskRecord)),
    ("fdx_0005", "shap_explanations.explainer / base_value", _add_columns(ShapExplanation, ["explainer", "base_value"])),
]


def current(engine: Engine | None = None) -> list[str]:
    engine = engine or make_engine()
    if not inspect(engine).has_table(SchemaVersion.__tablename__):
        return []
    with engine.connect() as c:
        return [r[0] for r in c.execute(select(SchemaVersion.revision))]


def upgrade(engine: Engine | None = None, target: str = "head") -> list[str]:
    engine = engine or make_engine()
    Base.metadata.create_all(bind=engine, tables=[SchemaVersion.__table__])
    done = set(current(engine))
    applied = []
    for rev, desc, op in REVISIONS:
        if rev not in done:
            logger.info("migrating %s: %s", rev, desc)
            op(engine)
            with engine.begin() as c:
                c.execute(SchemaVersion.__table__.insert().values(revision=rev))
            applied.append(rev)
        if rev == target:
            break
    return applied


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("cmd", choices=["upgrade", "current"])
    ap.add_argument("target", nargs="?", default="head")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    if a.cmd == "upgrade":
        print("applied:", upgrade(target=a.target))
    else:
        print("current:", current())


if __name__ == "__main__":
    main()
