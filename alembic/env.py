"""alembic environment for the fraud_detection_amd store.

URL: DATABASE_URL through Settings (same default as the app and the built-in migration runner).
Metadata: fraud_detection_amd.store.models.Base, so `alembic revision --autogenerate` diffs the
ORM tables (transaction_results, shap_explanations, task_queue).  Logging is configured here,
not in alembic.ini.
"""
import logging

from alembic import context
from sqlalchemy import create_engine, pool

from fraud_detection_amd.config import Settings
from fraud_detection_amd.store.models import Base

logging.basicConfig(level=logging.INFO, format="%(levelname)-5.5s [%(name)s] %(message)s")
logging.getLogger("sqlalchemy.engine").setLevel(logging.WARNING)

URL = Settings.load().database_url
META = Base.metadata


def _offline() -> None:
    # emit SQL to stdout (alembic upgrade --sql)
    context.configure(url=URL, target_metadata=META, literal_binds=True,
                      dialect_opts={"paramstyle": "named"})
    with context.begin_transaction():
        context.run_migrations()


def _online() -> None:
    engine = create_engine(URL, poolclass=pool.NullPool)
    try:
        with engine.connect() as conn:
            context.configure(connection=conn, target_metadata=META, compare_type=True)
            with context.begin_transaction():
                context.run_migrations()
    finally:
        engine.dispose()


(_offline if context.is_offline_mode() else _online)()
