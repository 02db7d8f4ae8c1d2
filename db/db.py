"""Engine / session (reference path db/db.py).  DATABASE_URL as in the reference; default is a
local SQLite file (see fraud_detection_amd/store/db.py)."""
from fraud_detection_amd.store.db import database_url, init_db_tables, make_engine, session_factory  # noqa: F401

DATABASE_URL = database_url()
engine = make_engine(DATABASE_URL)
SessionLocal = session_factory(engine)
