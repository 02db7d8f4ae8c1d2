"""FastAPI service (reference path api/app.py).  Run: uvicorn api.app:app  or
gunicorn -k uvicorn.workers.UvicornWorker api.app:app --workers 2
Implementation: fraud_detection_amd/serve/app.py."""
from fraud_detection_amd.serve.app import create_app, load_production_engine  # noqa: F401

app = create_app()
