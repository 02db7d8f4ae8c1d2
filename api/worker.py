"""Reference path api/worker.py was a dead duplicate of xai_tasks.py.
Kept as an alias so ``celery -A api.worker`` style invocations resolve to the live task app."""
from xai_tasks import celery_app, compute_shap  # noqa: F401
