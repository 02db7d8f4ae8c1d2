#!/usr/bin/env bash
# Apply DB migrations, then exec the container command (reference: run_migrations.sh).
set -euo pipefail
echo "Running database migrations against ${DATABASE_URL:-sqlite:///./fraud.db}"
python -m fraud_detection_amd.store.migrations upgrade head
exec "$@"
