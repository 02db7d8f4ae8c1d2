# MI355X (gfx950) image: ROCm PyTorch base, native HIP kernels compiled at build time.
#   docker build -t fraud-detection-amd .
#   docker run --device=/dev/kfd --device=/dev/dri --group-add video --group-add render \
#              -p 8000:8000 fraud-detection-amd
ARG BASE=rocm/pytorch:rocm7.0_ubuntu22.04_py3.10_pytorch_release_2.10.0
FROM ${BASE}

ENV PYTHONDONTWRITEBYTECODE=1 \
    PYTHONUNBUFFERED=1 \
    PYTORCH_ROCM_ARCH=gfx950 \
    HSA_ENABLE_IPC_MODE_LEGACY=0 \
    FDX_DEVICE=auto

WORKDIR /app
COPY requirements.txt .
RUN pip install --no-cache-dir -r requirements.txt

COPY . .
# hipcc --offload-arch=gfx950 for every kernel + the RCCL communicator + the CSV reader
RUN python -m fraud_detection_amd.build_native && python -c "import __graft_entry__ as g; g.build()"

RUN useradd --create-home --uid 10001 appuser \
    && usermod -aG video,render appuser 2>/dev/null || true \
    && chown -R appuser /app
USER appuser

EXPOSE 8000 8001
ENTRYPOINT ["/app/run_migrations.sh"]
# one GPU-owner process + 2 HTTP workers forwarding through a shared-memory ring (serve/launch.py);
# the reference ran gunicorn --workers 2 with a model copy per worker (Dockerfile:21)
CMD ["python", "-m", "fraud_detection_amd.serve.launch", "--host", "0.0.0.0", "--port", "8000", "--workers", "2"]
