set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/s11_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s11_pytest.log
timeout -k 10 300 python tools/ubench.py --json gpurun_out/s11_ubench.json > gpurun_out/s11_ubench.log 2>&1 && \
timeout -k 10 300 python tools/newton_trace.py --json gpurun_out/s11_newton_trace.json > gpurun_out/s11_newton_trace.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s11_bench.log 2>&1
rc=$?; tail -4 gpurun_out/s11_pytest.log; cat gpurun_out/s11_ubench.log; grep "==" gpurun_out/s11_newton_trace.log; tail -c 1600 gpurun_out/s11_bench.log; exit $rc
