set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q > gpurun_out/s6_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s6_pytest.log
timeout -k 10 300 python tools/ubench.py --json gpurun_out/s6_ubench.json > gpurun_out/s6_ubench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s6_bench.log 2>&1
rc=$?; tail -4 gpurun_out/s6_pytest.log; cat gpurun_out/s6_ubench.log; tail -c 1500 gpurun_out/s6_bench.log; exit $rc
