set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x > gpurun_out/s26_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s26_pytest.log
tail -3 gpurun_out/s26_pytest.log
grep -q "pytest rc=0$" gpurun_out/s26_pytest.log || { grep -n "Error\|assert\|FAILED" gpurun_out/s26_pytest.log | head -40; exit 3; }
timeout -k 10 300 python tools/ubench.py --only scaler_stats_cast_bf16,smote_generate_n > gpurun_out/s26_ubench_default.log 2>&1 && \
FDX_NT_STORES=1 timeout -k 10 300 python tools/ubench.py --only scaler_stats_cast_bf16,smote_generate_n > gpurun_out/s26_ubench_nt.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s26_bench.log 2>&1 && \
FDX_NT_STORES=1 timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s26_bench_nt.log 2>&1 && \
timeout -k 10 400 python tools/newton_trace.py --rows 10000000 > gpurun_out/s26_trace.log 2>&1
rc=$?
tail -2 gpurun_out/s26_ubench_default.log gpurun_out/s26_ubench_nt.log; grep -h "^{" gpurun_out/s26_bench.log gpurun_out/s26_bench_nt.log | cut -c 1-330; grep "^==" gpurun_out/s26_trace.log; exit $rc
