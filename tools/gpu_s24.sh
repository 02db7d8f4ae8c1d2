set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "scale or smote or affine or fold or scaler" > gpurun_out/s24_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s24_pytest.log
tail -3 gpurun_out/s24_pytest.log
grep -q "pytest rc=0$" gpurun_out/s24_pytest.log || { grep -n "Error\|assert\|FAILED" gpurun_out/s24_pytest.log | head -40; exit 3; }
timeout -k 10 300 python tools/ubench.py --only scaler_stats,scale_cast_bf16,scaler_stats_cast_bf16,smote_generate_n > gpurun_out/s24_ubench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s24_bench.log 2>&1
rc=$?
cat gpurun_out/s24_ubench.log; grep "^{" gpurun_out/s24_bench.log | head -c 1200; exit $rc
