set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q -x -k "fp8 or logreg_pass or predict" > gpurun_out/s30_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s30_pytest.log
tail -3 gpurun_out/s30_pytest.log
grep -q "pytest rc=0$" gpurun_out/s30_pytest.log || { grep -n "Error\|assert\|FAILED\|^E " gpurun_out/s30_pytest.log | head -40; exit 3; }
timeout -k 10 300 python tools/ubench.py --only logreg_pass_fp8_hess,logreg_pass_hess_s3_2n,predict_fp8,predict_bf16_2n,scale_cast_fp8 > gpurun_out/s30_ubench.log 2>&1 && \
timeout -k 10 600 python tools/baseline_configs.py --only c5 > gpurun_out/s30_c5.log 2>&1
rc=$?
grep us gpurun_out/s30_ubench.log; grep "^{" gpurun_out/s30_c5.log; exit $rc
