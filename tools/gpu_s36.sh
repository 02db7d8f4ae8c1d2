set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s36
timeout -k 10 600 python -u -m pytest tests/test_virtual_smote_gpu.py tests/test_kernels_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s36/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s36/pytest.log
tail -3 gpurun_out/s36/pytest.log
grep -q "pytest rc=0$" gpurun_out/s36/pytest.log || { grep -n "Error\|assert\|FAILED\|^E " gpurun_out/s36/pytest.log | head -40; exit 3; }
timeout -k 10 300 python tools/ubench.py --only logreg_pass_hess_s3_2n,logreg_pass_grad_2n,logreg_pass_virtual_hess_s3_2n,logreg_pass_virtual_grad_2n,newton_fit_2n_tol1e-4,newton_fit_virtual_2n_tol1e-4,smote_generate_n > gpurun_out/s36/ubench.txt 2>&1 && \
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > gpurun_out/s36/bench.log 2>&1
rc=$?
grep " us" gpurun_out/s36/ubench.txt; grep -h "^{" gpurun_out/s36/bench.log | cut -c 1-900; exit $rc
