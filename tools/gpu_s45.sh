set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s45
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "knn or smote" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s45/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s45/pytest.log
tail -3 gpurun_out/s45/pytest.log
grep -q "pytest rc=0$" gpurun_out/s45/pytest.log || { grep -n "Error\|assert\|FAILED\|^E " gpurun_out/s45/pytest.log | head -40; exit 3; }
timeout -k 10 300 python tools/ubench.py --only knn_topk_13600,knn_topk_13600_unseeded,knn_topk_13600_bf16x3,knn_topk_13600_bf16x3_unseeded > gpurun_out/s45/ubench.txt 2>&1
rc=$?
grep " us" gpurun_out/s45/ubench.txt; exit $rc
