set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -q -x -k "knn or smote" > gpurun_out/s17_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s17_pytest.log
tail -3 gpurun_out/s17_pytest.log
grep -q "pytest rc=0$" gpurun_out/s17_pytest.log || exit 3
timeout -k 10 300 python tools/ubench.py --only knn_topk_13600,smote_generate_n,compact_indices > gpurun_out/s17_ubench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s17_bench.log 2>&1
rc=$?; cat gpurun_out/s17_ubench.log; tail -c 900 gpurun_out/s17_bench.log; exit $rc
