set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s50
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s50/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s50/pytest.log
tail -3 gpurun_out/s50/pytest.log
grep -q "pytest rc=0$" gpurun_out/s50/pytest.log || { grep -n "Error\|assert\|FAILED\|^E " gpurun_out/s50/pytest.log | head -40; exit 3; }
timeout -k 10 300 python tools/ubench.py --only smote_generate_n,smote_generate_n_bf16_parents,write_only_fill_n_rows > gpurun_out/s50/ubench.txt 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 5 > gpurun_out/s50/bench.log 2>&1
rc=$?
grep " us" gpurun_out/s50/ubench.txt; grep -h "^{" gpurun_out/s50/bench.log | cut -c 1-300; grep -o '"phase_ms.*' gpurun_out/s50/bench.log | cut -c 1-200; exit $rc
