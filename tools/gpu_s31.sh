set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s31_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s31_pytest.log
tail -3 gpurun_out/s31_pytest.log
grep -q "pytest rc=0$" gpurun_out/s31_pytest.log || { grep -n "Error\|assert\|FAILED\|^E " gpurun_out/s31_pytest.log | head -40; exit 3; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s31_smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/s31_bench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 5 > gpurun_out/s31_bench50.log 2>&1
rc=$?
tail -2 gpurun_out/s31_smoke.log; grep -h "^{" gpurun_out/s31_bench.log gpurun_out/s31_bench50.log | cut -c 1-600; exit $rc
