set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s48
timeout -k 10 600 python -u -m pytest tests -k "kernelshap or explain or xai" -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s48/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s48/pytest.log
tail -3 gpurun_out/s48/pytest.log
grep -q "pytest rc=0$" gpurun_out/s48/pytest.log || { grep -n "Error\|assert\|FAILED\|^E " gpurun_out/s48/pytest.log | head -40; exit 3; }
timeout -k 10 120 python tools/kernelshap_stamps.py > gpurun_out/s48/stamps.txt 2>&1 && \
timeout -k 10 300 python tools/ubench.py --only kernelshap_1k_expl > gpurun_out/s48/ubench.txt 2>&1
rc=$?
grep -hv amdgpu.ids gpurun_out/s48/stamps.txt; grep " us" gpurun_out/s48/ubench.txt; exit $rc
