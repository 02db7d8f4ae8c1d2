set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import torch; print(torch.cuda.get_device_name(0))" > gpurun_out/s1_info.log 2>&1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -x -q > gpurun_out/s1_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s1_pytest.log
tail -5 gpurun_out/s1_pytest.log
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/s1_smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/s1_bench.log 2>&1
rc=$?; tail -3 gpurun_out/s1_smoke.log gpurun_out/s1_bench.log; exit $rc
