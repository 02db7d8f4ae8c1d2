set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -m pytest tests/test_gbdt_gpu.py -q -x > gpurun_out/s12_gbdt_pytest.log 2>&1; echo "gbdt pytest rc=$?" >> gpurun_out/s12_gbdt_pytest.log
tail -30 gpurun_out/s12_gbdt_pytest.log
grep -q "gbdt pytest rc=0" gpurun_out/s12_gbdt_pytest.log || grep -q "rc=1$" gpurun_out/s12_gbdt_pytest.log || exit 3
timeout -k 10 600 python -m pytest tests -m gpu -q -x --deselect tests/test_gbdt_gpu.py > gpurun_out/s12_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s12_pytest.log
timeout -k 10 300 python tools/gbdt_bench.py --rows 2000000 --json gpurun_out/s12_gbdt_bench.json > gpurun_out/s12_gbdt_bench.log 2>&1 && \
timeout -k 10 300 python tools/ubench.py --json gpurun_out/s12_ubench.json > gpurun_out/s12_ubench.log 2>&1 && \
timeout -k 10 300 python tools/newton_trace.py --json gpurun_out/s12_newton_trace.json > gpurun_out/s12_newton_trace.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s12_bench.log 2>&1
rc=$?; tail -3 gpurun_out/s12_pytest.log; cat gpurun_out/s12_gbdt_bench.log; cat gpurun_out/s12_ubench.log; grep "==" gpurun_out/s12_newton_trace.log; tail -c 1500 gpurun_out/s12_bench.log; exit $rc
