set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/s25_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s25_pytest.log
tail -3 gpurun_out/s25_pytest.log
grep -q "pytest rc=0$" gpurun_out/s25_pytest.log || { grep -n "Error\|assert\|FAILED" gpurun_out/s25_pytest.log | head -40; exit 3; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s25_bench.log 2>&1 && \
timeout -k 10 400 python tools/newton_trace.py --rows 10000000 > gpurun_out/s25_trace.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof25 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s25_prof.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; grep "^{" gpurun_out/s25_bench.log | head -c 1500; echo; grep -E "^(auto|s[0-9])" gpurun_out/s25_trace.log | head -20; exit $rc
