set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/s28_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s28_pytest.log
tail -3 gpurun_out/s28_pytest.log
grep -q "pytest rc=0$" gpurun_out/s28_pytest.log || { grep -n "Error\|assert\|FAILED" gpurun_out/s28_pytest.log | head -40; exit 3; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s28_bench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 5 --no-extras > gpurun_out/s28_bench50.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof28 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s28_prof.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; grep -h "^{" gpurun_out/s28_bench.log gpurun_out/s28_bench50.log | cut -c 1-400; exit $rc
