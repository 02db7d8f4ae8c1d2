set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/prof
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -m gpu -q > gpurun_out/s2_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s2_pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof/bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s2_bench_prof.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; tail -3 gpurun_out/s2_pytest.log; find gpurun_out/prof -name "*stats*"; exit $rc
