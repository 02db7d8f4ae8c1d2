set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/s9_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s9_pytest.log
timeout -k 10 300 python tools/ubench.py --json gpurun_out/s9_ubench.json > gpurun_out/s9_ubench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s9_bench.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof9 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s9_prof.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; tail -4 gpurun_out/s9_pytest.log; cat gpurun_out/s9_ubench.log; tail -c 1600 gpurun_out/s9_bench.log; exit $rc
