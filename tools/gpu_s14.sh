set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/s14_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s14_pytest.log
tail -3 gpurun_out/s14_pytest.log
grep -q "pytest rc=[01]$" gpurun_out/s14_pytest.log || exit 3
timeout -k 10 300 python tools/ubench.py --json gpurun_out/s14_ubench.json > gpurun_out/s14_ubench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s14_bench.log 2>&1 && timeout -k 10 300 python tools/gbdt_bench.py --rows 10000000 --json gpurun_out/s14_gbdt.json > gpurun_out/s14_gbdt.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof14 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s14_prof.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof14g -o run -- python3 $GRAFT_REPO_ROOT/tools/gbdt_bench.py --rows 10000000 --trees 100 > $GRAFT_REPO_ROOT/gpurun_out/s14_profg.log 2>&1
rc=$?; cd $GRAFT_REPO_ROOT; cat gpurun_out/s14_ubench.log; tail -c 1500 gpurun_out/s14_bench.log; tail -2 gpurun_out/s14_profg.log; exit $rc
