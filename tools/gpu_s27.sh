set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/s27_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s27_pytest.log
tail -3 gpurun_out/s27_pytest.log
grep -q "pytest rc=0$" gpurun_out/s27_pytest.log || { grep -n "Error\|assert\|FAILED" gpurun_out/s27_pytest.log | head -40; exit 3; }
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s27_bench.log 2>&1 && \
FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --rows-per-gpu 4000000 > gpurun_out/s27_bench_dp2_gloo.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof27 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s27_prof.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; grep -h "^{" gpurun_out/s27_bench.log gpurun_out/s27_bench_dp2_gloo.log | cut -c 1-400; tail -5 gpurun_out/s27_bench_dp2_gloo.log; exit $rc
