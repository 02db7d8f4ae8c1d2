set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s49
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/s49/pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s49/pytest.log
tail -3 gpurun_out/s49/pytest.log
grep -q "pytest rc=0$" gpurun_out/s49/pytest.log || { grep -n "Error\|assert\|FAILED\|^E " gpurun_out/s49/pytest.log | head -40; exit 3; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s49/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py > gpurun_out/s49/bench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 50 --warmup 5 > gpurun_out/s49/bench50.log 2>&1 && \
FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --rows-per-gpu 4000000 > gpurun_out/s49/bench_dp2_gloo.log 2>&1 && \
timeout -k 10 600 python tools/baseline_configs.py --json gpurun_out/s49/configs.json > gpurun_out/s49/configs.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s49/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s49/prof.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s49/pmc_fetch -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s49/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s49/pmc_write -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s49/pmc_write.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; tail -1 gpurun_out/s49/smoke.log; grep -h "^{" gpurun_out/s49/bench.log gpurun_out/s49/bench50.log gpurun_out/s49/bench_dp2_gloo.log | cut -c 1-420; grep -v amdgpu gpurun_out/s49/configs.log | cut -c 1-300; exit $rc
