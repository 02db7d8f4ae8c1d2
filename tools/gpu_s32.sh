set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s32
timeout -k 10 600 python tools/baseline_configs.py --json gpurun_out/s32/configs.json > gpurun_out/s32/configs.log 2>&1 && \
timeout -k 10 300 python tools/ubench.py --json gpurun_out/s32/ubench.json > gpurun_out/s32/ubench.txt 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s32/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s32/prof.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE SQ_WAVES SQ_INSTS_VALU_MFMA_MOPS_BF16 --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/s32/pmc1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s32/pmc1.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT; grep -v amdgpu.ids gpurun_out/s32/configs.log; grep " us" gpurun_out/s32/ubench.txt | head -40; exit $rc
