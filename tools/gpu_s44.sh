set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s44
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/s44/kt -o run -- python3 $R/tools/mfma_probe.py > $R/gpurun_out/s44/kt.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY --output-format csv -d $R/gpurun_out/s44/p1 -o run -- python3 $R/tools/mfma_probe.py > $R/gpurun_out/s44/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA --output-format csv -d $R/gpurun_out/s44/p2 -o run -- python3 $R/tools/mfma_probe.py > $R/gpurun_out/s44/p2.log 2>&1
rc=$?
cd $R; tail -n 2 gpurun_out/s44/p1.log gpurun_out/s44/p2.log; exit $rc
