set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s38
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $R/gpurun_out/s38/counters_list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD --output-format csv -d $R/gpurun_out/s38/p1 -o run -- python3 $R/tools/pass_probe.py > $R/gpurun_out/s38/p1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/s38/p2 -o run -- python3 $R/tools/pass_probe.py > $R/gpurun_out/s38/p2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d $R/gpurun_out/s38/p3 -o run -- python3 $R/tools/pass_probe.py > $R/gpurun_out/s38/p3.log 2>&1
rc=$?
cd $R; tail -2 gpurun_out/s38/p*.log; exit $rc
