set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/r2_i
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --storage fp8 --no-extras > gpurun_out/r2_i/bench_fp8.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_i/prof_fp8 -o run -- python3 $R/bench.py --storage fp8 --steps 5 --warmup 1 --no-extras > $R/gpurun_out/r2_i/prof_fp8.log 2>&1 || exit 2
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r2_i/prof_bf16 -o run -- python3 $R/bench.py --steps 5 --warmup 1 --no-extras > $R/gpurun_out/r2_i/prof_bf16.log 2>&1 || exit 3
