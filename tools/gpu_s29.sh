set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python tools/baseline_configs.py --json gpurun_out/s29_configs.json > gpurun_out/s29_configs.log 2>&1
rc=$?
cat gpurun_out/s29_configs.log | grep -v amdgpu.ids; exit $rc
