set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s46
timeout -k 10 120 python tools/kernelshap_stamps.py > gpurun_out/s46/stamps.txt 2>&1 && \
timeout -k 10 120 python tools/kernelshap_stamps.py --link logit_model > gpurun_out/s46/stamps_logit.txt 2>&1
rc=$?
grep -hv amdgpu.ids gpurun_out/s46/stamps*.txt; exit $rc
