set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s40
timeout -k 10 120 python tools/newton_stamps.py > gpurun_out/s40/stamps.txt 2>&1 && \
timeout -k 10 300 python tools/ubench.py --only newton_update,logreg_reduce,smote_generate_n_bf16_parents,write_only_fill_n_rows > gpurun_out/s40/ubench.txt 2>&1
rc=$?
cat gpurun_out/s40/stamps.txt | grep -v amdgpu.ids; grep " us" gpurun_out/s40/ubench.txt; exit $rc
