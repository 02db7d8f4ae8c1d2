set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
mkdir -p gpurun_out/s37
timeout -k 10 300 python tools/ubench.py --only logreg_pass_grad_2n,logreg_pass_virtual_grad_2n,logreg_pass_virtual_grad_2n_sorted,logreg_pass_virtual_hess_s3_2n,logreg_pass_virtual_hess_s3_2n_sorted,smote_plan_n,smote_generate_n > gpurun_out/s37/ubench.txt 2>&1
rc=$?
grep " us" gpurun_out/s37/ubench.txt; tail -3 gpurun_out/s37/ubench.txt; exit $rc
