set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/s19_counters.txt 2>&1; echo "list rc=$?"
grep -o "SQ_[A-Z0-9_]*" $GRAFT_REPO_ROOT/gpurun_out/s19_counters.txt | sort -u > $GRAFT_REPO_ROOT/gpurun_out/s19_sq.txt
for C in "SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY"; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc19 -o run -- python3 $GRAFT_REPO_ROOT/tools/ubench.py --only knn_topk_13600 --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/s19_pmc.log 2>&1; echo "pmc rc=$?"
done
wc -l $GRAFT_REPO_ROOT/gpurun_out/s19_sq.txt
