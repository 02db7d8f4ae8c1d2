set -o pipefail
cd $GRAFT_REPO_ROOT
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/s21_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/s21_pytest.log
tail -3 gpurun_out/s21_pytest.log
grep -q "pytest rc=[01]$" gpurun_out/s21_pytest.log || exit 3
timeout -k 10 300 python tools/ubench.py --json gpurun_out/s21_ubench.json > gpurun_out/s21_ubench.log 2>&1 && \
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/s21_bench.log 2>&1 && \
FDX_GBDT_GRAPH=0 timeout -k 10 300 python tools/gbdt_bench.py --rows 4000000 > gpurun_out/s21_gbdt_eager.log 2>&1 && \
timeout -k 10 300 python tools/gbdt_bench.py --rows 4000000 > gpurun_out/s21_gbdt_graph.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof21 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --no-extras > $GRAFT_REPO_ROOT/gpurun_out/s21_prof.log 2>&1
rc=$?
cd /tmp && timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc21 -o run -- python3 $GRAFT_REPO_ROOT/tools/ubench.py --only knn_topk_13600,smote_generate_n,newton_update --reps 3 > $GRAFT_REPO_ROOT/gpurun_out/s21_pmc.log 2>&1; echo "pmc rc=$?" >> $GRAFT_REPO_ROOT/gpurun_out/s21_pmc.log
cd $GRAFT_REPO_ROOT; cat gpurun_out/s21_ubench.log; tail -c 1500 gpurun_out/s21_bench.log; tail -3 gpurun_out/s21_pmc.log; tail -1 gpurun_out/s21_gbdt_eager.log gpurun_out/s21_gbdt_graph.log; exit $rc
