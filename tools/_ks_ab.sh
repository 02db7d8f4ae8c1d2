set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_s5b; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernelshap.py tests/test_xai_kernel_service.py tests/test_serving_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -2
FDX_KS_PAIRED=0 timeout -k 10 200 python tools/kernelshap_bench.py --quick --skip-tree --reps 20 > $O/bench_unpaired.jsonl 2>&1 || exit 1
FDX_KS_PAIRED=1 timeout -k 10 200 python tools/kernelshap_bench.py --quick --skip-tree --reps 20 > $O/bench_paired.jsonl 2>&1 || exit 1
cut -c1-300 $O/bench_unpaired.jsonl $O/bench_paired.jsonl
timeout -k 10 300 python tools/ks_check.py > $O/ks_check.jsonl 2>&1 || { tail -20 $O/ks_check.jsonl; exit 1; }
grep '^{' $O/ks_check.jsonl
