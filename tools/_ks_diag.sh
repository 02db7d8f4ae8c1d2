set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_s5e; mkdir -p $O
timeout -k 10 300 python tools/ks_check.py > $O/ks_check.jsonl 2>&1 || { tail -20 $O/ks_check.jsonl; exit 1; }
grep '^{' $O/ks_check.jsonl
timeout -k 10 400 python -u -m pytest tests/test_kernelshap.py tests/test_xai_kernel_service.py tests/test_serving_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; grep -E "passed|failed|FAILED" $O/tests.log | tail -5
timeout -k 10 200 python tools/kernelshap_bench.py --quick --skip-tree --reps 20 > $O/bench_paired.jsonl 2>&1 || exit 1
grep '^{' $O/bench_paired.jsonl
