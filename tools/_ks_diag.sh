set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_s5k; mkdir -p $O
for P in 1 0; do
  FDX_KS_PAIRED=$P timeout -k 10 200 python tools/kernelshap_bench.py --quick --skip-tree --reps 20 > $O/bench_$P.jsonl 2>&1 || exit 1
  grep '^{' $O/bench_$P.jsonl | cut -c1-200
done
timeout -k 10 300 python tools/ks_check.py > $O/ks_check.jsonl 2>&1 || { tail -20 $O/ks_check.jsonl; exit 1; }
grep '^{' $O/ks_check.jsonl | cut -c1-180
for P in 1 0; do
  FDX_KS_PAIRED=$P timeout -k 10 400 python -u -m pytest tests/test_kernelshap.py tests/test_xai_kernel_service.py tests/test_serving_gpu.py -m gpu -v --timeout 120 --timeout-method thread > $O/tests_$P.log 2>&1; grep -E "passed|failed|FAILED" $O/tests_$P.log | tail -4
done
