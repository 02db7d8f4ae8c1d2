set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_s5p; mkdir -p $O
for r in 1 2; do
for S in bf16 fp8; do
for L in 2 1; do
  FDX_NEWTON_LOOKAHEAD=$L timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-extras --storage $S > $O/b_${S}_${L}_$r.log 2>&1 || exit 1
  echo "$S lookahead=$L $(grep -o '"ms_per_step": [0-9.]*' $O/b_${S}_${L}_$r.log)"
done
done
done
