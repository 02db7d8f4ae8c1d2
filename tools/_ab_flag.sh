set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_s5o; mkdir -p $O
for r in 1 2 3; do
for F in copy map; do
  FDX_NEWTON_FLAG=$F timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-extras > $O/b_${F}_$r.log 2>&1 || exit 1
  echo "$F $(grep -o '"ms_per_step": [0-9.]*' $O/b_${F}_$r.log)"
done
done
