set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2_s5h; mkdir -p $O
timeout -k 10 300 python tools/ks_check.py > $O/ks_check.jsonl 2>&1 || { tail -20 $O/ks_check.jsonl; exit 1; }
grep '^{' $O/ks_check.jsonl
