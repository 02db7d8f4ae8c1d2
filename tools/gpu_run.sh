#!/bin/bash
# One parameterised GPU-box runner (replaces the per-session scratch scripts).
#
#   gpurun --timeout 1200 -- bash tools/gpu_run.sh <tag> <stage> [<stage> ...]
#
# Stages (run in order, each under its own time limit; the first failure ends the call):
#   tests        pytest -m gpu (one process, per-test timeout)
#   tests:<expr> pytest -m gpu -k <expr>
#   smoke        __graft_entry__.smoke()
#   bench        bench.py defaults (N=1)
#   bench50      bench.py --steps 50
#   configs      tools/baseline_configs.py (every BASELINE config)
#   latency      tools/serve_latency.py
#   plots        the reference script chain (generate -> eda -> preprocess -> train -> evaluate -> explain) with its plots
#   prof         rocprofv3 --kernel-trace --stats of a short bench
#   proffp8      the same with fp8 training rows
#   marker       rocprofv3 --marker-trace --kernel-trace with the pipeline's roctx phase markers
#   benchfp8     bench.py --storage fp8
#   quick        bench.py --no-extras, bf16 then fp8 (20 steps)
#   pmc          two PMC passes over a short bench
#   ksab         KernelSHAP: accuracy vs fp64 + us per batch on three models (tools/ks_check.py), and
#                tools/kernelshap_bench.py with the paired and the unpaired kernel
#   newtonab     bench 50 steps x 3 with the Newton flag copied (event) vs polled (mapped pinned word)
#   sideab       bench 50 steps x 2: class counts on a side stream vs in front of the scaler pass
#   reserveab    bench 50 steps x 2 with 0/1/2 scaler block slots per CU reserved
#   lookab       bench 50 steps x 4: Newton flag lookahead 1 vs 2
#   ntab         kernel stats with nontemporal row stores on vs off
#   ntscab       bench 50 steps x 3: scaler row stores plain vs nontemporal
#   smoteab      SMOTE up-front gathers (FDX_SMOTE_G2) A/B: exactness tests, kernel stats, bench
#   dp2          2-rank DP rehearsal of bench.py on one GPU over gloo (both SMOTE scopes)
#   dp2self      the same rehearsal through bench.py's own launcher (python bench.py --gpus 2, no torchrun)
#   py:<script>  python <script> (extra args via FDX_PY_ARGS)
# Output lands in gpurun_out/<tag>/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=$1; shift
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
R=$GRAFT_REPO_ROOT

step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "[gpu_run] $name: $*"
  timeout -k 10 "$secs" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "[gpu_run] $name rc=$rc"
  if [ $rc -ne 0 ]; then
    tail -40 "$OUT/$name.log"
    exit $rc
  fi
  grep -h '^{' "$OUT/$name.log" | cut -c 1-600 || true
}

for st in "$@"; do
  case "$st" in
    tests) step tests 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ;;
    tests:*) step tests_k 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${st#tests:}" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    bench50) step bench50 600 python bench.py --steps 50 --warmup 5 ;;
    benchfp8) step benchfp8 600 python bench.py --storage fp8 ;;
    quick) step quick_bf16 300 python bench.py --steps 20 --warmup 3 --no-extras &&
           step quick_fp8 300 python bench.py --steps 20 --warmup 3 --no-extras --storage fp8 ;;
    configs) step configs 900 python tools/baseline_configs.py --json "$OUT/configs.json" ;;
    plots) step plots 900 python scripts/run_reference_pipeline.py --out "$OUT/plots" --kernel ;;
    latency) step latency 600 python tools/serve_latency.py --json "$OUT/latency.json" ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --steps 5 --warmup 1 --no-extras
      cd "$R" ;;
    proffp8)
      cd /tmp && export TMPDIR=/tmp
      step proffp8 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/proffp8" -o run -- python3 "$R/bench.py" --storage fp8 --steps 5 --warmup 1 --no-extras
      cd "$R" ;;
    marker)  # roctx phase markers + kernels of a short bench (FDX_ROCTX_PHASES=1)
      cd /tmp && export TMPDIR=/tmp
      export FDX_ROCTX_PHASES=1
      step marker 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d "$OUT/marker" -o run -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-extras
      unset FDX_ROCTX_PHASES
      cd "$R" ;;
    pmc)
      cd /tmp && export TMPDIR=/tmp
      step pmc_a 120 rocprofv3 --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU --output-format csv -d "$OUT/pmc_a" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras
      step pmc_b 120 rocprofv3 --pmc WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY --output-format csv -d "$OUT/pmc_b" -o run -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-extras
      cd "$R" ;;
    pmcks)  # KernelSHAP linear kernel counters (3 passes, 1000-explanation batches)
      cd /tmp && export TMPDIR=/tmp
      KS="python3 $R/tools/kernelshap_bench.py --quick --skip-tree --reps 5"
      step pmcks_a 120 rocprofv3 --kernel-include-regex "kernelshap_(linear|paired)" --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$OUT/pmcks_a" -o run -- $KS
      step pmcks_b 120 rocprofv3 --kernel-include-regex "kernelshap_(linear|paired)" --pmc SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmcks_b" -o run -- $KS
      step pmcks_t 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmcks_t" -o run -- $KS
      cd "$R" ;;
    ksab)
      step ks_check 300 python tools/ks_check.py
      for P in 1 0; do
        FDX_KS_PAIRED=$P step ks_bench_paired$P 200 python tools/kernelshap_bench.py --quick --skip-tree --reps 20
      done ;;
    newtonab)
      for r in 1 2 3; do for F in copy map; do
        FDX_NEWTON_FLAG=$F step newton_${F}_$r 300 python bench.py --steps 50 --warmup 5 --no-extras
      done; done ;;
    sideab)  # class-count kernels on a side stream beside the fused scaler pass vs in front of it
      for i in 1 2; do
        FDX_COUNT_SIDE=0 step "sideab_front_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras &&
        FDX_COUNT_SIDE=1 step "sideab_side_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras || exit 1
      done ;;
    reserveab)  # fused scaler pass grid: 0 / 1 / 2 block slots per CU left free for the side-stream count
      for i in 1 2; do
        for r in 0 1 2; do
          FDX_SCALER_RESERVE=$r step "reserve${r}_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras || exit 1
        done
      done ;;
    lookab)  # Newton convergence-flag lookahead 1 vs 2 (single GPU), 50-step benches interleaved x4
      for i in 1 2 3 4; do
        for la in 1 2; do
          FDX_NEWTON_LOOKAHEAD=$la step "look${la}_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras || exit 1
        done
      done ;;
    ntab)  # kernel stats with nontemporal row-stream stores on vs off (scaler pass + SMOTE output)
      cd /tmp && export TMPDIR=/tmp
      FDX_NT_STORES=1 step ntab_on 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nt_on" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-extras &&
      FDX_NT_STORES=0 step ntab_off 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nt_off" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-extras || exit 1
      cd "$R" ;;
    ntscab)  # fused scaler pass row stores: plain (default) vs nontemporal, 50-step benches interleaved x3
      for i in 1 2 3; do
        FDX_NT_SCALER=0 step "ntsc0_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras &&
        FDX_NT_SCALER=1 step "ntsc1_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras || exit 1
      done ;;
    smoteab)  # SMOTE: both halves' gathers up front (FDX_SMOTE_G2=1) vs per half; exactness tests under G2, kernel stats, bench x2
      FDX_SMOTE_G2=1 step smoteab_tests 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "smote or pipeline or back_to_back" &&
      cd /tmp && export TMPDIR=/tmp &&
      FDX_SMOTE_G2=0 step smoteab_prof0 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g2_0" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-extras &&
      FDX_SMOTE_G2=1 step smoteab_prof1 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/g2_1" -o run -- python3 "$R/bench.py" --steps 10 --warmup 2 --no-extras &&
      cd "$R" || exit 1
      for i in 1 2; do
        FDX_SMOTE_G2=0 step "g2off_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras &&
        FDX_SMOTE_G2=1 step "g2on_$i" 300 python bench.py --steps 50 --warmup 5 --no-extras || exit 1
      done ;;
    dp2)  # DP rehearsal on one GPU: 2 ranks over host-staged gloo (the RCCL path needs a GPU per rank)
      step dp2 300 env FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
        --rows-per-gpu 2000000 ;;
    dp2self)  # bench.py --gpus 2 starts its own 2 ranks (self-launch path), one GPU, gloo
      step dp2self 300 env FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 3 --warmup 1 \
        --rows-per-gpu 2000000 ;;
    py:*) # shellcheck disable=SC2086
      s=${st#py:}; step "py_$(basename "$s" .py)" 600 python -u "$s" $FDX_PY_ARGS ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "[gpu_run] all stages ok"
