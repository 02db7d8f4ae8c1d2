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
#   ubench       tools/ubench.py per-kernel event timings
#   schedlab     tools/sched_lab.py: Newton warm-up schedules on the virtual-SMOTE bench fit
#   passlab      tools/pass_lab.py: solver pass / reduce / update launches and whole fits at the bench shape
#   latency      tools/serve_latency.py
#   plots        the reference script chain (generate -> eda -> preprocess -> train -> evaluate -> explain) with its plots
#   prof         rocprofv3 --kernel-trace --stats of a short Newton bench + its one-step timeline
#   proffp8      the same with fp8 training rows
#   profsgd      kernel trace + one-step timeline of the SGD fit
#   marker       rocprofv3 --marker-trace --kernel-trace with the pipeline's roctx phase markers
#   benchfp8     bench.py --storage fp8
#   quick        bench.py --solver newton --no-extras, bf16 then fp8 (20 steps); quickfuse: fused Newton iterations (FDX_NEWTON_FUSE=1); proffuse: their trace
#   quicksgd     the same with the SGD solver
#   quicksgdnc   quicksgd bf16 with the cooperative persistent launch (FDX_SGD_COOP=1)
#   pmc          two PMC passes over a short bench
#   pmcfp8       logreg pass counters + kernel stats with fp8 and with bf16 rows
#   gbdt         tools/gbdt_bench.py at the bench shape; gbdtprof: its kernel trace (20 trees)
#   dp2          2-rank DP rehearsal of bench.py on one GPU over gloo (both SMOTE scopes)
#   dp2self      the same rehearsal through bench.py's own launcher (python bench.py --gpus 2, no torchrun)
#   dpscope      tools/dp_scope_probe.py: global vs shard SMOTE scope attribution (2 ranks, one GPU, gloo)
#   gbdtvar      GBDT histogram kernel variants under a kernel trace (FDX_GBDT_VARS, default "0 3")
#   dpstored     dp_scope_probe.py on stored SMOTE rows (bf16 and fp8), per-phase times of each synced fit
#   stall        tools/stall_probe.py: 2 ranks on one GPU under rocprofv3 markers + kernel trace, stall attribution
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
    quicksgd) step quicksgd_bf16 300 python bench.py --steps 20 --warmup 3 --no-extras --solver sgd &&
           step quicksgd_fp8 300 python bench.py --steps 20 --warmup 3 --no-extras --solver sgd --storage fp8 ;;
    smoteov)  # the virtual-SMOTE bucket sort beside the scaler pass / beside the k-NN / in line (quick SGD benches)
      step smoteov_scaler 300 env FDX_SMOTE_OVERLAP=scaler python bench.py --steps 30 --warmup 3 --no-extras &&
      step smoteov_knn 300 env FDX_SMOTE_OVERLAP=knn python bench.py --steps 30 --warmup 3 --no-extras &&
      step smoteov_off 300 env FDX_SMOTE_OVERLAP=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step smoteov_scaler2 300 env FDX_SMOTE_OVERLAP=scaler python bench.py --steps 30 --warmup 3 --no-extras &&
      step smoteov_scaler_hi 300 env FDX_SMOTE_OVERLAP=scaler FDX_SMOTE_SIDE_PRIO=-1 python bench.py --steps 30 --warmup 3 --no-extras ;;
    sortpoll)  # host-polled bucket-sort completion (default) vs the cross-stream wait, alternating
      step sortpoll_on1 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step sortpoll_off1 300 env FDX_SORT_POLL_US=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step sortpoll_on2 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step sortpoll_off2 300 env FDX_SORT_POLL_US=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step sortpoll_on3 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step sortpoll_off3 300 env FDX_SORT_POLL_US=0 python bench.py --steps 30 --warmup 3 --no-extras ;;
    benchclk)  # per-fit boundaries from the device clock in the exports (default) vs events behind every fit
      step benchclk_c1 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step benchclk_e1 300 env FDX_BENCH_EVENTS=1 python bench.py --steps 30 --warmup 3 --no-extras &&
      step benchclk_c2 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step benchclk_e2 300 env FDX_BENCH_EVENTS=1 python bench.py --steps 30 --warmup 3 --no-extras &&
      step benchclk_c3 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step benchclk_e3 300 env FDX_BENCH_EVENTS=1 python bench.py --steps 30 --warmup 3 --no-extras ;;
    cgather)  # minority rows gathered by the index-list launch (default) vs a scale_cast launch behind it
      step cgather_on1 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step cgather_off1 300 env FDX_COMPACT_GATHER=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step cgather_on2 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step cgather_off2 300 env FDX_COMPACT_GATHER=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step cgather_on3 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step cgather_off3 300 env FDX_COMPACT_GATHER=0 python bench.py --steps 30 --warmup 3 --no-extras ;;
    quicksgdnc) step quicksgd_coop 300 env FDX_SGD_COOP=1 python bench.py --steps 20 --warmup 3 --no-extras --solver sgd ;;
    evab)  # per-fit timing events and the side-stream export, on / off (quick SGD bench each)
      step evab_default 300 python bench.py --steps 30 --warmup 3 --no-extras &&
      step evab_noev 300 env FDX_BENCH_EVENTS=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step evab_noside 300 env FDX_EXPORT_SIDE=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step evab_noev_noside 300 env FDX_BENCH_EVENTS=0 FDX_EXPORT_SIDE=0 python bench.py --steps 30 --warmup 3 --no-extras &&
      step evab_default2 300 python bench.py --steps 30 --warmup 3 --no-extras ;;
    stall)  # 2-rank one-GPU rehearsal under a marker + kernel trace: attribute the intermittent fit stall
      cd /tmp && export TMPDIR=/tmp FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo
      step stall 400 rocprofv3 --marker-trace --kernel-trace --output-format csv -d "$OUT/stall" -o run -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29523 "$R/tools/stall_probe.py" --fits 12
      unset FDX_BENCH_ONE_GPU FDX_BENCH_BACKEND
      cd "$R"
      python tools/stall_probe.py --analyze "$OUT/stall" --json "$OUT/stall_attribution.json" > "$OUT/stall_analyze.log" 2>&1 || true ;;
    quick) step quick_bf16 300 python bench.py --steps 20 --warmup 3 --no-extras --solver newton &&
           step quick_fp8 300 python bench.py --steps 20 --warmup 3 --no-extras --solver newton --storage fp8 ;;
    quickfuse)  # the Newton iteration fused into the pass launch (FDX_NEWTON_FUSE=1)
      step quickfuse_bf16 300 env FDX_NEWTON_FUSE=1 python bench.py --steps 20 --warmup 3 --no-extras --solver newton &&
      step quickfuse_fp8 300 env FDX_NEWTON_FUSE=1 python bench.py --steps 20 --warmup 3 --no-extras --solver newton --storage fp8 ;;
    proffuse)  # kernel trace + timeline of the fused Newton iteration
      cd /tmp && export TMPDIR=/tmp FDX_NEWTON_FUSE=1
      step proffuse 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/proffuse" -o run -- python3 "$R/bench.py" --solver newton --steps 5 --warmup 1 --no-extras
      unset FDX_NEWTON_FUSE
      cd "$R"
      python tools/timeline.py "$OUT/proffuse/run_kernel_trace.csv" > "$OUT/timeline_newton_fused_step.txt" 2>&1 || true ;;
    schedlab) step schedlab 400 python tools/sched_lab.py --json "$OUT/sched_lab.json" ;;
    knnprof)  # kernel trace of the k-NN lab (engines/splits from FDX_KNN_ARGS)
      cd /tmp && export TMPDIR=/tmp
      # shellcheck disable=SC2086
      step knnprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/knnprof" -o run -- python3 "$R/tools/knn_lab.py" --reps 5 $FDX_KNN_ARGS
      cd "$R" ;;
    pmcknn)  # bf16x3r collect / rerank counters (FDX_KNN_ARGS picks engines and splits)
      cd /tmp && export TMPDIR=/tmp
      # shellcheck disable=SC2086
      step pmcknn_a 180 rocprofv3 --kernel-include-regex "knn_(collect|rerank|topk_kernel|b3top)" --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM SQ_INSTS_SALU --output-format csv -d "$OUT/pmcknn_a" -o run -- python3 "$R/tools/knn_lab.py" --reps 3 $FDX_KNN_ARGS || exit 1
      # shellcheck disable=SC2086
      step pmcknn_b 180 rocprofv3 --kernel-include-regex "knn_(collect|rerank|topk_kernel|b3top)" --pmc SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY --output-format csv -d "$OUT/pmcknn_b" -o run -- python3 "$R/tools/knn_lab.py" --reps 3 $FDX_KNN_ARGS
      cd "$R" ;;
    knndepth)  # bf16x3r collect: 2 vs 4 candidate tiles in flight (FDX_KNN3R_DEPTH), lab at DP1 / DP8 shapes
      step knndepth_4 300 env FDX_KNN3R_DEPTH=4 python tools/knn_lab.py --engines bf16x3r --splits 2,4,8 --json "$OUT/knndepth_4.json" &&
      step knndepth_2 300 env FDX_KNN3R_DEPTH=2 python tools/knn_lab.py --engines bf16x3r --splits 2,4,8 --json "$OUT/knndepth_2.json" ;;
    knnab)  # the pipeline's k-NN engine at DP1: bf16x3r vs the fp32 default (quick SGD benches, twice each)
      step knnab_3r 300 env FDX_KNN=bf16x3r python bench.py --steps 30 --warmup 3 --no-extras &&
      step knnab_fp32 300 env FDX_KNN=fp32 python bench.py --steps 30 --warmup 3 --no-extras &&
      step knnab_3r_b 300 env FDX_KNN=bf16x3r python bench.py --steps 30 --warmup 3 --no-extras &&
      step knnab_fp32_b 300 env FDX_KNN=fp32 python bench.py --steps 30 --warmup 3 --no-extras ;;
    knnquad)  # fp32 and bf16x3r engines around their default splits (append-path A/Bs)
      step knnquad 300 python tools/knn_lab.py --engines fp32,bf16x3r --splits 4,16,19 --json "$OUT/knnquad.json" ;;
    knnlab) step knnlab 400 python tools/knn_lab.py --json "$OUT/knn_lab.json" $FDX_KNN_ARGS ;;  # shellcheck disable=SC2086
    passlab) step passlab 300 python tools/pass_lab.py --json "$OUT/pass_lab.json" ;;
    ubench) step ubench 300 python tools/ubench.py --json "$OUT/ubench.json" ;;
    configs) step configs 900 python tools/baseline_configs.py --json "$OUT/configs.json" ;;
    plots) step plots 900 python scripts/run_reference_pipeline.py --out "$OUT/plots" --kernel ;;
    latency) step latency 600 python tools/serve_latency.py --json "$OUT/latency.json" ;;
    prof)
      cd /tmp && export TMPDIR=/tmp
      step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python3 "$R/bench.py" --solver newton --steps 5 --warmup 1 --no-extras
      cd "$R"
      python tools/timeline.py "$OUT/prof/run_kernel_trace.csv" > "$OUT/timeline_newton_step.txt" 2>&1 || true ;;
    profsgd)  # kernel trace of the SGD fit (config 3's solver)
      cd /tmp && export TMPDIR=/tmp
      step profsgd 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/profsgd" -o run -- python3 "$R/bench.py" --solver sgd --steps 5 --warmup 1 --no-extras
      cd "$R"
      python tools/timeline.py "$OUT/profsgd/run_kernel_trace.csv" > "$OUT/timeline_sgd_step.txt" 2>&1 || true ;;
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
    pmcfp8)  # logreg pass counters, fp8 vs bf16 rows (decode-VALU vs HBM question)
      cd /tmp && export TMPDIR=/tmp
      for ST in fp8 bf16; do
        step "pmc_pass_$ST" 120 rocprofv3 --kernel-include-regex "logreg_pass" --pmc FETCH_SIZE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD --output-format csv -d "$OUT/pmc_pass_$ST" -o run -- python3 "$R/bench.py" --storage $ST --steps 2 --warmup 1 --no-extras || exit 1
        step "pmc_pass_t_$ST" 120 rocprofv3 --kernel-include-regex "logreg_pass" --kernel-trace --stats --output-format csv -d "$OUT/pmc_pass_t_$ST" -o run -- python3 "$R/bench.py" --storage $ST --steps 2 --warmup 1 --no-extras || exit 1
      done
      cd "$R" ;;
    gbdt)  # GBDT: 100-tree bench at the bench shape (10M raw rows -> 16M post-SMOTE)
      step gbdt 300 python tools/gbdt_bench.py --rows 10000000 --json "$OUT/gbdt.json" ;;
    hostprof) step hostprof 300 python tools/host_profile.py --steps 30 ;;
    hostprofn) step hostprof_newton 300 python tools/host_profile.py --steps 30 --solver newton ;;
    gapprobe)  # idle gap after kernels that store to mapped pinned memory
      cd /tmp && export TMPDIR=/tmp
      step gapprobe 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/gapprobe" -o run -- python3 "$R/tools/gap_probe.py"
      cd "$R"
      python tools/gap_probe.py --report "$OUT/gapprobe/run_kernel_trace.csv" > "$OUT/gap_probe.txt" 2>&1 || true ;;
    cvhost) step cvhost 300 python tools/cv_probe.py --host-profile ;;
    cvprof)  # kernel trace + timeline of one device CV job (anchor: its gathered scaler pass)
      cd /tmp && export TMPDIR=/tmp
      step cvprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/cvprof" -o run -- python3 "$R/tools/cv_probe.py" --runs 3
      cd "$R"
      python tools/timeline.py "$OUT/cvprof/run_kernel_trace.csv" --anchor "scaler_stats_cast_kernel<false, false, true>" > "$OUT/timeline_cv_job.txt" 2>&1 || true ;;
    gbdtprof)  # GBDT round kernel trace (20 trees at the bench shape)
      cd /tmp && export TMPDIR=/tmp
      step gbdtprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gbdtprof" -o run -- python3 "$R/tools/gbdt_bench.py" --rows 10000000 --trees 20
      cd "$R" ;;
    pmcgbdt)  # GBDT histogram kernel counters (LDS atomics: bank / address conflicts), 10 trees at the bench shape
      cd /tmp && export TMPDIR=/tmp
      GB="python3 $R/tools/gbdt_bench.py --rows 10000000 --trees 10"
      step pmcgbdt_a 180 rocprofv3 --kernel-include-regex "gbdt_hist_kernel" --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM --output-format csv -d "$OUT/pmcgbdt_a" -o run -- $GB
      step pmcgbdt_b 180 rocprofv3 --kernel-include-regex "gbdt_hist_kernel" --pmc SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS --output-format csv -d "$OUT/pmcgbdt_b" -o run -- $GB
      step pmcgbdt_t 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmcgbdt_t" -o run -- $GB
      cd "$R" ;;
    gbdtvar)  # GBDT histogram variants (0 lockstep, 2 split g/h int32 adds, 1 rotated): kernel stats, 10 trees
      cd /tmp && export TMPDIR=/tmp
      for V in ${FDX_GBDT_VARS:-0 3}; do
        export FDX_GBDT_HIST_VAR=$V
        step "gbdtvar_$V" 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/gbdtvar_$V" -o run -- python3 "$R/tools/gbdt_bench.py" --rows 10000000 --trees 10 || exit 1
      done
      unset FDX_GBDT_HIST_VAR
      cd "$R" ;;
    pmcks)  # KernelSHAP linear kernel counters (3 passes, 1000-explanation batches)
      cd /tmp && export TMPDIR=/tmp
      KS="python3 $R/tools/kernelshap_bench.py --quick --skip-tree --reps 5"
      step pmcks_a 120 rocprofv3 --kernel-include-regex "kernelshap_(linear|paired)" --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS --output-format csv -d "$OUT/pmcks_a" -o run -- $KS
      step pmcks_b 120 rocprofv3 --kernel-include-regex "kernelshap_(linear|paired)" --pmc SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$OUT/pmcks_b" -o run -- $KS
      step pmcks_t 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/pmcks_t" -o run -- $KS
      cd "$R" ;;
    dp2)  # DP rehearsal on one GPU: 2 ranks over host-staged gloo (the RCCL path needs a GPU per rank)
      step dp2 300 env FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 \
        --rows-per-gpu 2000000 ;;
    dp2self)  # bench.py --gpus 2 starts its own 2 ranks (self-launch path), one GPU, gloo
      step dp2self 300 env FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo python bench.py --gpus 2 --steps 3 --warmup 1 \
        --rows-per-gpu 2000000 ;;
    dpscope)  # global vs shard SMOTE scope attribution (2 ranks, one GPU, gloo): per-fit times, phases, host profile
      step dpscope 400 env FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29519 tools/dp_scope_probe.py --rows 2000000 ;;
    dpstored)  # stored-SMOTE fits at global scope (2 ranks, one GPU, gloo): per-phase times of every synced fit
      for ST in bf16 fp8; do
        step "dpstored_$ST" 300 env FDX_BENCH_ONE_GPU=1 FDX_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 \
          --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29521 tools/dp_scope_probe.py --rows 2000000 \
          --scopes global,shard --storage $ST --smote-virtual 0 --phases 1 --fits 6 || exit 1
      done ;;
    py:*) # shellcheck disable=SC2086
      s=${st#py:}; step "py_$(basename "$s" .py)" 600 python -u "$s" $FDX_PY_ARGS ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo "[gpu_run] all stages ok"
