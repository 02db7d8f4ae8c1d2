// Host-side launch entry points for every HIP kernel in fraud_detection_amd.
// Each launcher enqueues on the caller's hipStream_t (torch's current stream when called from
// Python) and throws std::runtime_error on a launch error.  No allocation, no synchronisation:
// every launcher is safe to capture into a hipGraph (cdna_hip_programming.md Guideline 9).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>
#include <stdexcept>
#include <string>

namespace fdx {

// FDX_SYNC_LAUNCH=1: synchronise after every launch so an asynchronous fault is reported with
// the name of the kernel that caused it (debug mode, like AMD_SERIALIZE_KERNEL=3 but attributed).
// Store policy of the big write-once outputs, fixed by measurement (the A/B switches are gone):
// SMOTE rows use streaming (nontemporal) stores -- the output stream no longer evicts the
// L2-resident parent rows (SMOTE 164 -> 150 us, profiles/r1_s26; 122 vs 127 us on the current
// kernel, profiles/r2_s6) -- while the fused scaler pass's rows use plain stores (269 us plain vs
// 280 us nontemporal, profiles/r2_s6/nt_stores_ab.txt).

inline bool sync_launch_mode() {
  static const int mode = [] {
    const char* v = std::getenv("FDX_SYNC_LAUNCH");
    return (v != nullptr && v[0] != '\0' && v[0] != '0') ? 1 : 0;
  }();
  return mode != 0;
}

inline void check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e == hipSuccess && sync_launch_mode()) e = hipDeviceSynchronize();
  if (e != hipSuccess) {
    throw std::runtime_error(std::string("fdx kernel launch failed [") + what +
                             "]: " + hipGetErrorString(e));
  }
}

// ---- scaler.hip ----
void launch_scaler_partial(const float* X, int64_t n, int ld, int d, const float* pivot,
                           double* partial, int nblocks, hipStream_t stream);
int scaler_reduce_scratch_rows(int nblocks);  // extra [64] rows launch_scaler_reduce needs after the partials
void launch_scaler_reduce(const double* partial, int nblocks, double* sums, hipStream_t stream);
int launch_scaler_reduce_level1(const double* partial, int nblocks, double* mid, hipStream_t stream);
void launch_scaler_finalize(const double* sums, double n, const float* pivot, int d,
                            double* mean64, double* var64, double* scale64, float* mean32,
                            float* inv32, double* aff, hipStream_t stream,
                            const float* colscale = nullptr, int nparts = 1);
void launch_fp8_hw_check(float* dec, const float* vals, int n, uint8_t* enc, hipStream_t stream);
int fp8_prescale_blocks();  // partial rows ([n][64] fp64) launch_fp8_prescale needs
void launch_fp8_prescale(const float* X, int64_t n, int d, int64_t ns, int64_t stride, double* partial,
                         double* sums, float* mu, float* k, hipStream_t stream);
int scaler_stats_cast_blocks(int fp8 = 0);  // resident blocks of the fused kernel (per row format)
// fused K1+K2: shifted sums -> partial[nblocks][64], rows s = x - pivot in bf16, or (colscale set)
// fp8 e4m3 of (x - pivot) * colscale * out_scale
void launch_scaler_stats_cast(const float* X, int64_t n, int d, const float* pivot, const uint8_t* labels,
                              float bias_value, void* out, double* partial, int nblocks, hipStream_t stream,
                              const float* colscale = nullptr, float out_scale = 1.0f,
                              const int64_t* idx = nullptr);
void launch_scale_cast(const float* X, int64_t n, int ld, int d, const int64_t* idx,
                       const float* mean32, const float* inv32, const uint8_t* labels,
                       float bias_value, float out_scale, int out_kind, void* out,
                       hipStream_t stream);
void launch_compact_count(const uint8_t* labels, int64_t n, int target, int64_t* counts,
                          int nblocks, hipStream_t stream);
void launch_exclusive_scan_small(int64_t* a, int n, int64_t* total, hipStream_t stream,
                                 int64_t* host_total = nullptr);
void launch_compact_write(const uint8_t* labels, int64_t n, int target, const int64_t* offsets,
                          int64_t* out_idx, int nblocks, hipStream_t stream);
// K3 stratified split/fold codes (split.hip): 255 = test, 0..k-1 = fold; offsets/total from
// compact_count(target=1) + exclusive_scan_small over the same nblocks.
void launch_strat_assign(const uint8_t* labels, int64_t n, const int64_t* offsets, const int64_t* total,
                         uint32_t seed, double test_frac, int k, uint8_t* out, int nblocks, hipStream_t stream);

// ---- predict.hip ----
void launch_predict_bf16(const uint16_t* X, int64_t n, const float* w, float* prob, float* logit,
                         hipStream_t stream);
void launch_predict_fp8(const uint8_t* X, int64_t n, const float* w, float* prob, float* logit,
                        hipStream_t stream);
// Fused predict + linear SHAP.  in_kind: 0 = bf16 [n][32], 1 = raw fp32 [n][ld].
// z = sum_{j<dz} a_j x_j + bias;  phi_j = a_j (x_j - c_j), j < dphi.
void launch_predict_raw64(const float* X, int64_t n, int ld, int d, const float* a, float bias, double* prob,
                          double* logit, hipStream_t stream);
// Persistent serving kernel (serve/gpu_owner.py native owner, small batches): ONE workgroup that
// polls a mailbox in fine-grained (coherent, mapped) host memory, scores the posted rows and
// acknowledges -- no kernel launch and no event per batch.  Every field is written with
// system-scope atomics on both sides.  The kernel exits on `stop`, after `idle_ticks` of wall
// clock without a request, or after `life_ticks` in total (every wave reaches the exit; the
// owner relaunches on demand).
struct PersistCtl {
  uint32_t doorbell;  // host: sequence number of the posted batch
  uint32_t n;         // host: rows of the posted batch (<= the kernel's cap)
  uint32_t done;      // kernel: sequence number of the last finished batch
  uint32_t state;     // kernel: 1 running, 2 exited
  uint32_t stop;      // host: 1 = exit now
  uint32_t served;    // kernel: batches served by this launch
  uint32_t pad[2];
};
constexpr uint32_t kPersistRunning = 1, kPersistExited = 2;
void launch_predict_persistent(PersistCtl* ctl, const float* X, int d, int cap, const float* a, const float* c,
                               float bias, float* prob, float* logit, uint64_t idle_ticks, uint64_t life_ticks,
                               hipStream_t stream);
// CV fold scoring: logits of raw rows idx[0..n) under a fit's device state (w: fp64 [32]
// standardized-space weights; mean / scale: fp64 scaler stats)
void launch_predict_gather_logit(const float* X, const int64_t* idx, int64_t n, int d, const double* w,
                                 const double* mean, const double* scale, float* logit, hipStream_t stream);
void launch_predict_shap(const void* X, int in_kind, int64_t n, int ld, int dz, int dphi,
                         const float* a, const float* c, float bias, float* prob, float* logit,
                         float* phi, int ld_phi, hipStream_t stream);

// ---- logreg.hip ----
constexpr int kLRPartStride = 1088;  // [0,32) grad, 32 loss, 33 wsum, [64,1088) Hessian 32x32
int logreg_pass_blocks(int fmt = 0);
// Virtual SMOTE rows: the fit's rows are the stored rows [0, n_real) followed by SMOTE samples
// that are never written.  Sample s = a_i + lam (b_j - a_i) with i = pick / k, j = nbr[pick]; its
// logit is (1 - lam) z(a_i) + lam z(b_j), so a pass needs per pick (i, j) only sums over the
// pick's lambdas: smote_bucket (once per fit) groups the samples' lambdas by pick, and the pass
// folds each pick's sums into gradient / loss / Hessian terms of its two parent rows.
struct SmoteView {
  const uint16_t* parents = nullptr;  // bf16 [m, 32] output-space parents (smote_parents)
  const int* nbr = nullptr;           // int32 [mq * k] neighbour rows (indices into parents)
  const uint16_t* lam = nullptr;      // [n_new] lambda * 2^16 grouped by pick
  const int* off = nullptr;           // [mq * k] start of each pick's run in lam
  const int* cnt = nullptr;           // [mq * k] length of each pick's run
  int64_t n_real = 0;                 // stored rows; the pass covers n_real + n_new rows
  int64_t q_offset = 0;               // parent row of query 0
  int mq = 0, k = 1;
};
// Lambda buckets of SMOTE samples [sample_offset, sample_offset + n_new) of one global draw
// sequence (smote.hip, two-level LDS counting sort).  table: int32 [blocks(n_new) * bins];
// stage 0 fills it with per-(block, bin) counts (and zeroes *bump), stage 1 turns each block's row
// into its within-block exclusive prefix and writes the coarse records rec (uint32 [n_new]; a
// block's run starts at a closed-form offset, no global scan), stage 2 writes each pick's lambda
// run (pstart, pcnt: int32 [mq k]) into lam (uint16 [n_new]); tmp (uint32 [n_new]) is scratch for
// bins too big for the LDS stage.
constexpr uint64_t kSmoteBucketMaxPicks = 1ull << 21;  // <= 16384 coarse bins of <= 128 picks
int smote_bucket_bins(int64_t range, int64_t n_new);
int smote_bucket_blocks(int64_t n_new);
int64_t smote_bucket_max_samples();
void launch_smote_bucket(int stage, int mq, int k, int64_t n_new, int64_t sample_offset, uint64_t seed,
                         uint64_t counter_base, int* table, uint32_t* rec, uint32_t* tmp, int* pstart, int* pcnt,
                         uint16_t* lam, unsigned long long* bump, hipStream_t stream);
// A block of stored rows a pass steps over (the validation fold of a cross-validation fit on the
// fold-sorted training table): logical row r >= at reads physical row r + len.
struct RowHole {
  int64_t at = 0, len = 0;
};
// A Newton iteration in ONE launch (single process): the pass's blocks write their partials as
// usual; the last block of each group of kNewtonGroup blocks reduces its group's partials to fp64
// (fixed block order; the Hessian's upper triangle only), the last of those reduces the groups
// (fixed order) into `red` -- logreg_reduce's output with H mirrored exactly symmetric -- and runs
// the Newton update on its first wave.  Replaces the logreg_reduce + newton_update launches.
// Opt-in (FDX_NEWTON_FUSE=1): measured SLOWER than the two launches it replaces -- a warm-up
// iteration 64 us against 21 + 6 + 12 (profiles/r6_newton_fuse): inside one launch the cross-XCD
// hand-off needs agent-coherent loads and ticket round trips (~3 us each, ~9 on the chain), where a
// kernel boundary publishes the partials to the next launch's ordinary cached loads for free.
constexpr int kNewtonGroup = 16;
constexpr int kNewtonMaxGroups = 128;
constexpr int kNewtonCols = 35 + 528;  // grad, loss, weight, H weight + the upper triangle of H
constexpr int kNewtonColStride = 576;
// workspace (8-byte words): tickets (kNewtonMaxGroups + 1 uint32, zero, left zero), then the fp64
// group sums [kNewtonMaxGroups][kNewtonColStride]
constexpr int kNewtonFuseWords = (kNewtonMaxGroups + 2) / 2 + kNewtonMaxGroups * kNewtonColStride;
struct NewtonFuse {
  double* red = nullptr;  // null: no fused update (the plain pass)
  unsigned long long* ws = nullptr;  // [kNewtonFuseWords]
  double* st = nullptr;
  float* w32 = nullptr;
  int* done = nullptr;
  const double* aff = nullptr;
  int* done_host = nullptr;
  double C = 1.0, tol = 0.0;
  int d = 30, max_iter = 1, fit_intercept = 1, phase_start = 0, seq = 0;
};
void launch_logreg_pass(const uint16_t* X, int64_t row_begin, int64_t row_end, const float* w,
                        const float* class_w, const int* done, int hessian, int row_sub,
                        float* partial, int nblocks, hipStream_t stream, const SmoteView* sv = nullptr,
                        int row_phase = 0, bool fisher = false, RowHole hole = {},
                        const NewtonFuse* nf = nullptr);
void launch_logreg_pass_fp8(const uint8_t* X, int64_t row_begin, int64_t row_end, const float* w,
                            const float* class_w, const int* done, int hessian, int row_sub,
                            float x_scale, float* partial, int nblocks, hipStream_t stream,
                            const SmoteView* sv = nullptr, int row_phase = 0, bool fisher = false,
                            RowHole hole = {}, const NewtonFuse* nf = nullptr);
void launch_logreg_reduce(const float* partial, int nblocks, int ncols, double* out,
                          const int* done, hipStream_t stream);
// state layout: see logreg.hip NewtonState.
// aff (nullable, [64] = c | 1/sigma): the rows are pivot-shifted, not standardized -- the kernel
// maps the reduced sums into standardized space and writes folded weights to w32.
// done_host (nullable): device address of a mapped pinned int that receives (seq << 1) | done
void launch_newton_update(const double* red, double* state, float* w32, int* done, int d,
                          double C, double tol, int max_iter, int fit_intercept, int phase_start,
                          const double* aff, hipStream_t stream, int* done_host = nullptr, int seq = 0);
// tools/newton_stamps.py: the d = 30 update with s_memtime stamps at its 7 phase boundaries
void launch_newton_update_stamped(const double* red, double* state, float* w32, int* done, double C,
                                  const double* aff, unsigned long long* stamps, hipStream_t stream);
void launch_logreg_fold(const double* state, const double* aff, float* w32, hipStream_t stream);
// Fit-start state from kernel arguments (w0 in padded layout, class weights).
struct LRInitArgs {
  double w0[32];
  float cw0, cw1;
};
// persist_ws (nullable): also do the persistent SGD launch's prep (zero the barrier/accumulator
// words, back up the initial state) in the same kernel -- SgdPersistArgs::prepped
void launch_logreg_init(const LRInitArgs& a, double* state, float* w32, float* class_w, int* done,
                        const double* aff, hipStream_t stream, const double* w0_dev = nullptr,
                        unsigned long long* persist_ws = nullptr);
void launch_logreg_export(const double* state, double* host_dev, hipStream_t stream, long long seq = 0);
// Minibatch SGD step (logreg.hip sgd_apply): c = epoch step scalar (lr = c / mean curvature),
// nb = minibatches per epoch, avg = add this step's iterate to the Polyak average, epoch_end =
// settle the epoch's convergence state (and return the average when one was taken).
struct SgdArgs {
  double C = 1.0, c = 0.5, momentum = 0.5, tol = 1e-3;
  int d = 30, fit_intercept = 1, nb = 1, avg = 0, epoch_end = 0;
};
// one process: fixed-order reduce of the FISH pass's partials + the update, one launch
void launch_sgd_step(const float* partial, int nblocks, double* state, float* w32, int* done, const double* aff,
                     const SgdArgs& a, hipStream_t stream);
// one process, one launch per step: the FISH pass with fixed-point atomic sums and the update in
// its last block (acc: kSgdAccWords = 32 x 36 int64 replicas, ticket: 1 uint32 -- both zero between
// steps)
void launch_sgd_pass_fused(const void* X, int fp8, float x_scale, int64_t row_end, float* w32, const float* class_w,
                           int* done, int row_sub, int row_phase, int nblocks, const SmoteView* sv, RowHole hole,
                           unsigned long long* acc, unsigned int* ticket, double* state, const double* aff,
                           const SgdArgs& a, hipStream_t stream);
// data parallel: the update from the all-reduced [36] sums
void launch_sgd_update(const double* red, double* state, float* w32, int* done, const double* aff,
                       const SgdArgs& a, hipStream_t stream);
// Data parallel, lean step: the FISH pass adds its fixed-point sums into the replicated
// accumulators and its last block folds them into sums[36] (int64, 2^-20 units) and zeroes them --
// the vector the ranks all-reduce (integer: exact, order-free) before launch_sgd_update_fixed.
void launch_sgd_pass_sums(const void* X, int fp8, float x_scale, int64_t row_end, const float* w32,
                          const float* class_w, const int* done, int row_sub, int row_phase, int nblocks,
                          const SmoteView* sv, RowHole hole, unsigned long long* acc, unsigned int* ticket,
                          long long* sums, const double* aff, hipStream_t stream);
void launch_sgd_update_fixed(const long long* sums, double* state, float* w32, int* done, const double* aff,
                             const SgdArgs& a, hipStream_t stream);
// One process: the whole SGD schedule (steps [s0, s1) of epochs x nb minibatches) in ONE
// persistent launch (logreg.hip sgd_persist_kernel): one 512-thread block per CU whose 8 waves are
// waves of the per-step grid, a grid barrier per step, the update applied redundantly by every
// block to its LDS copy of the state (bitwise the per-step launches' fit).
// The SGD pass grid (its waves define the minibatch partition): 2 x 256-thread blocks per CU, so
// that the persistent launch holds it as one 8-wave block per CU.
int sgd_full_blocks();
constexpr int kSgdMaxEpochs = 8;
// barrier shards (1 KB) | 3 accumulator sets | fault word | backup of the initial state + weights + done
// (logreg.hip kWs*: static_assert that it fits)
constexpr int kSgdPersistWords = 128 + 3 * 32 * 36;
struct SgdPersistArgs {
  unsigned long long* ws = nullptr;  // [kSgdPersistWords] int64 workspace (zeroed by the launcher)
  double* st = nullptr;
  float* w32 = nullptr;
  int* done = nullptr;
  const double* aff = nullptr;
  double C = 1.0, momentum = 0.5, tol = 1e-3;
  double lr[kSgdMaxEpochs] = {};
  int sub[kSgdMaxEpochs] = {1, 1, 1, 1, 1, 1, 1, 1};  // per-epoch row sub-sample (1 = every row)
  int nbe[kSgdMaxEpochs] = {1, 1, 1, 1, 1, 1, 1, 1};  // per-epoch minibatch count (steps)
  int estart[kSgdMaxEpochs + 1] = {};                  // first step of every epoch (prefix of nbe)
  // avg_from: steps of epochs >= avg_from add to the Polyak average (each such epoch returns its
  // own average); >= epochs: no averaging
  int d = 30, fit_intercept = 1, nb = 1, epochs = 1, avg_from = 0, serpentine = 0;
  int s0 = 0, s1 = 0;
  int64_t Gw = 0;  // waves of the per-step pass grid (4 x its blocks): sets the minibatch partition
  unsigned long long* stamps = nullptr;  // nullable: [steps][3 + 8][blocks] wall_clock64 at pass end,
                                         // barrier exit, update end, then each wave's pass end
                                         // (tools/sgd_stamps.py)
  unsigned spin_limit = 1u << 20;        // barrier polls before a block declares the grid not resident
  int fault_test = 0;                    // test knob: barrier s0 unreachable -> the recovery launch runs
  // nullable: device address of a mapped pinned [kStateSize + 1] fp64 slot -- the recovery launch
  // exports the final state there (instead of a separate logreg_export launch behind it), then
  // export_seq into word kStateSize (int64): the host polls that stamp, so no event is recorded
  // behind the launch (a marker the command processor spends ~7 us on at the fit boundary)
  double* export_host = nullptr;
  long long export_seq = 0;
  int prepped = 0;  // logreg_init already zeroed ws and backed up the initial state (no prep launch)
};
// Returns 0 when enqueued (prep kernel, the persistent launch, its recovery launch); 1 when the
// cooperative launch refused the grid (nothing enqueued: the caller runs the per-step launches).
int launch_sgd_persist(const void* X, int fp8, float x_scale, int64_t row_end, const float* class_w,
                       const SmoteView* sv, RowHole hole, const SgdPersistArgs& a, hipStream_t stream);
// blocks of the persistent launch for a per-step grid of `grid_blocks` 256-thread blocks, or 0 when
// that many 512-thread blocks cannot all be resident (the caller then launches per step)
int sgd_persist_blocks(int grid_blocks);

// ---- knn.hip ----
// role 0: candidate rows [x, -0.5||x||^2, 0]; role 1: query rows [x, 1, 0] (features = cols 0..29);
// role 2: both from one read (candidates -> out, queries -> outq).  P (roles 0/2, optional): the
// bf16 SMOTE parents of launch_smote_parents (with aff) written by the same launch.
// chl / qhl / tmax (role 2, all or none): the bf16x3 engines' hi/lo split fused in (knn_split role 2
// for the candidates, role 1 for the queries)
void launch_knn_prep(const float* X, int m, int m_pad, int role, float* out, float* outq,
                     const double* aff, uint16_t* P, hipStream_t stream, void* chl = nullptr, void* qhl = nullptr,
                     float* tmax = nullptr);
int knn_splits(int mq_pad, int mc_pad);
// bf16x3 MFMA filter + exact fp32 re-score (knn.hip): hl [m_pad][8] uint4 = hi | lo bf16 rows of
// the prepped rows; tmax [mc_pad / 32] max candidate norm per tile (role 0 only)
void launch_knn_split(const float* Xp, int m_pad, int role, uint4* hl, float* tmax, hipStream_t stream);
int knn3_splits(int mq_pad, int mc_pad);
// LDS-tiled fp32 engine: workgroups of 4 waves x 32 queries share staged candidate chunks
// (mq_pad multiple of 128)
int knn_lds_splits(int mq_pad, int mc_pad);
// bf16x3 collect (per-lane candidate lists [nsplit][mq_pad / 32][cap][64] int32 pairs + counts
// [nsplit][mq_pad / 32][64]) then exact fp32 re-rank of the listed candidates (knn.hip)
// bf16x3 scores with register top-8 approximate lists per (slice, query), then ONE merge kernel that
// re-scores the 8 best exactly and proves the exact top-k; the queries it cannot prove go to an exact
// scan (one workgroup each).  ws_m [nsplit][mq][2]; fail int [1 + mq] (count, query ids).
int knn_b3top_splits(int mq_pad, int mc_pad);
void launch_knn_b3top(const float* Q, const void* Qhl, int mq_pad, int mq, const float* C, const void* Chl,
                      const float* tmax, int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                      float* out_score, float* ws_s, int* ws_i, float* ws_m, int* fail, int nsplit,
                      hipStream_t stream);
int knn3r_list_cap();
int knn3r_splits(int mq_pad, int mc_pad);
void launch_knn_topk3r(const float* Q, const void* Qhl, int mq_pad, int mq, const float* C, const void* Chl,
                       const float* tmax, int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                       float* out_score, int* lists, int* counts, int nsplit, hipStream_t stream);
void launch_knn_topk_lds(const float* Q, int mq_pad, int mq, const float* C, int mc_pad, int mc,
                         int64_t self_offset, int k, int* out_idx, float* out_score, float* ws_score, int* ws_idx,
                         int nsplit, hipStream_t stream);
void launch_knn_topk3(const float* Q, const void* Qhl, int mq_pad, int mq, const float* C, const void* Chl,
                      const float* tmax, int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                      float* out_score, float* ws_score, int* ws_idx, int nsplit, hipStream_t stream);
void launch_knn_topk(const float* Q, int mq_pad, int mq, const float* C,
                     int mc_pad, int mc, int64_t self_offset, int k, int* out_idx,
                     float* out_score, float* ws_score, int* ws_idx, int nsplit, hipStream_t stream);

// ---- smote.hip ----
// P [m, 32] bf16 = output-space parents: bf16(C * sigma + c) on the feature columns (aff nullable)
void launch_smote_parents(const float* C, int64_t m, const double* aff, uint16_t* P, hipStream_t stream);
// C: fp32 standardized parents (+ aff applied per sample) or, parents_bf16, smote_parents output
void launch_smote_generate(const void* C, int parents_bf16, const int* nbr, int mq, int k, int64_t q_offset,
                           int64_t n_new, int64_t sample_offset, uint64_t seed, uint64_t counter_base, float label,
                           int out_kind, float out_scale, const double* aff, void* out, hipStream_t stream);

// ---- auc.hip ----
void launch_auc_compact(const float* scores, const uint8_t* labels, int64_t n, float* pos,
                        unsigned long long* counter, hipStream_t stream);
void launch_sort_chunks(float* pos, int64_t npos_cap, const unsigned long long* counter,
                        int chunk, int nchunks, hipStream_t stream);
// exact AUC from sorted scores: 2 * pairs won + ties, summed over tie segments (u64, exact)
size_t auc_radix_workspace_bytes(int64_t n);
void auc_radix_layout(int64_t n, size_t off[8]);
void launch_auc_radix(const float* scores, const uint8_t* labels, int64_t n, void* ws, int64_t* res, double* auc,
                      hipStream_t stream);
void launch_auc_count(const float* scores, const uint8_t* labels, int64_t n, const float* pos,
                      const unsigned long long* counter, int chunk, int nchunks,
                      unsigned long long* out_pairs, hipStream_t stream);
void launch_confusion(const float* scores, const uint8_t* labels, int64_t n, float threshold,
                      unsigned long long* out4, hipStream_t stream);
// histogram AUC: hist = [2][2^bits] u32 (negatives, positives) keyed on the order-preserving
// score key's top bits; reduce -> {twice pair count, P, N}.  Mergeable by summing histograms.
void launch_auc_hist(const float* scores, const uint8_t* labels, int64_t n, int bits, unsigned* hist,
                     hipStream_t stream);
void launch_auc_hist_reduce(const unsigned* hist, int bits, unsigned long long* out, hipStream_t stream);

// ---- kernelshap.hip ----
// X [E][d] raw explanations; a [32] folded weights; bg = W [n_bg][32] = [a o B_b, 0.., -c_b] (the
// background rows pre-multiplied by the weights, col 31 = minus the background logit); cb [n_bg]
// background logits; Z [S_pad][32] bf16 coalitions (col 31 = 1); Amat [d-1][S_pad] (zero-padded);
// Az [d-1].  parts: coalition parts per explanation (grid = E x parts); parts > 1 needs ws
// [E][8][32] f32 and cnt [E] u32 (zeroed once; the kernel leaves it zeroed).
void launch_kernelshap(const float* X, int n_expl, int d, const float* a, float bias, const float* bg,
                       const float* cb, int n_bg, const uint16_t* Z, int S, int S_pad, int parts,
                       const float* Amat, const float* Az, int link, float* phi, float* fx_out, float* f0_out,
                       float* ws, unsigned* cnt, hipStream_t stream, unsigned long long* stamps = nullptr);
// Complement-paired design: Zm [Ppad] base coalition bitmasks (bit k = feature k taken from x,
// bit 31 = 1: the intercept column), slot Ppad + p of Amat [d-1][2 Ppad] is the complement of base
// p (zero column when it is not in the design).
void launch_kernelshap_paired(const float* X, int n_expl, int d, const float* a, float bias, const float* bg,
                              const float* cb, int n_bg, const uint32_t* Zm, int Ppad, int parts, const float* Amat,
                              const float* Az, int link, float* phi, float* fx_out, float* f0_out, float* ws,
                              unsigned* cnt, hipStream_t stream);
// workgroups of the linear kernel resident on the device at once (parts -> LDS per workgroup)
int kernelshap_linear_resident(int S_pad, int parts);
// Tree-ensemble model (depth <= 5): Xs [E][ldx] standardized rows; feat/thr [T][2^D-1], leaf
// [T][2^D]; bw [T][bw_ld] direction bits of the background rows (bit n+1 = node n goes right);
// Zm [S_pad] coalition bitmasks (bit k = feature k taken from x).
// interventional TreeSHAP (treeshap.hip): exact SHAP of the ensemble margin vs a background set;
// Xs standardized [n_expl][ldx], bw [T][bw_ld] background direction bits, f0 = mean background margin
void launch_treeshap(const float* Xs, int ldx, int n_expl, int d, const int* feat, const float* thr,
                     const float* leaf, int ntrees, int depth, float base_margin, const uint32_t* bw, int bw_ld,
                     int n_bg, float f0, float* phi, float* fx_out, float* f0_out, hipStream_t stream);
void launch_kernelshap_tree(const float* Xs, int ldx, int n_expl, int d, const int* feat, const float* thr,
                            const float* leaf, int ntrees, int depth, float base_margin, const uint32_t* bw,
                            int bw_ld, int n_bg, const uint32_t* Zm, int S, int S_pad, int parts,
                            const float* Amat, const float* Az, int link, float* phi, float* fx_out,
                            float* f0_out, float* ws, unsigned* cnt, hipStream_t stream);

// ---- K11 gbdt (gbdt.hip) ----
void launch_gbdt_bin(const float* X, int64_t n, int ld, int d, const float* cuts, const int* nbins,
                     uint8_t* bins, hipStream_t stream);
void launch_gbdt_grad(const float* margin, const uint8_t* label, int64_t n, float spw, float gscale,
                      float hscale, uint32_t* gh, hipStream_t stream);
int gbdt_hist_blocks();
// exact per-feature order statistics of the cut sample (quantile.hip): out [max_bin][d] holds the
// minimum (row 0) and the values at ranks floor(t m / max_bin); rows r * stride of X [., ld]
int64_t quantile_select_ws_bytes(int64_t m, int d);
void launch_quantile_select(const float* X, int64_t m, int64_t stride, int ld, int d, int max_bin, void* ws,
                            float* out, hipStream_t stream);
int64_t gbdt_hist_slot_words();  // int64 words of the per-(node, block) histogram slots
// hole_at / hole_len (hist and partition): the fit's rows are the table minus the block
// [hole_at, hole_at + hole_len) -- a cross-validation fold on the fold-sorted table (n counts the
// fit's rows, not the table's)
// histogram kernel variant for labs/tests (-1: FDX_GBDT_HIST_VAR; 0 lockstep, 1 rotated, 2 split g/h)
void set_gbdt_hist_variant(int v);
void launch_gbdt_hist(const uint8_t* bins, const uint32_t* gh, const int* ridx, const int64_t* seg,
                      const int64_t* gcnt, int level, int d, unsigned long long* hist, long long* slots,
                      hipStream_t stream, int64_t flush_rows = 0, int64_t hole_at = 0, int64_t hole_len = 0);
// Level 0 of a round after a fit's first: the previous tree's margin walk + (g, h) fused in front of
// the histogram (gbdt.hip gbdt_hist_l0_fused_kernel); replaces gbdt_margin<GRAD> + gbdt_hist(level 0).
void launch_gbdt_hist_l0_fused(const uint8_t* bins, uint32_t* gh, const int64_t* seg, const int64_t* gcnt, int d,
                               unsigned long long* hist, long long* slots, hipStream_t stream, int64_t flush_rows,
                               int64_t hole_at, int64_t hole_len, const int* feat, const int* bin, const float* leaf,
                               int depth, float* margin, const uint8_t* label, float spw, float gscale, float hscale);
void launch_gbdt_split(unsigned long long* hist, const int64_t* gcnt, int level, int d, const int* nbins,
                       const float* cuts, double ginv, double hinv, double lambda,
                       double min_child_weight, double gamma, int* feat, int* bin, float* thr,
                       double* gain, long long* ng, long long* nh, hipStream_t stream);
// row-major [n][32] bins -> feature-major [d][ldt] (the partition's per-row feature reads)
void launch_gbdt_transpose(const uint8_t* bins, int64_t n, int d, uint8_t* binsT, int64_t ldt, hipStream_t stream);
void launch_gbdt_partition(const uint8_t* binsT, int64_t ldt, const int* ridx, const uint8_t* nid, int64_t n,
                           const int* feat, const int* bin, int level, uint8_t* flag, int64_t* counts,
                           int nblocks, int64_t* seg, int64_t* node_r, int* ridx_out, uint8_t* nid_out,
                           hipStream_t stream, int64_t* gcnt = nullptr, int64_t hole_at = 0, int64_t hole_len = 0);
// node_r[0, n_nodes) (per-node right counts of the partition) is zeroed too
void launch_gbdt_round_init(unsigned long long* hist, int64_t hist_words, int64_t* seg, int64_t* gcnt, int64_t n,
                            int64_t n_global, hipStream_t stream, int64_t* node_r, int n_nodes);
void launch_gbdt_leaf(const long long* ng, const long long* nh, int depth, double ginv, double hinv,
                      double lambda, double min_child_weight, double eta, float* leaf, hipStream_t stream);
void launch_gbdt_margin(const uint8_t* binsT, int64_t ldt, int64_t n, const int* feat, const int* bin,
                        const float* leaf, int depth, float* margin, const uint8_t* label, float spw, float gscale,
                        float hscale, uint32_t* gh, hipStream_t stream);
void launch_gbdt_predict(const float* X, int64_t n, int ld, int d, const int* feat, const float* thr,
                         const float* leaf, int ntrees, int depth, float base_margin, float* out,
                         hipStream_t stream);

}  // namespace fdx
