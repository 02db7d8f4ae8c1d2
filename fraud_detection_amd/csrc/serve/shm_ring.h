// Shared-memory request ring between serving front-ends and the single GPU-owner process
// (SURVEY.md §2.4 "web-server process parallelism": the reference runs gunicorn --workers 2 with a
// model copy per worker, Dockerfile:21 / docker-compose.yml:74; here N front-end processes forward
// rows to ONE process that owns the GPU context and micro-batches them into one launch).
//
// Layout (one file in /dev/shm, mmap'ed MAP_SHARED by every process, or an anonymous mapping when
// owner and front-end share a process):
//   Header | Slot[nslots] (64-byte header each) | inputs  [nslots][slot_rows][d] f32
//                                               | outputs [nslots][slot_rows][out_w] f32
// A request of n rows takes ceil(n / slot_rows) consecutive tickets.  Ticket t owns slot t % nslots
// while the slot's tag holds turn t (a bounded MPSC ring, Vyukov-style lap counters), so producers
// never block each other except when the ring is full.  The tag packs (turn << 3) | state into ONE
// 64-bit word and every hand-off is a compare-and-swap on it, so no transition can land on another
// lap's slot:
//   (t, FREE) -producer-> (t, CLAIMED) -writes rows-> (t, READY) -owner gathers-> (t, TAKEN)
//   -owner scatters results-> (t, DONE | FAILED) -producer reads results-> (t + N, FREE).
// Abandonment (a producer that times out, dies, or gives up on a ticket) never frees a slot the
// owner may still hold:
//   * waiting for results: the producer CASes (t, READY | TAKEN) -> (t, CANCELLED) and leaves; the
//     owner frees a cancelled slot when it meets it (at the tail, or when its CAS TAKEN -> DONE
//     fails in complete()), so a late batch result is never written into the next lap's slot;
//   * waiting for room: tickets are taken only together with free slots (a CAS on head after
//     checking that the slots at head are FREE at their turns), so a producer that times out
//     there holds nothing;
//   * a producer that died between taking its tickets and publishing (or between DONE and
//     freeing): the owner reclaims a tail ticket that stays unpublished / unfreed for
//     reclaim_ms (a late CAS by that producer then fails and it raises instead of corrupting).
// Wake-ups are futexes on 32-bit words in the shared mapping: the owner sleeps on `doorbell` (bumped
// once per published or cancelled slot, woken only while the owner says it sleeps), producers sleep
// on `completions` (bumped once per completed BATCH, one FUTEX_WAKE for the whole batch -- not one
// syscall per row).  Everything is lock-free; the only kernel calls are the futex sleeps and wakes.
#pragma once
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <fcntl.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <climits>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace fdx_ring {
namespace {

constexpr uint32_t kMagic = 0x46445852;  // "FDXR"
constexpr uint32_t kVersion = 2;
enum : uint32_t { FREE = 0, CLAIMED = 1, READY = 2, TAKEN = 3, DONE = 4, FAILED = 5, CANCELLED = 6 };
constexpr double kReclaimMs = 30000.0;  // default: 3x the producers' default request timeout

inline uint64_t tag_of(uint64_t turn, uint32_t st) { return (turn << 3) | st; }
inline uint64_t turn_of(uint64_t tag) { return tag >> 3; }
inline uint32_t state_of(uint64_t tag) { return (uint32_t)(tag & 7u); }
enum : uint32_t { OWNER_STARTING = 0, OWNER_READY = 1, OWNER_STOPPED = 2 };

struct alignas(64) Header {
  uint32_t magic, version;
  uint32_t nslots, d, slot_rows, out_w;
  uint64_t total_bytes;
  alignas(64) std::atomic<uint64_t> head;  // next ticket handed to a producer
  alignas(64) std::atomic<uint64_t> tail;  // next ticket the owner gathers
  alignas(64) std::atomic<uint32_t> doorbell;
  std::atomic<uint32_t> owner_sleeping;
  alignas(64) std::atomic<uint32_t> completions;
  std::atomic<uint32_t> sleepers;  // producers inside a futex wait on `completions`
  alignas(64) std::atomic<uint32_t> owner_state;
  std::atomic<int32_t> owner_pid;
  std::atomic<int32_t> host_max_rows;  // owner's calibrated small-batch threshold (-1 = unknown)
  std::atomic<uint64_t> batches;       // owner statistics (exported by the front-ends' /metrics)
  std::atomic<uint64_t> rows;
  std::atomic<uint64_t> slots_done;
  std::atomic<uint64_t> cancelled;     // slots freed by the owner for an abandoning producer
  std::atomic<uint64_t> reclaimed;     // tickets reclaimed from a stalled / dead producer
  std::atomic<uint64_t> reclaim_ns;    // how long a tail ticket may stay unpublished / unfreed
};

struct alignas(64) Slot {
  std::atomic<uint64_t> tag;  // (turn << 3) | state
  uint32_t n_rows;
  uint32_t op;
};

long futex(std::atomic<uint32_t>* addr, int op, uint32_t val, const struct timespec* ts) {
  return syscall(SYS_futex, reinterpret_cast<uint32_t*>(addr), op, val, ts, nullptr, 0);
}

inline void cpu_relax() { __builtin_ia32_pause(); }

inline uint64_t now_ns() {
  return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Taken {
  uint64_t ticket;
  uint32_t row0, n;
};

class Ring {
 public:
  // create: the owner side (or an in-process ring when path is empty)
  Ring(const std::string& path, uint32_t nslots, uint32_t d, uint32_t slot_rows, uint32_t out_w) : path_(path) {
    if (nslots < 2 || d == 0 || slot_rows == 0 || out_w == 0) throw std::runtime_error("ring: bad geometry");
    size_t in_b = (size_t)nslots * slot_rows * d * 4, out_b = (size_t)nslots * slot_rows * out_w * 4;
    bytes_ = sizeof(Header) + (size_t)nslots * sizeof(Slot) + in_b + out_b;
    map(true);
    h_->magic = kMagic;
    h_->version = kVersion;
    h_->nslots = nslots;
    h_->d = d;
    h_->slot_rows = slot_rows;
    h_->out_w = out_w;
    h_->total_bytes = bytes_;
    h_->head.store(0);
    h_->tail.store(0);
    h_->doorbell.store(0);
    h_->owner_sleeping.store(0);
    h_->completions.store(0);
    h_->sleepers.store(0);
    h_->owner_pid.store((int32_t)getpid());
    h_->host_max_rows.store(-1);
    h_->batches.store(0);
    h_->rows.store(0);
    h_->slots_done.store(0);
    h_->cancelled.store(0);
    h_->reclaimed.store(0);
    h_->reclaim_ns.store((uint64_t)(kReclaimMs * 1e6));
    for (uint32_t i = 0; i < nslots; ++i) {
      slots_[i].tag.store(tag_of(i, FREE));
    }
    h_->owner_state.store(OWNER_STARTING, std::memory_order_release);
  }
  // view of a mapping owned by another Ring object of this process (the native owner loop)
  Ring(char* base, size_t bytes) : bytes_(bytes), base_(base), owns_(false) {
    bind();
    if (h_->magic != kMagic || h_->version != kVersion || h_->total_bytes != bytes_)
      throw std::runtime_error("ring: not an fdx ring view");
  }
  // attach: a front-end process
  explicit Ring(const std::string& path) : path_(path) {
    int fd = ::open(path.c_str(), O_RDWR);
    if (fd < 0) throw std::runtime_error("ring: cannot open " + path);
    struct stat st;
    fstat(fd, &st);
    bytes_ = (size_t)st.st_size;
    void* m = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (m == MAP_FAILED) throw std::runtime_error("ring: mmap failed");
    base_ = static_cast<char*>(m);
    bind();
    if (h_->magic != kMagic || h_->version != kVersion || h_->total_bytes != bytes_)
      throw std::runtime_error("ring: not an fdx ring (or version mismatch): " + path);
  }
  ~Ring() {
    if (base_ && owns_) munmap(base_, bytes_);
  }
  Ring(const Ring&) = delete;
  Ring& operator=(const Ring&) = delete;

  uint32_t d() const { return h_->d; }
  uint32_t out_w() const { return h_->out_w; }
  uint32_t slot_rows() const { return h_->slot_rows; }
  uint32_t nslots() const { return h_->nslots; }

  // ---- owner lifecycle / shared state -----------------------------------------------------
  void set_owner_state(uint32_t s) {
    h_->owner_state.store(s, std::memory_order_release);
    if (s == OWNER_STOPPED) {  // fail everything still queued and wake every sleeper
      h_->completions.fetch_add(1);
      futex(&h_->completions, FUTEX_WAKE, INT_MAX, nullptr);
    }
  }
  uint32_t owner_state() const { return h_->owner_state.load(std::memory_order_acquire); }
  int owner_pid() const { return h_->owner_pid.load(); }
  void set_host_max_rows(int v) { h_->host_max_rows.store(v); }
  int host_max_rows() const { return h_->host_max_rows.load(); }
  struct Stats {
    uint64_t batches, rows, slots, queued, cancelled, reclaimed;
  };
  Stats stats() const {
    return {h_->batches.load(), h_->rows.load(), h_->slots_done.load(), h_->head.load() - h_->tail.load(),
            h_->cancelled.load(), h_->reclaimed.load()};
  }
  void set_reclaim_ms(double ms) { h_->reclaim_ns.store((uint64_t)(ms * 1e6)); }
  double reclaim_ms() const { return (double)h_->reclaim_ns.load() * 1e-6; }
  // Rows in the consecutive READY slots at the tail (the owner's look before pipelining a batch)
  uint32_t ready_rows(uint32_t limit) const {
    const uint32_t N = h_->nslots;
    uint64_t t = h_->tail.load(std::memory_order_relaxed);
    uint32_t rows = 0;
    while (rows < limit) {
      const Slot& s = slots_[t % N];
      if (s.tag.load(std::memory_order_acquire) != tag_of(t, READY)) break;
      rows += s.n_rows;
      ++t;
    }
    return rows;
  }
  char* base_address() const { return base_; }
  size_t total_bytes() const { return bytes_; }
  uint32_t d_() const { return h_->d; }

  // ---- producer ------------------------------------------------------------------------------
  // Rows X [n, d] -> out [n, out_w]; op: 0 = predict, 1 = explain.  Blocks (GIL released) until
  // every chunk is DONE.  Raises on owner failure or after timeout_ms -- having cancelled or
  // abandoned every ticket it took, so the ring stays consistent for the next request.
  void request(const float* X, float* out, uint32_t n, uint32_t op, double timeout_ms) {
    const uint32_t R = h_->slot_rows, d = h_->d, W = h_->out_w, N = h_->nslots;
    const uint32_t nchunks = (n + R - 1) / R;
    if (nchunks > N) throw std::runtime_error("ring: request larger than the ring");
    const uint64_t deadline = now_ns() + (uint64_t)(timeout_ms * 1e6);
    // Tickets are taken only together with free slots (CAS on head after checking that the
    // slots at head are FREE at their turns; only a ticket's holder leaves FREE, so they stay
    // free): a producer that times out waiting for room holds no ticket it has not published, and
    // the owner never waits on a ticket nobody will publish -- except one whose producer died
    // right after this CAS, which the owner reclaims after reclaim_ms.  A large request takes its
    // tickets in pieces of at most a quarter of the ring (publishing each piece before it takes
    // the next), so a stream of one-chunk requests cannot starve it of nchunks free slots at once.
    const uint32_t piece = std::max<uint32_t>(1u, N / 4);
    std::vector<uint64_t> tix;
    tix.reserve(nchunks);
    uint32_t published = 0, consumed = 0;
    bool failed = false, timed_out = false;
    const char* err = nullptr;
    // consume this request's finished chunks in order (frees their slots for its later pieces)
    auto consume_finished = [&] {
      while (consumed < published) {
        const uint64_t t = tix[consumed];
        const uint32_t st = state_of(slots_[t % N].tag.load(std::memory_order_acquire));
        if (st != DONE && st != FAILED) break;
        const uint32_t m = std::min(R, n - consumed * R);
        if (cancel_or_consume(t, out + (size_t)consumed * R * W, m, W) != DONE) failed = true;
        ++consumed;
      }
    };
    for (uint32_t c = 0; c < nchunks; ++c) {
      if (c == tix.size()) {  // the next piece of tickets
        const uint32_t want = std::min(piece, nchunks - c);
        uint64_t t0 = 0;
        bool took = false;  // sleep_until may evaluate the predicate again after it held: take once
        if (!sleep_until([&] {
              if (took) return true;
              consume_finished();
              return took = try_take(want, t0);
            }, deadline)) {
          for (uint32_t e = consumed; e < published; ++e) cancel_or_consume(tix[e], nullptr, 0, 0);
          ring_doorbell();
          throw std::runtime_error(owner_gone() ? "ring: GPU owner stopped" : "ring: timed out waiting for a free slot");
        }
        for (uint32_t e = 0; e < want; ++e) tix.push_back(t0 + e);
      }
      const uint64_t t = tix[c];
      Slot& s = slots_[t % N];
      uint64_t g = tag_of(t, FREE);
      if (!s.tag.compare_exchange_strong(g, tag_of(t, CLAIMED), std::memory_order_acq_rel)) {
        err = "ring: ticket reclaimed by the owner";  // this producer stalled past reclaim_ms
        break;
      }
      const uint32_t m = std::min(R, n - c * R);
      std::memcpy(in_ptr(t % N), X + (size_t)c * R * d, (size_t)m * d * 4);
      s.n_rows = m;
      s.op = op;
      g = tag_of(t, CLAIMED);
      if (!s.tag.compare_exchange_strong(g, tag_of(t, READY), std::memory_order_acq_rel)) {
        err = "ring: ticket reclaimed by the owner";
        break;
      }
      ++published;
      ring_doorbell();
    }
    if (err != nullptr) {  // the unpublished tickets were (or will be) reclaimed by the owner
      for (uint32_t c = consumed; c < published; ++c) cancel_or_consume(tix[c], nullptr, 0, 0);
      ring_doorbell();
      throw std::runtime_error(err);
    }
    for (uint32_t c = consumed; c < nchunks; ++c) {
      const uint64_t t = tix[c];
      const uint32_t m = std::min(R, n - c * R);
      Slot& s = slots_[t % N];
      const bool fin = !timed_out && sleep_until([&] {
        const uint32_t st = state_of(s.tag.load(std::memory_order_acquire));
        return st == DONE || st == FAILED;
      }, deadline);
      if (!fin) timed_out = true;
      // finished, or cancelled (the owner frees it) -- unless the result landed meanwhile
      const uint32_t st = cancel_or_consume(t, out + (size_t)c * R * W, m, W);
      if (st != DONE) failed = true;
    }
    ring_doorbell();
    if (timed_out) throw std::runtime_error(owner_gone() ? "ring: GPU owner stopped" : "ring: timed out waiting for results");
    if (failed) throw std::runtime_error("ring: the GPU owner failed this request");
  }

  // Test hook: take n tickets and never publish them -- a producer that died right after its
  // head.fetch_add (tests/test_ring_abandon.py drills the owner's reclaim with it).
  uint64_t debug_take_tickets(uint32_t n) { return h_->head.fetch_add(n); }
  // Test hook: take tickets, publish n rows and return without waiting for (or ever consuming) the
  // results -- a producer killed while it waited for them (its slots end at (t, DONE)).
  uint64_t debug_publish(const float* X, uint32_t n, uint32_t op) {
    const uint32_t R = h_->slot_rows, d = h_->d, N = h_->nslots;
    const uint32_t nchunks = (n + R - 1) / R;
    uint64_t t0 = 0;
    if (nchunks == 0 || nchunks > N || !try_take(nchunks, t0)) throw std::runtime_error("ring: no room to publish");
    for (uint32_t c = 0; c < nchunks; ++c) {
      const uint64_t t = t0 + c;
      Slot& s = slots_[t % N];
      const uint32_t m = std::min(R, n - c * R);
      std::memcpy(in_ptr(t % N), X + (size_t)c * R * d, (size_t)m * d * 4);
      s.n_rows = m;
      s.op = op;
      s.tag.store(tag_of(t, READY), std::memory_order_release);
    }
    ring_doorbell();
    return t0;
  }
  // Test hook: (turn, state) of every slot plus (head, tail).
  std::vector<uint64_t> debug_tags() const {
    std::vector<uint64_t> v;
    for (uint32_t i = 0; i < h_->nslots; ++i) v.push_back(slots_[i].tag.load());
    v.push_back(h_->head.load());
    v.push_back(h_->tail.load());
    return v;
  }

  // ---- owner -------------------------------------------------------------------------------
  // Gather up to max_rows rows of READY slots (same op, ticket order) into dst [max_rows, d], as
  // batch `set` (0 or 1: the owner keeps one batch on the device while it gathers the next).
  // Waits up to timeout_ms for the first slot (timeout_ms <= 0: one look, no wait), then up to
  // window_us for more.  Cancelled and abandoned tickets at the tail are skipped (their slots
  // freed), and a tail ticket stuck for reclaim_ms is reclaimed.  Returns (rows, op); rows == 0 on
  // timeout.
  std::pair<uint32_t, uint32_t> collect(float* dst, uint32_t max_rows, double window_us, double timeout_ms,
                                        int set) {
    const uint32_t N = h_->nslots, d = h_->d;
    std::vector<Taken>& taken_ = taken_sets_[set & 1];
    taken_.clear();
    uint64_t t = h_->tail.load(std::memory_order_relaxed);
    const uint64_t deadline = now_ns() + (uint64_t)((timeout_ms > 0 ? timeout_ms : 0.0) * 1e6);
    if (!wait_ready(t, deadline, timeout_ms > 0)) {
      h_->tail.store(t, std::memory_order_release);
      return {0, 0};
    }
    uint32_t op = slots_[t % N].op;
    uint32_t rows = 0;
    const uint64_t wdl = now_ns() + (uint64_t)(window_us * 1e3);
    while (true) {
      Slot& s = slots_[t % N];
      const uint64_t g = s.tag.load(std::memory_order_acquire);
      if (g != tag_of(t, READY)) {
        if (skip_dead(t)) continue;
        if (rows == 0) {  // the first READY slot was cancelled under us: wait again, within the deadline
          if (!wait_ready(t, deadline, timeout_ms > 0)) break;
          op = slots_[t % N].op;
          continue;
        }
        if (rows > 0 && now_ns() >= wdl) break;
        if (h_->head.load(std::memory_order_acquire) <= t && now_ns() >= wdl) break;
        if (window_us <= 0 && rows > 0) break;
        cpu_relax();
        continue;
      }
      if (s.op != op || rows + s.n_rows > max_rows) break;
      std::memcpy(dst + (size_t)rows * d, in_ptr(t % N), (size_t)s.n_rows * d * 4);
      uint64_t e = g;
      if (!s.tag.compare_exchange_strong(e, tag_of(t, TAKEN), std::memory_order_acq_rel)) continue;  // cancelled
      taken_.push_back({t, rows, s.n_rows});
      rows += s.n_rows;
      ++t;
      if (rows == max_rows) break;
    }
    h_->tail.store(t, std::memory_order_release);
    return {rows, taken_.empty() ? 0u : op};
  }

  // Scatter the batch results: column-major pieces prob[rows], logit[rows], phi[rows][dphi]
  // (any may be null) into each taken slot's [n][out_w] rows, then one completion wake.  A slot
  // its producer cancelled meanwhile is freed instead (its late result is never handed out).
  void complete(const float* prob, const float* logit, const float* phi, uint32_t dphi, bool ok, int set) {
    const uint32_t N = h_->nslots, W = h_->out_w;
    std::vector<Taken>& taken_ = taken_sets_[set & 1];
    uint64_t rows = 0;
    for (const Taken& tk : taken_) {
      Slot& s = slots_[tk.ticket % N];
      if (s.tag.load(std::memory_order_acquire) == tag_of(tk.ticket, TAKEN)) {
        float* o = out_ptr(tk.ticket % N);
        if (ok) {
          for (uint32_t i = 0; i < tk.n; ++i) {
            float* r = o + (size_t)i * W;
            size_t g = tk.row0 + i;
            r[0] = prob ? prob[g] : 0.f;
            if (W > 1) r[1] = logit ? logit[g] : 0.f;
            if (phi && dphi && W >= 2 + dphi) std::memcpy(r + 2, phi + g * dphi, (size_t)dphi * 4);
          }
        }
      }
      uint64_t e = tag_of(tk.ticket, TAKEN);
      if (!s.tag.compare_exchange_strong(e, tag_of(tk.ticket, ok ? DONE : FAILED), std::memory_order_acq_rel)) {
        // the producer gave up (CANCELLED): the owner frees the slot for the next lap
        e = tag_of(tk.ticket, CANCELLED);
        if (s.tag.compare_exchange_strong(e, tag_of(tk.ticket + N, FREE), std::memory_order_acq_rel))
          h_->cancelled.fetch_add(1);
      }
      rows += tk.n;
    }
    h_->batches.fetch_add(1);
    h_->rows.fetch_add(rows);
    h_->slots_done.fetch_add(taken_.size());
    taken_.clear();
    wake_producers();
  }

  size_t pending_slots() const { return taken_sets_[0].size() + taken_sets_[1].size(); }

 private:
  void map(bool create) {
    if (path_.empty()) {
      void* m = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_ANONYMOUS, -1, 0);
      if (m == MAP_FAILED) throw std::runtime_error("ring: anonymous mmap failed");
      base_ = static_cast<char*>(m);
    } else {
      int fd = ::open(path_.c_str(), O_RDWR | O_CREAT | (create ? O_TRUNC : 0), 0600);
      if (fd < 0) throw std::runtime_error("ring: cannot create " + path_);
      if (ftruncate(fd, (off_t)bytes_) != 0) {
        ::close(fd);
        throw std::runtime_error("ring: ftruncate failed (is /dev/shm large enough?)");
      }
      void* m = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
      ::close(fd);
      if (m == MAP_FAILED) throw std::runtime_error("ring: mmap failed");
      base_ = static_cast<char*>(m);
      std::memset(base_, 0, sizeof(Header));
    }
    bind_raw();
  }
  void bind_raw() {
    h_ = reinterpret_cast<Header*>(base_);
    slots_ = reinterpret_cast<Slot*>(base_ + sizeof(Header));
  }
  void bind() { bind_raw(); }
  float* in_ptr(uint64_t i) {
    char* p = base_ + sizeof(Header) + (size_t)h_->nslots * sizeof(Slot);
    return reinterpret_cast<float*>(p) + i * h_->slot_rows * h_->d;
  }
  float* out_ptr(uint64_t i) {
    char* p = base_ + sizeof(Header) + (size_t)h_->nslots * sizeof(Slot) +
              (size_t)h_->nslots * h_->slot_rows * h_->d * 4;
    return reinterpret_cast<float*>(p) + i * h_->slot_rows * h_->out_w;
  }
  bool owner_gone() const { return h_->owner_state.load(std::memory_order_acquire) == OWNER_STOPPED; }

  // Producer: take nchunks consecutive tickets if their slots are FREE at those turns.
  bool try_take(uint32_t nchunks, uint64_t& t0) {
    const uint32_t N = h_->nslots;
    uint64_t h = h_->head.load(std::memory_order_acquire);
    for (int tries = 0; tries < 64; ++tries) {
      bool room = true;
      for (uint32_t c = 0; c < nchunks && room; ++c)
        room = slots_[(h + c) % N].tag.load(std::memory_order_acquire) == tag_of(h + c, FREE);
      if (!room) return false;
      if (h_->head.compare_exchange_weak(h, h + nchunks, std::memory_order_acq_rel)) {
        t0 = h;
        return true;
      }
    }
    return false;
  }

  void ring_doorbell() {
    h_->doorbell.fetch_add(1, std::memory_order_seq_cst);
    if (h_->owner_sleeping.load(std::memory_order_seq_cst)) futex(&h_->doorbell, FUTEX_WAKE, 1, nullptr);
  }
  void wake_producers() {
    h_->completions.fetch_add(1, std::memory_order_seq_cst);
    if (h_->sleepers.load(std::memory_order_seq_cst)) futex(&h_->completions, FUTEX_WAKE, INT_MAX, nullptr);
  }
  // Producer, ticket t published: if its result is in (DONE / FAILED) copy it out (dst may be
  // null) and free the slot for the next lap; otherwise cancel it (READY / TAKEN -> CANCELLED)
  // and leave the freeing to the owner.  Returns the state it resolved from.
  uint32_t cancel_or_consume(uint64_t t, float* dst, uint32_t m, uint32_t W) {
    Slot& s = slots_[t % h_->nslots];
    const uint32_t N = h_->nslots;
    while (true) {
      uint64_t g = s.tag.load(std::memory_order_acquire);
      if (turn_of(g) != t) return CANCELLED;  // reclaimed by the owner already
      const uint32_t st = state_of(g);
      if (st == DONE || st == FAILED) {
        if (st == DONE && dst != nullptr) std::memcpy(dst, out_ptr(t % N), (size_t)m * W * 4);
        if (s.tag.compare_exchange_strong(g, tag_of(t + N, FREE), std::memory_order_acq_rel)) {
          wake_producers();  // producers waiting for this slot's turn sleep on `completions` too
          return st;
        }
        continue;
      }
      if (st == READY || st == TAKEN) {
        if (s.tag.compare_exchange_strong(g, tag_of(t, CANCELLED), std::memory_order_acq_rel)) return CANCELLED;
        continue;
      }
      return CANCELLED;  // CANCELLED already (or a state no producer reaches here)
    }
  }

  // sleep on `completions` until pred() or the deadline; spins first (a batch completes in ~tens of us)
  template <class Pred>
  bool sleep_until(Pred pred, uint64_t deadline) {
    for (int i = 0; i < 128; ++i) {
      if (pred()) return true;
      cpu_relax();
    }
    while (!pred()) {
      if (owner_gone()) return pred();
      uint64_t now = now_ns();
      if (now >= deadline) return false;
      uint32_t c = h_->completions.load(std::memory_order_seq_cst);
      h_->sleepers.fetch_add(1, std::memory_order_seq_cst);
      if (!pred()) {
        uint64_t left = std::min<uint64_t>(deadline - now, 50'000'000ull);  // re-check liveness every 50 ms
        struct timespec ts = {(time_t)(left / 1000000000ull), (long)(left % 1000000000ull)};
        futex(&h_->completions, FUTEX_WAIT, c, &ts);
      }
      h_->sleepers.fetch_sub(1, std::memory_order_seq_cst);
    }
    return true;
  }
  bool wait_turn(Slot& s, uint64_t t, uint64_t deadline) {
    return sleep_until([&] { return s.tag.load(std::memory_order_acquire) == tag_of(t, FREE); }, deadline);
  }
  // Owner: the tail ticket t is dead -- cancelled by its producer, abandoned before publishing, or
  // stuck (unpublished, or its previous lap unfreed) for reclaim_ns -- so free its slot and move
  // the tail past it.  Returns true if it advanced t (or unblocked the slot for ticket t).
  bool skip_dead(uint64_t& t) {
    const uint32_t N = h_->nslots;
    Slot& s = slots_[t % N];
    uint64_t g = s.tag.load(std::memory_order_acquire);
    const uint64_t turn = turn_of(g);
    const uint32_t st = state_of(g);
    if (turn == t && st == CANCELLED) {
      if (s.tag.compare_exchange_strong(g, tag_of(t + N, FREE), std::memory_order_acq_rel)) {
        h_->cancelled.fetch_add(1);
        ++t;
        stuck_t_ = ~0ull;
        wake_producers();
        return true;
      }
      return false;
    }
    // The previous lap of slot t % N never freed (its producer died or hung after DONE / FAILED, or
    // cancelled a slot nobody freed): try_take needs (t, FREE) there, so head can never pass t --
    // this case must run the stall clock even when no producer holds ticket t yet.
    const bool lap_unfreed = turn + N == t && (st == DONE || st == FAILED || st == CANCELLED);
    if ((h_->head.load(std::memory_order_acquire) <= t && !lap_unfreed) || (turn == t && st == READY)) {
      stuck_t_ = ~0ull;
      return false;
    }
    const uint64_t now = now_ns();
    if (stuck_t_ != t || stuck_g_ != g) {  // the stall clock restarts on any progress of the slot
      stuck_t_ = t;
      stuck_g_ = g;
      stuck_since_ = now;
      return false;
    }
    if (now - stuck_since_ < h_->reclaim_ns.load(std::memory_order_relaxed)) return false;
    if (turn == t && (st == FREE || st == CLAIMED)) {  // taken but never published: reclaim the ticket
      if (s.tag.compare_exchange_strong(g, tag_of(t + N, FREE), std::memory_order_acq_rel)) {
        h_->reclaimed.fetch_add(1);
        ++t;
        stuck_t_ = ~0ull;
        wake_producers();
        return true;
      }
    } else if (lap_unfreed) {  // previous lap never freed
      if (s.tag.compare_exchange_strong(g, tag_of(t, FREE), std::memory_order_acq_rel)) {
        h_->reclaimed.fetch_add(1);
        stuck_t_ = ~0ull;
        wake_producers();
        return true;
      }
    }
    return false;
  }

  // Owner: wait (up to deadline; no wait when !block) until the tail ticket t is READY, skipping
  // dead tickets on the way.  Sleeps on `doorbell` in <= 50 ms slices (liveness and reclaim checks).
  bool wait_ready(uint64_t& t, uint64_t deadline, bool block) {
    auto rdy = [&] { return slots_[t % h_->nslots].tag.load(std::memory_order_acquire) == tag_of(t, READY); };
    for (int i = 0;; ++i) {
      if (rdy()) return true;
      if (skip_dead(t)) continue;
      if (!block) return false;
      if (i < 512) {
        cpu_relax();
        continue;
      }
      const uint64_t now = now_ns();
      if (now >= deadline || h_->owner_state.load() == OWNER_STOPPED) return false;
      uint32_t db = h_->doorbell.load(std::memory_order_seq_cst);
      h_->owner_sleeping.store(1, std::memory_order_seq_cst);
      if (!rdy()) {
        uint64_t left = std::min<uint64_t>(deadline - now, 50'000'000ull);
        struct timespec ts = {(time_t)(left / 1000000000ull), (long)(left % 1000000000ull)};
        futex(&h_->doorbell, FUTEX_WAIT, db, &ts);
      }
      h_->owner_sleeping.store(0, std::memory_order_seq_cst);
    }
  }

  std::string path_;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  Header* h_ = nullptr;
  Slot* slots_ = nullptr;
  std::vector<Taken> taken_sets_[2];
  bool owns_ = true;
  uint64_t stuck_t_ = ~0ull, stuck_g_ = 0, stuck_since_ = 0;  // owner: the tail ticket's stall clock
};

}  // namespace
}  // namespace fdx_ring
