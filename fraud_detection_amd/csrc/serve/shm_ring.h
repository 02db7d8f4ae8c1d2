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
// once slot.turn == t (a bounded MPSC ring, Vyukov-style lap counters), so producers never block
// each other except when the ring is full.  Slot state is the hand-off:
//   FREE -> (producer writes rows) READY -> (owner gathers) TAKEN -> (owner scatters results) DONE
//   -> (producer reads results) FREE with turn += nslots.
// Wake-ups are futexes on 32-bit words in the shared mapping: the owner sleeps on `doorbell` (bumped
// once per published slot, woken only while the owner says it sleeps), producers sleep on
// `completions` (bumped once per completed BATCH, one FUTEX_WAKE for the whole batch -- not one
// syscall per row).  Everything is lock-free; the only kernel calls are the futex sleeps and wakes.
#pragma once
#include <linux/futex.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <fcntl.h>
#include <time.h>
#include <unistd.h>

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
constexpr uint32_t kVersion = 1;
enum : uint32_t { FREE = 0, READY = 2, TAKEN = 3, DONE = 4, FAILED = 5 };
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
};

struct alignas(64) Slot {
  std::atomic<uint32_t> state;
  uint32_t n_rows;
  uint32_t op;
  uint32_t pad;
  std::atomic<uint64_t> turn;
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
    for (uint32_t i = 0; i < nslots; ++i) {
      slots_[i].state.store(FREE);
      slots_[i].turn.store(i);
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
    uint64_t batches, rows, slots, queued;
  };
  Stats stats() const {
    return {h_->batches.load(), h_->rows.load(), h_->slots_done.load(), h_->head.load() - h_->tail.load()};
  }
  // Rows in the consecutive READY slots at the tail (the owner's look before pipelining a batch)
  uint32_t ready_rows(uint32_t limit) const {
    const uint32_t N = h_->nslots;
    uint64_t t = h_->tail.load(std::memory_order_relaxed);
    uint32_t rows = 0;
    while (rows < limit) {
      const Slot& s = slots_[t % N];
      if (!(s.turn.load(std::memory_order_acquire) == t && s.state.load(std::memory_order_acquire) == READY)) break;
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
  // every chunk is DONE.  Raises on owner failure or after timeout_ms.
  void request(const float* X, float* out, uint32_t n, uint32_t op, double timeout_ms) {
    const uint32_t R = h_->slot_rows, d = h_->d, W = h_->out_w, N = h_->nslots;
    const uint32_t nchunks = (n + R - 1) / R;
    if (nchunks > N) throw std::runtime_error("ring: request larger than the ring");
    const uint64_t deadline = now_ns() + (uint64_t)(timeout_ms * 1e6);
    uint64_t t0 = h_->head.fetch_add(nchunks);
    for (uint32_t c = 0; c < nchunks; ++c) {
      uint64_t t = t0 + c;
      Slot& s = slots_[t % N];
      wait_turn(s, t, deadline);
      uint32_t m = std::min(R, n - c * R);
      std::memcpy(in_ptr(t % N), X + (size_t)c * R * d, (size_t)m * d * 4);
      s.n_rows = m;
      s.op = op;
      s.state.store(READY, std::memory_order_release);
      h_->doorbell.fetch_add(1, std::memory_order_seq_cst);
      if (h_->owner_sleeping.load(std::memory_order_seq_cst)) futex(&h_->doorbell, FUTEX_WAKE, 1, nullptr);
    }
    bool failed = false;
    for (uint32_t c = 0; c < nchunks; ++c) {
      uint64_t t = t0 + c;
      Slot& s = slots_[t % N];
      uint32_t st = wait_done(s, deadline);
      uint32_t m = std::min(R, n - c * R);
      if (st == DONE) std::memcpy(out + (size_t)c * R * W, out_ptr(t % N), (size_t)m * W * 4);
      else failed = true;
      s.turn.store(t + N, std::memory_order_release);  // hand the slot to the next lap
      s.state.store(FREE, std::memory_order_release);
      h_->completions.fetch_add(1);  // producers waiting for this slot's turn sleep there too
      if (h_->sleepers.load()) futex(&h_->completions, FUTEX_WAKE, INT_MAX, nullptr);
    }
    if (failed) throw std::runtime_error("ring: the GPU owner failed this request");
  }

  // ---- owner -------------------------------------------------------------------------------
  // Gather up to max_rows rows of READY slots (same op, ticket order) into dst [max_rows, d], as
  // batch `set` (0 or 1: the owner keeps one batch on the device while it gathers the next).
  // Waits up to timeout_ms for the first slot (timeout_ms <= 0: one look, no wait), then up to
  // window_us for more.  Returns (rows, op); rows == 0 on timeout.
  std::pair<uint32_t, uint32_t> collect(float* dst, uint32_t max_rows, double window_us, double timeout_ms,
                                        int set) {
    const uint32_t N = h_->nslots, d = h_->d;
    std::vector<Taken>& taken_ = taken_sets_[set & 1];
    taken_.clear();
    uint64_t t = h_->tail.load(std::memory_order_relaxed);
    if (timeout_ms <= 0) {
      Slot& s0 = slots_[t % N];
      if (!(s0.turn.load(std::memory_order_acquire) == t && s0.state.load(std::memory_order_acquire) == READY))
        return {0, 0};
    } else if (!wait_ready(slots_[t % N], t, now_ns() + (uint64_t)(timeout_ms * 1e6))) {
      return {0, 0};
    }
    const uint32_t op = slots_[t % N].op;
    uint32_t rows = 0;
    const uint64_t wdl = now_ns() + (uint64_t)(window_us * 1e3);
    while (true) {
      Slot& s = slots_[t % N];
      bool ready = s.turn.load(std::memory_order_acquire) == t && s.state.load(std::memory_order_acquire) == READY;
      if (!ready) {
        if (rows > 0 && now_ns() >= wdl) break;
        if (h_->head.load(std::memory_order_acquire) <= t && now_ns() >= wdl) break;
        cpu_relax();
        continue;
      }
      if (s.op != op || rows + s.n_rows > max_rows) break;
      std::memcpy(dst + (size_t)rows * d, in_ptr(t % N), (size_t)s.n_rows * d * 4);
      s.state.store(TAKEN, std::memory_order_relaxed);
      taken_.push_back({t, rows, s.n_rows});
      rows += s.n_rows;
      ++t;
      if (rows == max_rows) break;
      if (window_us <= 0 && !(slots_[t % N].turn.load() == t && slots_[t % N].state.load() == READY)) break;
    }
    h_->tail.store(t, std::memory_order_release);
    return {rows, op};
  }

  // Scatter the batch results: column-major pieces prob[rows], logit[rows], phi[rows][dphi]
  // (any may be null) into each taken slot's [n][out_w] rows, then one completion wake.
  void complete(const float* prob, const float* logit, const float* phi, uint32_t dphi, bool ok, int set) {
    const uint32_t N = h_->nslots, W = h_->out_w;
    std::vector<Taken>& taken_ = taken_sets_[set & 1];
    uint64_t rows = 0;
    for (const Taken& tk : taken_) {
      Slot& s = slots_[tk.ticket % N];
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
      s.state.store(ok ? DONE : FAILED, std::memory_order_release);
      rows += tk.n;
    }
    h_->batches.fetch_add(1);
    h_->rows.fetch_add(rows);
    h_->slots_done.fetch_add(taken_.size());
    taken_.clear();
    h_->completions.fetch_add(1, std::memory_order_seq_cst);
    if (h_->sleepers.load(std::memory_order_seq_cst)) futex(&h_->completions, FUTEX_WAKE, INT_MAX, nullptr);
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
  void wait_turn(Slot& s, uint64_t t, uint64_t deadline) {
    if (!sleep_until([&] { return s.turn.load(std::memory_order_acquire) == t && s.state.load() == FREE; },
                     deadline))
      throw std::runtime_error(owner_gone() ? "ring: GPU owner stopped" : "ring: timed out waiting for a free slot");
  }
  uint32_t wait_done(Slot& s, uint64_t deadline) {
    auto fin = [&] {
      uint32_t st = s.state.load(std::memory_order_acquire);
      return st == DONE || st == FAILED;
    };
    if (!sleep_until(fin, deadline)) return FAILED;
    return s.state.load(std::memory_order_acquire);
  }
  bool wait_ready(Slot& s, uint64_t t, uint64_t deadline) {
    auto rdy = [&] {
      return s.turn.load(std::memory_order_acquire) == t && s.state.load(std::memory_order_acquire) == READY;
    };
    for (int i = 0; i < 512; ++i) {
      if (rdy()) return true;
      cpu_relax();
    }
    while (!rdy()) {
      uint64_t now = now_ns();
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
    return true;
  }

  std::string path_;
  size_t bytes_ = 0;
  char* base_ = nullptr;
  Header* h_ = nullptr;
  Slot* slots_ = nullptr;
  std::vector<Taken> taken_sets_[2];
  bool owns_ = true;
};

}  // namespace
}  // namespace fdx_ring
