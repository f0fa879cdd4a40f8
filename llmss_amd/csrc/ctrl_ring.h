// Shared-memory control ring: the serving driver's leader -> follower channel on one node. The protocol lives here
// with no Python dependency, so tests/native/ctrl_host_test.cpp can build it alone under AddressSanitizer +
// UndefinedBehaviorSanitizer and under ThreadSanitizer; csrc/ctrl.cpp binds it into llmss_amd._C.
//
// Reference: the consumer broadcasts a pickled request list with dist.broadcast_object_list on every
// poll iteration (poc-server/producer-consumer/consumer_server.py:75-111), i.e. a collective round trip
// per step over the GPU communicator. serving/driver.py sends one control record per engine step (the
// new requests / aborts of that step, or an empty header); over gloo TCP that record costs ~0.1-0.3 ms
// per step at 2-8 ranks (profiles/r3_ctrl). All ranks of a tensor-parallel replica live on one node
// (xGMI), so the records go through a POSIX shared-memory ring instead:
//   * single producer (the leader), R readers (the followers), a byte ring of fixed capacity;
//   * records are [u32 len | u32 flags | bytes, padded to 8]; a message longer than a quarter of the
//     ring travels as several fragments (flag MORE on all but the last) and is reassembled by recv();
//   * the producer publishes with one release store of write_pos; each reader owns a cache line with
//     its read position (release store after it has copied the record out); the producer only waits when
//     the slowest reader is a whole ring behind;
//   * waits spin briefly, then sleep with a growing back-off (an idle follower costs ~no CPU), and give
//     up after the caller's timeout (a dead leader / follower surfaces as TimeoutError, not a hang);
//   * the leader unlinks the name as soon as every follower has attached (attach count in the header),
//     so a crash leaves nothing behind in /dev/shm.
#pragma once

#include <errno.h>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>

namespace llmss_ctrl {

constexpr uint64_t kMagic = 0x6c6c6d7373637472ULL;  // "llmssctr"
constexpr int kMaxReaders = 64;
constexpr uint32_t kMore = 1u;

struct alignas(64) Line {
  std::atomic<uint64_t> v;
  char pad[64 - sizeof(std::atomic<uint64_t>)];
};

struct RingHeader {
  std::atomic<uint64_t> magic;  // published last (release) by the creator
  uint64_t capacity;            // bytes of the data area (power of two)
  uint32_t nreaders;
  int32_t producer_pid;  // readers give up at once when this process is gone
  Line attached;         // followers that mapped the ring
  Line write_pos;        // bytes published (monotonic)
  Line closed;           // producer gone (orderly)
  Line read_pos[kMaxReaders];
};

struct Timeout : std::runtime_error {
  using std::runtime_error::runtime_error;
};

inline double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

inline void cpu_relax() {
#if defined(__x86_64__) || defined(__i386__)
  __builtin_ia32_pause();
#endif
}

// Waiting for a record: pause-spin for the first 50 us (a follower that is in step with its leader),
// then sched_yield up to 5 ms (a step or two late: still wakes within microseconds), then sleep 50 us ..
// 1 ms doubling (an idle replica costs ~no CPU); returns false once `deadline` has passed.
class Backoff {
 public:
  explicit Backoff(double timeout_s) : t0_(now_s()), deadline_(timeout_s < 0 ? -1.0 : t0_ + timeout_s) {}
  bool wait() {
    ++n_;
    if ((n_ & 63) != 0 && phase_ == 0) {
      cpu_relax();
      return true;
    }
    const double t = now_s();
    if (deadline_ >= 0 && t > deadline_) return false;
    const double waited = t - t0_;
    if (waited < 50e-6) {
      cpu_relax();
    } else if (waited < 5e-3) {
      phase_ = 1;
      sched_yield();
    } else {
      phase_ = 2;
      struct timespec ts{0, sleep_ns_};
      nanosleep(&ts, nullptr);
      if (sleep_ns_ < 1000000) sleep_ns_ *= 2;
    }
    return true;
  }
  bool sleeping() const { return phase_ == 2; }

 private:
  double t0_, deadline_;
  long n_ = 0;
  int phase_ = 0;
  long sleep_ns_ = 50000;
};

// false once `pid` has exited (also while it is an unreaped zombie of a parent that has not waited yet)
inline bool process_alive(int pid) {
  if (kill(pid, 0) != 0 && errno == ESRCH) return false;
  char path[64];
  snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  FILE* f = fopen(path, "r");
  if (f == nullptr) return true;  // no procfs: only the kill() probe
  char buf[256];
  const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');  // "pid (comm) S ..."
  return !(rp != nullptr && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X'));
}

// The protocol on one mapping of the ring (header + data area): the producer's or one reader's end.
class RingView {
 public:
  RingView() = default;
  RingView(RingHeader* h, bool producer, int reader)
      : h_(h), data_(reinterpret_cast<char*>(h) + sizeof(RingHeader)), mask_(h->capacity - 1), producer_(producer),
        reader_(reader) {
    if (!producer_) pos_ = h_->read_pos[reader].v.load(std::memory_order_acquire);
  }

  void send(const std::string& msg, double timeout_s) {
    if (!producer_) throw std::runtime_error("CtrlRing: send() on a reader");
    const uint64_t frag_max = h_->capacity / 4 - 8;
    size_t off = 0;
    do {
      const size_t n = std::min<size_t>(msg.size() - off, frag_max);
      const uint32_t flags = off + n < msg.size() ? kMore : 0u;
      put(msg.data() + off, (uint32_t)n, flags, timeout_s);
      off += n;
    } while (off < msg.size());
  }

  // next message; throws Timeout after timeout_s (< 0: forever). A message split into fragments is assembled in
  // pend_, which survives a timeout between fragments: the next recv() resumes it instead of returning its tail
  // as a message of its own.
  std::string recv(double timeout_s) {
    if (producer_) throw std::runtime_error("CtrlRing: recv() on the producer");
    for (;;) {
      Backoff b(timeout_s);
      unsigned polls = 0;
      while (h_->write_pos.v.load(std::memory_order_acquire) <= pos_) {
        // closed: records published before the close still drain (the close store follows them, so an
        // acquire reload of write_pos after seeing it observes every one of them)
        if (h_->closed.v.load(std::memory_order_acquire)) {
          if (h_->write_pos.v.load(std::memory_order_acquire) > pos_) break;
          throw std::runtime_error("CtrlRing: producer closed");
        }
        if (!b.wait()) throw Timeout("CtrlRing: timed out");
        if (b.sleeping() && ++polls % 64 == 0 && !process_alive(h_->producer_pid))
          throw std::runtime_error("CtrlRing: producer process died");
      }
      uint32_t hdr[2];
      copy_out(pos_, reinterpret_cast<char*>(hdr), 8);
      const uint32_t len = hdr[0], flags = hdr[1];
      if ((uint64_t)len + 8 > h_->capacity) throw std::runtime_error("CtrlRing: corrupt record header");
      const size_t at = pend_.size();
      pend_.resize(at + len);
      copy_out(pos_ + 8, &pend_[at], len);
      pos_ += rec_bytes(len);
      h_->read_pos[reader_].v.store(pos_, std::memory_order_release);
      if (!(flags & kMore)) break;
    }
    std::string out;
    out.swap(pend_);
    return out;
  }

  // producer: orderly end (readers blocked in recv() raise instead of timing out)
  void close_producer() {
    if (producer_ && h_ != nullptr) h_->closed.v.store(1, std::memory_order_release);
  }

 private:
  static uint64_t rec_bytes(uint32_t len) { return 8 + (((uint64_t)len + 7) & ~7ULL); }

  void put(const char* src, uint32_t len, uint32_t flags, double timeout_s) {
    const uint64_t need = rec_bytes(len);
    const uint64_t wp = h_->write_pos.v.load(std::memory_order_relaxed);
    Backoff b(timeout_s);
    for (;;) {  // the slowest reader must have consumed enough of the ring
      uint64_t lo = wp;
      for (uint32_t r = 0; r < h_->nreaders; ++r) lo = std::min(lo, h_->read_pos[r].v.load(std::memory_order_acquire));
      if (wp + need - lo <= h_->capacity) break;
      if (!b.wait()) throw Timeout("CtrlRing: timed out");
    }
    const uint32_t hdr[2] = {len, flags};
    copy_in(wp, reinterpret_cast<const char*>(hdr), 8);
    copy_in(wp + 8, src, len);
    h_->write_pos.v.store(wp + need, std::memory_order_release);
  }

  void copy_in(uint64_t pos, const char* src, size_t n) {
    const uint64_t at = pos & mask_;
    const size_t first = std::min<size_t>(n, h_->capacity - at);
    std::memcpy(data_ + at, src, first);
    if (n > first) std::memcpy(data_, src + first, n - first);
  }
  void copy_out(uint64_t pos, char* dst, size_t n) const {
    const uint64_t at = pos & mask_;
    const size_t first = std::min<size_t>(n, h_->capacity - at);
    std::memcpy(dst, data_ + at, first);
    if (n > first) std::memcpy(dst + first, data_, n - first);
  }

  RingHeader* h_ = nullptr;
  char* data_ = nullptr;
  uint64_t mask_ = 0;
  bool producer_ = false;
  int reader_ = 0;
  uint64_t pos_ = 0;  // reader position
  std::string pend_;  // reader: fragments of a message not yet complete (kept across a recv() timeout)
};

// The named POSIX shared-memory ring: the producer creates and initialises it, readers attach by name.
class CtrlRing {
 public:
  // producer: create (name must be fresh); reader: attach as reader `reader` (0 .. nreaders-1)
  CtrlRing(const std::string& name, bool create, int64_t capacity, int nreaders, int reader)
      : name_(name), producer_(create) {
    if (name.empty() || name[0] != '/') throw std::invalid_argument("CtrlRing: name must start with '/'");
    if (create) {
      if (nreaders < 1 || nreaders > kMaxReaders) throw std::invalid_argument("CtrlRing: 1..64 readers");
      uint64_t cap = 1 << 16;
      while (cap < (uint64_t)capacity) cap <<= 1;
      int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("CtrlRing: shm_open(create) failed for " + name);
      bytes_ = sizeof(RingHeader) + cap;
      if (ftruncate(fd, (off_t)bytes_) != 0) {
        close(fd);
        shm_unlink(name.c_str());
        throw std::runtime_error("CtrlRing: ftruncate failed");
      }
      map(fd);
      h_->capacity = cap;
      h_->nreaders = (uint32_t)nreaders;
      h_->producer_pid = (int32_t)getpid();
      h_->attached.v.store(0);
      h_->write_pos.v.store(0);
      h_->closed.v.store(0);
      for (int i = 0; i < kMaxReaders; ++i) h_->read_pos[i].v.store(0);
      h_->magic.store(kMagic, std::memory_order_release);
      linked_ = true;
    } else {
      int fd = shm_open(name.c_str(), O_RDWR, 0600);
      if (fd < 0) throw std::runtime_error("CtrlRing: shm_open(attach) failed for " + name);
      struct stat st;
      if (fstat(fd, &st) != 0 || (size_t)st.st_size < sizeof(RingHeader)) {
        close(fd);
        throw std::runtime_error("CtrlRing: bad ring size");
      }
      bytes_ = (size_t)st.st_size;
      map(fd);
      if (h_->magic.load(std::memory_order_acquire) != kMagic) {
        unmap();
        throw std::runtime_error("CtrlRing: ring not initialised");
      }
      if (reader < 0 || reader >= (int)h_->nreaders) {
        unmap();
        throw std::invalid_argument("CtrlRing: bad reader index");
      }
      if (bytes_ != sizeof(RingHeader) + h_->capacity) {
        unmap();
        throw std::runtime_error("CtrlRing: size mismatch");
      }
      h_->attached.v.fetch_add(1, std::memory_order_acq_rel);
    }
    view_ = RingView(h_, create, create ? 0 : reader);
  }
  ~CtrlRing() { close_ring(); }
  CtrlRing(const CtrlRing&) = delete;
  CtrlRing& operator=(const CtrlRing&) = delete;

  // producer: wait until every reader attached (then the name can go), or timeout
  bool wait_attached(double timeout_s) {
    Backoff b(timeout_s);
    while (h_->attached.v.load(std::memory_order_acquire) < h_->nreaders)
      if (!b.wait()) return false;
    unlink();
    return true;
  }

  void unlink() {
    if (linked_) {
      shm_unlink(name_.c_str());
      linked_ = false;
    }
  }

  void send(const std::string& msg, double timeout_s) { view_.send(msg, timeout_s); }
  std::string recv(double timeout_s) { return view_.recv(timeout_s); }
  void close_producer() { view_.close_producer(); }

  int64_t capacity() const { return (int64_t)h_->capacity; }
  int nreaders() const { return (int)h_->nreaders; }
  int attached() const { return (int)h_->attached.v.load(); }

 private:
  void map(int fd) {
    void* p = mmap(nullptr, bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) throw std::runtime_error("CtrlRing: mmap failed");
    h_ = reinterpret_cast<RingHeader*>(p);
  }
  void unmap() {
    munmap(h_, bytes_);
    h_ = nullptr;
  }

  void close_ring() {
    if (h_ == nullptr) return;
    if (producer_) view_.close_producer();
    unlink();
    unmap();
  }

  std::string name_;
  bool producer_;
  bool linked_ = false;
  RingHeader* h_ = nullptr;
  size_t bytes_ = 0;
  RingView view_;
};

}  // namespace llmss_ctrl
