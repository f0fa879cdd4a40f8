// Host-only stress of the shared-memory control ring protocol (llmss_amd/csrc/ctrl_ring.h), built by
// tests/test_native_asan.py twice: under AddressSanitizer + UndefinedBehaviorSanitizer and under ThreadSanitizer.
//   threads   one producer and R readers as threads on ONE mapping (so TSan sees every access of the protocol):
//             messages of 0 .. 3/4 of the ring (fragmented past a quarter), wrap-around, a slow reader that
//             the producer must wait for, content and order verified by every reader
//   timeout   recv() on an empty ring and send() into a ring a reader never drains both time out
//   procs     producer and reader in two processes through the named ring (fork), orderly close at the end
//   dead      the producer process exits in the middle of a fragmented message: the reader gets the messages
//             published before it, then an error naming the dead producer - no hang, no partial message
// usage: ctrl_host_test [threads|timeout|procs|dead|all]; prints "ALL OK" on success.
#include <sys/wait.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <thread>
#include <vector>

#include "../../llmss_amd/csrc/ctrl_ring.h"

using namespace llmss_ctrl;

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

static uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  return x;
}

// message i: deterministic length and bytes, so a reader can verify without a side channel
static std::string make_msg(int i, uint64_t cap) {
  const size_t len = (size_t)(mix((uint64_t)i * 7919 + 1) % (cap * 3 / 4));
  std::string s(len, '\0');
  for (size_t k = 0; k < len; ++k) s[k] = (char)(mix((uint64_t)i * 131 + k) & 0xff);
  return s;
}

struct HeapRing {
  RingHeader* h;
  explicit HeapRing(uint64_t cap, int nreaders) {
    void* p = aligned_alloc(64, sizeof(RingHeader) + cap);
    CHECK(p != nullptr);
    memset(p, 0, sizeof(RingHeader) + cap);
    h = new (p) RingHeader();
    h->capacity = cap;
    h->nreaders = (uint32_t)nreaders;
    h->producer_pid = (int32_t)getpid();
    h->magic.store(kMagic, std::memory_order_release);
  }
  ~HeapRing() {
    h->~RingHeader();
    free(h);
  }
};

static void test_threads() {
  const uint64_t cap = 1 << 16;
  const int R = 3, N = 400;
  HeapRing ring(cap, R);
  std::vector<std::thread> readers;
  std::vector<int> ok(R, 0);
  for (int r = 0; r < R; ++r) {
    readers.emplace_back([&, r] {
      RingView v(ring.h, false, r);
      for (int i = 0; i < N; ++i) {
        std::string m = v.recv(30.0);
        if (m != make_msg(i, cap)) {
          fprintf(stderr, "reader %d: message %d differs (len %zu vs %zu)\n", r, i, m.size(), make_msg(i, cap).size());
          return;
        }
        if (r == R - 1 && i % 16 == 0) std::this_thread::sleep_for(std::chrono::milliseconds(2));  // slow reader
      }
      bool closed = false;
      try {
        v.recv(30.0);
      } catch (const Timeout&) {
      } catch (const std::runtime_error&) {
        closed = true;  // "producer closed" after the last record drained
      }
      ok[r] = closed ? 1 : 0;
    });
  }
  RingView prod(ring.h, true, 0);
  uint64_t bytes = 0;
  for (int i = 0; i < N; ++i) {
    const std::string m = make_msg(i, cap);
    bytes += m.size();
    prod.send(m, 30.0);
  }
  prod.close_producer();
  for (auto& t : readers) t.join();
  for (int r = 0; r < R; ++r) CHECK(ok[r] == 1);
  CHECK(bytes > 20 * cap);  // wrapped many times
  printf("threads ok (%d readers, %d messages, %.1f MB)\n", R, N, bytes / 1e6);
}

static void test_timeout() {
  const uint64_t cap = 1 << 16;
  HeapRing ring(cap, 1);
  RingView rd(ring.h, false, 0), prod(ring.h, true, 0);
  bool timed_out = false;
  try {
    rd.recv(0.02);
  } catch (const Timeout&) {
    timed_out = true;
  }
  CHECK(timed_out);
  // fill the ring: the reader never reads, so the producer must give up
  timed_out = false;
  try {
    for (int i = 0; i < 64; ++i) prod.send(std::string(cap / 8, 'x'), 0.02);
  } catch (const Timeout&) {
    timed_out = true;
  }
  CHECK(timed_out);
  // everything published before the stall is still intact
  std::string m = rd.recv(1.0);
  CHECK(m == std::string(cap / 8, 'x'));
  printf("timeout ok\n");
}

static std::string ring_name(const char* tag) {
  char b[96];
  snprintf(b, sizeof b, "/llmss_ctrl_test_%s_%d", tag, (int)getpid());
  return b;
}

static void test_procs() {
  const std::string name = ring_name("procs");
  const int N = 300;
  const uint64_t cap = 1 << 16;
  CtrlRing prod(name, true, (int64_t)cap, 1, 0);
  const pid_t pid = fork();
  CHECK(pid >= 0);
  if (pid == 0) {  // reader process
    int rc = 0;
    try {
      CtrlRing rd(name, false, 0, 0, 0);
      for (int i = 0; i < N && rc == 0; ++i)
        if (rd.recv(30.0) != make_msg(i, cap)) rc = 2;
      if (rc == 0) {
        try {
          rd.recv(30.0);
          rc = 3;
        } catch (const Timeout&) {
          rc = 4;
        } catch (const std::runtime_error&) {
        }
      }
    } catch (const std::exception& e) {
      fprintf(stderr, "reader: %s\n", e.what());
      rc = 5;
    }
    _exit(rc);
  }
  CHECK(prod.wait_attached(30.0));
  for (int i = 0; i < N; ++i) prod.send(make_msg(i, cap), 30.0);
  prod.close_producer();
  int st = 0;
  CHECK(waitpid(pid, &st, 0) == pid);
  CHECK(WIFEXITED(st) && WEXITSTATUS(st) == 0);
  printf("procs ok\n");
}

static void test_dead_producer() {
  const std::string name = ring_name("dead");
  const uint64_t cap = 1 << 16;
  const pid_t pid = fork();
  CHECK(pid >= 0);
  if (pid == 0) {  // producer process: two whole messages, then dies inside a fragmented third
    CtrlRing prod(name, true, (int64_t)cap, 1, 0);
    if (!prod.wait_attached(30.0)) _exit(7);
    prod.send("first", 5.0);
    prod.send(std::string(100, 'y'), 5.0);
    // then messages of 3 fragments each (half a ring) until a helper thread ends the process at an arbitrary
    // point - typically between two fragments of one message
    const std::string big(cap / 2, 'z');
    std::thread killer([] {
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
      _exit(0);
    });
    try {
      for (;;) prod.send(big, 5.0);
    } catch (...) {
    }
    killer.join();
    _exit(0);
  }
  // reader: attach once the name exists
  CtrlRing* rd = nullptr;
  for (int i = 0; i < 3000 && rd == nullptr; ++i) {
    try {
      rd = new CtrlRing(name, false, 0, 0, 0);
    } catch (const std::exception&) {
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
    }
  }
  CHECK(rd != nullptr);
  CHECK(rd->recv(10.0) == "first");
  CHECK(rd->recv(10.0) == std::string(100, 'y'));
  bool died = false;
  long whole = 0;
  // whole messages may keep arriving until the producer is gone; the one it was inside when it died must never
  // come out truncated: recv() ends with an error naming the dead producer
  try {
    for (;;) {
      std::string m = rd->recv(20.0);
      CHECK(m == std::string(cap / 2, 'z'));
      ++whole;
    }
  } catch (const Timeout&) {
    fprintf(stderr, "dead producer: timed out instead of noticing the exit\n");
  } catch (const std::runtime_error& e) {
    died = std::string(e.what()).find("died") != std::string::npos;
    if (!died) fprintf(stderr, "dead producer: unexpected error %s\n", e.what());
  }
  int st = 0;
  CHECK(waitpid(pid, &st, 0) == pid);
  delete rd;
  shm_unlink(name.c_str());  // the dead producer could not unlink (it had: wait_attached unlinks; harmless)
  CHECK(died);
  printf("dead ok (%ld whole messages before the exit)\n", whole);
}

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "all";
  if (which == "threads" || which == "all") test_threads();
  if (which == "timeout" || which == "all") test_timeout();
  if (which == "procs" || which == "all") test_procs();
  if (which == "dead" || which == "all") test_dead_producer();
  printf("ALL OK\n");
  return 0;
}
