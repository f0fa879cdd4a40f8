// Host-only test of the native runtime (csrc/runtime.cpp without its Python bindings), built and run
// under AddressSanitizer + UndefinedBehaviorSanitizer by tests/test_native_asan.py.
// Exercises the KV block allocator, the continuous-batching scheduler (admission, decode, block
// growth, preemption by recompute, finish/abort) and the safetensors reader (row / column shard
// copies, multi-threaded, malformed headers rejected).
#define LLMSS_HOST_TEST 1
#include "../../llmss_amd/csrc/runtime.cpp"

#include <cstdio>
#include <fstream>
#include <set>

#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      std::exit(1);                                                \
    }                                                              \
  } while (0)

template <typename F>
static bool throws(F f) {
  try {
    f();
  } catch (const std::exception&) {
    return true;
  }
  return false;
}

static void test_allocator() {
  BlockAllocator a(8, 16);
  auto bs = a.allocate_n(8);
  CHECK(a.num_free() == 0 && !a.can_allocate(1));
  CHECK(std::set<int>(bs.begin(), bs.end()).size() == 8);
  a.fork(bs[0]);
  a.free(bs[0]);
  CHECK(a.ref_count(bs[0]) == 1 && a.num_free() == 0);
  a.free_all(bs);
  CHECK(a.num_free() == 8);
  CHECK(throws([&] { a.free(bs[1]); }));   // double free
  CHECK(throws([&] { a.free(99); }));      // bad id
}

static void test_scheduler() {
  // 12 blocks of 4 tokens, up to 4 sequences, 64 batched tokens, max length 32
  Scheduler s(12, 4, 4, 64, 32);
  for (int i = 0; i < 4; ++i) s.add(i, 5 + i, 12);
  CHECK(throws([&] { s.add(0, 3, 1); }));   // duplicate id
  CHECK(throws([&] { s.add(9, 30, 10); })); // exceeds max_model_len
  auto b = s.schedule();
  CHECK(b.kind == 1);
  int64_t total = 0;
  for (auto q : b.query_lens) total += q;
  CHECK((int64_t)b.positions.size() == total && b.slots.size() == b.positions.size());
  std::vector<int64_t> ids(b.ids.begin(), b.ids.end());
  std::vector<char> fin(ids.size(), 0);
  s.on_tokens(ids.data(), reinterpret_cast<const bool*>(fin.data()), (int64_t)ids.size());
  int preempted = 0, steps = 0;
  while (s.has_work() && steps < 200) {
    auto d = s.schedule();
    ++steps;
    preempted += (int)d.preempted.size();
    if (d.kind == 0) break;
    CHECK((int64_t)d.block_table.size() == (int64_t)d.ids.size() * d.max_blocks);
    for (size_t i = 0; i < d.slots.size(); ++i) CHECK(d.slots[i] >= 0 && d.slots[i] < 12 * 4);
    std::vector<int64_t> di(d.ids.begin(), d.ids.end());
    std::vector<char> df(di.size(), 0);
    if (steps == 3 && !di.empty()) df[0] = 1;  // one sequence stops early (eos)
    s.on_tokens(di.data(), reinterpret_cast<const bool*>(df.data()), (int64_t)di.size());
  }
  CHECK(!s.has_work());
  CHECK(preempted > 0);  // 4 x up-to-23 tokens cannot fit 48 slots at once
  CHECK(s.num_free_blocks() == 12);
  s.add(20, 4, 4);
  s.abort(20);
  CHECK(!s.has_work() && s.num_free_blocks() == 12);
}

static void write_file(const std::string& path, const std::string& header, const std::vector<char>& data) {
  std::ofstream f(path, std::ios::binary);
  uint64_t n = header.size();
  f.write(reinterpret_cast<const char*>(&n), 8);
  f.write(header.data(), header.size());
  f.write(data.data(), data.size());
}

static void test_safetensors(const std::string& dir) {
  // t: int32 [6, 5] = row * 10 + col
  std::vector<char> data(6 * 5 * 4);
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 5; ++c) {
      int32_t v = r * 10 + c;
      std::memcpy(&data[(r * 5 + c) * 4], &v, 4);
    }
  const std::string p = dir + "/ok.safetensors";
  write_file(p, R"({"__metadata__":{"format":"pt"},"t":{"dtype":"I32","shape":[6,5],"data_offsets":[0,120]}})", data);
  SafetensorsFile f(p);
  CHECK(f.keys().size() == 1 && f.metadata().at("format") == "pt");
  std::vector<int32_t> rows(2 * 5), cols(6 * 2);
  f.copy_slice("t", 0, 2, 4, reinterpret_cast<uintptr_t>(rows.data()), 4);
  for (int r = 0; r < 2; ++r)
    for (int c = 0; c < 5; ++c) CHECK(rows[r * 5 + c] == (r + 2) * 10 + c);
  f.copy_slice("t", 1, 3, 5, reinterpret_cast<uintptr_t>(cols.data()), 3);
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 2; ++c) CHECK(cols[r * 2 + c] == r * 10 + c + 3);
  CHECK(throws([&] { f.copy_slice("t", 0, 4, 7, reinterpret_cast<uintptr_t>(rows.data()), 1); }));
  CHECK(throws([&] { f.copy_slice("nope", 0, 0, 1, reinterpret_cast<uintptr_t>(rows.data()), 1); }));
  // malformed: offsets past the end, shape larger than the bytes, truncated header
  const std::string bad1 = dir + "/bad1.safetensors", bad2 = dir + "/bad2.safetensors", bad3 = dir + "/bad3.safetensors";
  write_file(bad1, R"({"t":{"dtype":"I32","shape":[6,5],"data_offsets":[0,4000]}})", data);
  write_file(bad2, R"({"t":{"dtype":"I32","shape":[600,5],"data_offsets":[0,120]}})", data);
  write_file(bad3, R"({"t":{"dtype":"I32","shape":[6,)", data);
  CHECK(throws([&] { SafetensorsFile x(bad1); }));
  CHECK(throws([&] { SafetensorsFile x(bad2); }));
  CHECK(throws([&] { SafetensorsFile x(bad3); }));
  // a header length near 2^64 must be rejected (8 + hlen would wrap), not reach std::string
  {
    std::ofstream f(dir + "/bad4.safetensors", std::ios::binary);
    uint64_t n = ~uint64_t(0) - 3;
    f.write(reinterpret_cast<const char*>(&n), 8);
    f.write(data.data(), data.size());
  }
  CHECK(throws([&] { SafetensorsFile x(dir + "/bad4.safetensors"); }));
  // a throwing constructor must not leak its fd / mapping: far more failures than the fd limit
  for (int i = 0; i < 3000; ++i) {
    CHECK(throws([&] { SafetensorsFile x(bad1); }));
    CHECK(throws([&] { SafetensorsFile x(dir + "/bad4.safetensors"); }));
  }
  SafetensorsFile again(p);  // fds still available
  CHECK(again.keys().size() == 1);
}

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "/tmp";
  test_allocator();
  test_scheduler();
  test_safetensors(dir);
  std::printf("ALL OK\n");
  return 0;
}
