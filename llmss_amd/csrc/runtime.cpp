// Native host runtime for the serving engine (part of module llmss_amd._C).
//
//   * BlockAllocator  - paged KV-cache block pool (free stack + ref counts).
//   * Scheduler       - continuous-batching scheduler: FCFS admission of prefills under a token /
//                       sequence / free-block budget, then one decode token for every running
//                       sequence; when the pool runs dry the newest running sequence is preempted
//                       (blocks freed, re-queued at the front, recomputed later). It emits the
//                       flat step metadata the kernels consume (positions, slot mapping, padded
//                       block tables, context lengths) so Python never loops over tokens.
//   * SafetensorsFile - mmap'ed .safetensors reader that copies tensor-parallel shards (row or
//                       column slices) with several threads straight into caller memory (pinned
//                       host staging buffers), reading only the bytes of the shard.
//
// Reference: the reference has no scheduler at all - one request at a time, batch_size = 1,
// a spinning broadcast_object_list when idle (consumer_server.py:73-111), and a KV cache grown by
// torch.cat (gptj_modeling.py:229-236); weights via safetensors' Python safe_open
// (utils/weights.py:9-115).
#include <fcntl.h>
#ifndef LLMSS_HOST_TEST  // tests/native builds this file alone (no Python) under ASan/UBSan
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#endif
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <deque>
#include <map>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#ifndef LLMSS_HOST_TEST
namespace py = pybind11;
#endif

// ============================================================================ BlockAllocator
class BlockAllocator {
 public:
  BlockAllocator(int num_blocks, int block_size) : num_blocks_(num_blocks), block_size_(block_size), ref_(num_blocks, 0) {
    if (num_blocks <= 0 || block_size <= 0) throw std::invalid_argument("BlockAllocator: bad sizes");
    free_.reserve(num_blocks);
    for (int i = num_blocks - 1; i >= 0; --i) free_.push_back(i);
  }
  int num_free() const { return (int)free_.size(); }
  int num_blocks() const { return num_blocks_; }
  int block_size() const { return block_size_; }
  bool can_allocate(int n) const { return n <= (int)free_.size(); }
  int allocate() {
    if (free_.empty()) throw std::runtime_error("BlockAllocator: out of blocks");
    int b = free_.back();
    free_.pop_back();
    ref_[b] = 1;
    return b;
  }
  std::vector<int> allocate_n(int n) {
    if (!can_allocate(n)) throw std::runtime_error("BlockAllocator: out of blocks");
    std::vector<int> out;
    out.reserve(n);
    for (int i = 0; i < n; ++i) out.push_back(allocate());
    return out;
  }
  void fork(int b) {  // share a block (copy-on-write style prefix sharing)
    check(b);
    if (ref_[b] <= 0) throw std::runtime_error("BlockAllocator: fork of a free block");
    ++ref_[b];
  }
  void free(int b) {
    check(b);
    if (ref_[b] <= 0) throw std::runtime_error("BlockAllocator: double free of block " + std::to_string(b));
    if (--ref_[b] == 0) free_.push_back(b);
  }
  void free_all(const std::vector<int>& bs) {
    for (int b : bs) free(b);
  }
  int ref_count(int b) const {
    check(b);
    return ref_[b];
  }

 private:
  void check(int b) const {
    if (b < 0 || b >= num_blocks_) throw std::out_of_range("BlockAllocator: bad block id");
  }
  int num_blocks_, block_size_;
  std::vector<int> ref_;
  std::vector<int> free_;
};

// ============================================================================ Scheduler
struct SeqState {
  int64_t id;
  int prompt_len;
  int max_new;
  int num_tokens;    // prompt + generated tokens known
  int num_computed;  // tokens whose K/V are in the cache (scheduled into a step)
  std::vector<int> blocks;
  int status;  // 0 waiting, 1 running, 2 finished
  int64_t order;
  int preemptions = 0;
};

struct StepBatch {
  int kind = 0;        // 0 idle, 1 extend (prefill chunks, optionally mixed with decodes), 2 decode only
  int num_decode = 0;  // kind 1: items [0, num_decode) are single-token decodes, the rest prompt chunks
  std::vector<int64_t> ids;
  std::vector<int> query_lens;  // new tokens fed this step per sequence
  std::vector<int> ctx_lens;    // KV length after this step per sequence
  std::vector<uint8_t> sample;  // the step completes the sequence's known tokens -> sample one
  std::vector<int64_t> positions;
  std::vector<int64_t> slots;
  std::vector<int> block_table;  // [B, max_blocks] padded with 0
  int max_blocks = 0;
  std::vector<int64_t> preempted;
};

// Continuous batching with chunked prefill. Every step spends a budget of max_batched_tokens:
//   1. one token for every running sequence that is decoding (oldest first); when the KV pool runs
//      dry the newest running sequence is preempted (blocks freed, recomputed later);
//   2. the next chunk of every partially prefilled running sequence;
//   3. FCFS admission of waiting prompts, each with as much of its prompt as the budget allows
//      (prefill_chunk > 0 caps one chunk; prefill_chunk < 0 keeps prompts whole).
// Decodes therefore never stall behind a long prompt (the prompt is cut into chunks that ride along
// with the decode tokens), and a chunk's attention reads its own prefix from the paged cache.
class Scheduler {
 public:
  Scheduler(int num_blocks, int block_size, int max_num_seqs, int max_batched_tokens, int max_model_len,
            int prefill_chunk = 0)
      : alloc_(num_blocks, block_size),
        bs_(block_size),
        max_seqs_(max_num_seqs),
        max_tokens_(max_batched_tokens),
        max_len_(max_model_len),
        chunk_(prefill_chunk) {
    max_blocks_per_seq_ = (max_model_len + block_size - 1) / block_size;
    if (max_batched_tokens <= 0) throw std::invalid_argument("Scheduler: max_batched_tokens must be > 0");
  }

  void add(int64_t id, int prompt_len, int max_new) {
    if (seqs_.count(id)) throw std::invalid_argument("Scheduler.add: duplicate id " + std::to_string(id));
    if (prompt_len <= 0) throw std::invalid_argument("Scheduler.add: empty prompt");
    if (prompt_len + max_new > max_len_)
      throw std::invalid_argument("Scheduler.add: prompt_len + max_new_tokens exceeds max_model_len");
    if (chunk_ < 0 && prompt_len > max_tokens_)
      throw std::invalid_argument("Scheduler.add: prompt longer than max_batched_tokens (whole-prompt mode)");
    if ((int64_t)blocks_for(prompt_len + max_new) > (int64_t)alloc_.num_blocks())
      throw std::invalid_argument("Scheduler.add: sequence needs more KV blocks than the whole pool holds");
    SeqState s{id, prompt_len, max_new, prompt_len, 0, {}, 0, counter_++};
    seqs_.emplace(id, s);
    waiting_.push_back(id);
  }

  // A token was sampled for `id` (its step had sample=1); `finished` releases its blocks.
  void on_token(int64_t id, bool finished) {
    auto& s = get(id);
    if (s.status != 1) throw std::runtime_error("Scheduler.on_token: sequence not running");
    // the sampled token's step computed every known token (a step the engine launched on its own,
    // pipelined decode, computed the last one without a schedule() call)
    if (s.num_computed < s.num_tokens - 1) throw std::runtime_error("Scheduler.on_token: sequence still prefilling");
    s.num_computed = s.num_tokens;
    s.num_tokens += 1;
    if (finished || s.num_tokens - s.prompt_len >= s.max_new) finish(id);
  }

  // Batched on_token for a whole step (one call instead of one per sequence).
  void on_tokens(const int64_t* ids, const bool* finished, int64_t n) {
    for (int64_t i = 0; i < n; ++i) on_token(ids[i], finished[i]);
  }

  void finish(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return;
    auto& s = it->second;
    alloc_.free_all(s.blocks);
    s.blocks.clear();
    if (s.status == 1) running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    if (s.status == 0) waiting_.erase(std::remove(waiting_.begin(), waiting_.end(), id), waiting_.end());
    seqs_.erase(it);
  }

  void abort(int64_t id) { finish(id); }

  // One step. When prompt chunks hold the pool and none of them can grow while nothing decodes (the
  // chunked-prefill livelock: every step would come back empty), the newest running sequence is
  // preempted and the step re-planned, until the oldest prompt fits (add() guarantees one does).
  StepBatch schedule() {
    StepBatch b;
    for (;;) {
      bool starved = plan(b);
      if (!b.ids.empty() || !starved) break;
      int64_t victim = -1, oldest = -1;
      for (auto id : running_) {
        if (victim < 0 || get(id).order > get(victim).order) victim = id;
        if (oldest < 0 || get(id).order < get(oldest).order) oldest = id;
      }
      if (victim < 0 || victim == oldest)
        throw std::runtime_error("Scheduler: KV pool cannot hold the oldest running sequence");
      preempt(victim);
      b.preempted.push_back(victim);
    }
    if (b.ids.empty()) return b;
    b.kind = (b.num_decode == (int)b.ids.size()) ? 2 : 1;
    fill_tables(b);
    return b;
  }

  // The three stages of a step into `b`; returns true when a running prompt chunk could not get its
  // KV blocks (admission is then skipped: a new prompt would only take blocks the old one needs).
  bool plan(StepBatch& b) {
    int budget = max_tokens_;
    bool starved = false;
    std::vector<int64_t> order(running_.begin(), running_.end());
    std::sort(order.begin(), order.end(), [&](int64_t a, int64_t c) { return get(a).order < get(c).order; });
    // ---- 1. decodes
    for (size_t i = 0; i < order.size() && budget > 0; ++i) {
      auto& s = get(order[i]);
      if (s.status != 1 || s.num_tokens - s.num_computed != 1) continue;
      while ((int)s.blocks.size() * bs_ < s.num_tokens) {
        if (alloc_.can_allocate(1)) {
          s.blocks.push_back(alloc_.allocate());
          continue;
        }
        int64_t victim = -1;  // the newest running sequence (possibly s itself)
        for (size_t j = order.size(); j-- > i;) {
          if (get(order[j]).status == 1) {
            victim = order[j];
            break;
          }
        }
        preempt(victim);
        b.preempted.push_back(victim);
        if (victim == s.id) break;
      }
      if (s.status == 1) {
        emit(b, s, 1);
        budget -= 1;
      }
    }
    b.num_decode = (int)b.ids.size();
    // ---- 2. continuing prompt chunks
    for (size_t i = 0; i < order.size() && budget > 0; ++i) {
      auto& s = get(order[i]);
      if (s.status != 1 || s.num_tokens - s.num_computed <= 1) continue;
      const int q = chunk_len(s, budget);
      if (q <= 0) break;
      if (!grow(s, s.num_computed + q)) {
        starved = true;
        break;
      }
      emit(b, s, q);
      budget -= q;
    }
    // ---- 3. admission (FCFS, stop at the first prompt that does not fit)
    while (!starved && !waiting_.empty() && budget > 0 && (int)running_.size() < max_seqs_) {
      auto& s = get(waiting_.front());
      const int q = chunk_len(s, budget);  // after preemption the whole known sequence is recomputed
      if (q <= 0 || !grow(s, q)) break;
      s.status = 1;
      waiting_.pop_front();
      running_.push_back(s.id);
      emit(b, s, q);
      budget -= q;
    }
    return starved;
  }

 public:
  int num_waiting() const { return (int)waiting_.size(); }
  int num_running() const { return (int)running_.size(); }
  // running sequences with prompt tokens still to compute (the next step is not a pure decode)
  int num_prefilling() const {
    int n = 0;
    for (auto id : running_) {
      const auto& s = seqs_.at(id);
      n += (s.num_tokens - s.num_computed) > 1;
    }
    return n;
  }
  int num_free_blocks() const { return alloc_.num_free(); }
  int max_blocks_per_seq() const { return max_blocks_per_seq_; }
  bool has_work() const { return !waiting_.empty() || !running_.empty(); }
  // Blocks for `n_tokens` cached tokens of a running sequence ahead of its schedule() (the engine's pipelined
  // decode launches the next step before the scheduler runs: a sequence entering a new KV block needs that
  // block now). No preemption; returns the block holding token n_tokens - 1, or -1 when the pool is empty
  // or the sequence is gone (aborted while its step was in flight).
  // schedule() later finds the block already there.
  int reserve(int64_t id, int n_tokens) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) return -1;  // finished / aborted meanwhile: nothing to reserve for
    auto& s = it->second;
    if (s.status != 1 || n_tokens <= 0 || blocks_for(n_tokens) > max_blocks_per_seq_ || !grow(s, n_tokens)) return -1;
    return s.blocks[(n_tokens - 1) / bs_];
  }
  int num_tokens(int64_t id) { return get(id).num_tokens; }
  int num_computed(int64_t id) { return get(id).num_computed; }
  std::vector<int> blocks(int64_t id) { return get(id).blocks; }
  bool contains(int64_t id) const { return seqs_.count(id) > 0; }

 private:
  SeqState& get(int64_t id) {
    auto it = seqs_.find(id);
    if (it == seqs_.end()) throw std::out_of_range("Scheduler: unknown sequence " + std::to_string(id));
    return it->second;
  }
  int blocks_for(int n) const { return (n + bs_ - 1) / bs_; }
  int64_t slot(const SeqState& s, int p) const { return (int64_t)s.blocks[p / bs_] * bs_ + p % bs_; }
  int chunk_len(const SeqState& s, int budget) const {
    const int rem = s.num_tokens - s.num_computed;
    if (chunk_ < 0) return rem <= budget ? rem : 0;  // whole prompts only
    int q = std::min(rem, budget);
    if (chunk_ > 0) q = std::min(q, chunk_);
    return q;
  }
  bool grow(SeqState& s, int n_tokens) {  // blocks for n_tokens cached tokens, no preemption
    const int need = blocks_for(n_tokens) - (int)s.blocks.size();
    if (need <= 0) return true;
    if (!alloc_.can_allocate(need)) return false;
    for (int i = 0; i < need; ++i) s.blocks.push_back(alloc_.allocate());
    return true;
  }
  void emit(StepBatch& b, SeqState& s, int q) {
    const int p0 = s.num_computed;
    b.ids.push_back(s.id);
    b.query_lens.push_back(q);
    b.ctx_lens.push_back(p0 + q);
    for (int p = p0; p < p0 + q; ++p) {
      b.positions.push_back(p);
      b.slots.push_back(slot(s, p));
    }
    s.num_computed = p0 + q;
    b.sample.push_back(s.num_computed == s.num_tokens ? 1 : 0);
  }
  void preempt(int64_t id) {
    auto& s = get(id);
    alloc_.free_all(s.blocks);
    s.blocks.clear();
    s.num_computed = 0;
    s.status = 0;
    s.preemptions++;
    running_.erase(std::remove(running_.begin(), running_.end(), id), running_.end());
    waiting_.push_front(id);
  }
  void fill_tables(StepBatch& b) {
    const int B = (int)b.ids.size();
    b.max_blocks = max_blocks_per_seq_;
    b.block_table.assign((size_t)B * b.max_blocks, 0);
    for (int i = 0; i < B; ++i) {
      const auto& s = get(b.ids[i]);
      std::copy(s.blocks.begin(), s.blocks.end(), b.block_table.begin() + (size_t)i * b.max_blocks);
    }
  }

  BlockAllocator alloc_;
  int bs_, max_seqs_, max_tokens_, max_len_, max_blocks_per_seq_, chunk_;
  std::unordered_map<int64_t, SeqState> seqs_;
  std::deque<int64_t> waiting_;
  std::vector<int64_t> running_;
  int64_t counter_ = 0;
};

// ============================================================================ safetensors
// Minimal JSON reader for the safetensors header: {"name": {"dtype": "...", "shape": [...],
// "data_offsets": [a, b]}, ..., "__metadata__": {"k": "v"}}.
struct TensorInfo {
  std::string dtype;
  std::vector<int64_t> shape;
  int64_t begin = 0, end = 0;
};

class JsonCursor {
 public:
  explicit JsonCursor(const std::string& s) : s_(s) {}
  void ws() {
    while (i_ < s_.size() && isspace((unsigned char)s_[i_])) ++i_;
  }
  char peek() {
    ws();
    if (i_ >= s_.size()) throw std::runtime_error("safetensors header: unexpected end");
    return s_[i_];
  }
  void expect(char c) {
    if (peek() != c) throw std::runtime_error(std::string("safetensors header: expected ") + c);
    ++i_;
  }
  std::string str() {
    expect('"');
    std::string out;
    while (i_ < s_.size() && s_[i_] != '"') {
      if (s_[i_] == '\\') {
        ++i_;
        if (i_ >= s_.size()) break;
        char c = s_[i_];
        if (c == 'u') {  // keep escaped code points verbatim (names are ASCII in practice)
          out += "\\u";
        } else {
          out += c == 'n' ? '\n' : c == 't' ? '\t' : c;
        }
      } else {
        out += s_[i_];
      }
      ++i_;
    }
    expect('"');
    return out;
  }
  int64_t integer() {
    ws();
    size_t j = i_;
    if (j < s_.size() && (s_[j] == '-' || s_[j] == '+')) ++j;
    while (j < s_.size() && isdigit((unsigned char)s_[j])) ++j;
    int64_t v = std::stoll(s_.substr(i_, j - i_));
    i_ = j;
    return v;
  }
  void skip_value() {
    char c = peek();
    if (c == '"') {
      str();
    } else if (c == '{') {
      expect('{');
      if (peek() == '}') {
        ++i_;
        return;
      }
      while (true) {
        str();
        expect(':');
        skip_value();
        if (peek() == ',') {
          ++i_;
          continue;
        }
        expect('}');
        break;
      }
    } else if (c == '[') {
      expect('[');
      if (peek() == ']') {
        ++i_;
        return;
      }
      while (true) {
        skip_value();
        if (peek() == ',') {
          ++i_;
          continue;
        }
        expect(']');
        break;
      }
    } else {
      while (i_ < s_.size() && s_[i_] != ',' && s_[i_] != '}' && s_[i_] != ']') ++i_;
    }
  }
  size_t pos() const { return i_; }
  void advance() { ++i_; }

 private:
  const std::string& s_;
  size_t i_ = 0;
};

static int dtype_size_or0(const std::string& d) {
  if (d == "F64" || d == "I64" || d == "U64") return 8;
  if (d == "F32" || d == "I32" || d == "U32") return 4;
  if (d == "F16" || d == "BF16" || d == "I16" || d == "U16") return 2;
  if (d == "I8" || d == "U8" || d == "BOOL" || d == "F8_E4M3" || d == "F8_E5M2") return 1;
  return 0;
}
static int dtype_size(const std::string& d) {
  const int n = dtype_size_or0(d);
  if (!n) throw std::runtime_error("safetensors: unsupported dtype " + d);
  return n;
}

class SafetensorsFile {
 public:
  explicit SafetensorsFile(const std::string& path) : path_(path) {
    // the destructor does not run when the constructor throws: release the fd and the mapping here
    try {
      open_and_parse(path);
    } catch (...) {
      release();
      throw;
    }
  }
  ~SafetensorsFile() { release(); }
  SafetensorsFile(const SafetensorsFile&) = delete;
  SafetensorsFile& operator=(const SafetensorsFile&) = delete;
  std::vector<std::string> keys() const {
    std::vector<std::string> k;
    for (auto& kv : tensors_) k.push_back(kv.first);
    return k;
  }
  const TensorInfo& info(const std::string& name) const { return at(name); }
  std::map<std::string, std::string> metadata() const { return meta_; }

  // Copy rows [start, stop) along `dim` (0 or 1) of tensor `name` into dst (contiguous).
  void copy_slice(const std::string& name, int dim, int64_t start, int64_t stop, uintptr_t dst, int threads) {
    const auto& t = at(name);
    const int es = dtype_size(t.dtype);
    const char* src = data_ + t.begin;
    char* out = reinterpret_cast<char*>(dst);
    if (t.shape.empty()) {
      std::memcpy(out, src, es);
      return;
    }
    int64_t inner = es;
    for (size_t i = 1; i < t.shape.size(); ++i) inner *= t.shape[i];
    if (dim == 0) {
      if (start < 0 || stop > t.shape[0] || start > stop) throw std::out_of_range("copy_slice: bad range");
      parallel_copy(out, src + start * inner, (stop - start) * inner, threads);
      return;
    }
    if (dim != 1 || t.shape.size() < 2) throw std::invalid_argument("copy_slice: dim must be 0 or 1");
    int64_t inner2 = es;
    for (size_t i = 2; i < t.shape.size(); ++i) inner2 *= t.shape[i];
    if (start < 0 || stop > t.shape[1] || start > stop) throw std::out_of_range("copy_slice: bad range");
    const int64_t rows = t.shape[0], row_bytes = t.shape[1] * inner2, seg = (stop - start) * inner2;
    const int nt = std::max(1, std::min<int>(threads, (int)rows));
    std::vector<std::thread> pool;
    for (int w = 0; w < nt; ++w) {
      pool.emplace_back([=]() {
        for (int64_t r = w; r < rows; r += nt) std::memcpy(out + r * seg, src + r * row_bytes + start * inner2, seg);
      });
    }
    for (auto& th : pool) th.join();
  }
  int64_t nbytes(const std::string& name) const {
    const auto& t = at(name);
    return t.end - t.begin;
  }

 private:
  void open_and_parse(const std::string& path) {
    fd_ = ::open(path.c_str(), O_RDONLY);
    if (fd_ < 0) throw std::runtime_error("safetensors: cannot open " + path);
    struct stat st;
    if (fstat(fd_, &st) != 0) throw std::runtime_error("safetensors: cannot stat " + path);
    size_ = st.st_size;
    if (size_ < 8) throw std::runtime_error("safetensors: file too small");
    const void* m = mmap(nullptr, size_, PROT_READ, MAP_PRIVATE, fd_, 0);
    if (m == MAP_FAILED) throw std::runtime_error("safetensors: mmap failed");
    map_ = (const char*)m;
    uint64_t hlen;
    std::memcpy(&hlen, map_, 8);
    if (hlen > (uint64_t)size_ - 8) throw std::runtime_error("safetensors: bad header length");  // no 8 + hlen wrap
    data_ = map_ + 8 + hlen;
    std::string header(map_ + 8, hlen);
    parse(header);
  }
  void release() {
    if (map_) munmap((void*)map_, size_);
    map_ = nullptr;
    if (fd_ >= 0) ::close(fd_);
    fd_ = -1;
  }
  static void parallel_copy(char* dst, const char* src, int64_t n, int threads) {
    const int64_t chunk = 8 << 20;
    if (threads <= 1 || n < 2 * chunk) {
      std::memcpy(dst, src, n);
      return;
    }
    const int nt = std::min<int64_t>(threads, (n + chunk - 1) / chunk);
    std::vector<std::thread> pool;
    const int64_t per = (n + nt - 1) / nt;
    for (int w = 0; w < nt; ++w) {
      const int64_t b = w * per, e = std::min(n, b + per);
      if (b >= e) break;
      pool.emplace_back([=]() { std::memcpy(dst + b, src + b, e - b); });
    }
    for (auto& th : pool) th.join();
  }
  const TensorInfo& at(const std::string& name) const {
    auto it = tensors_.find(name);
    if (it == tensors_.end()) throw std::out_of_range("safetensors: no tensor " + name);
    return it->second;
  }
  void parse(const std::string& h) {
    JsonCursor c(h);
    c.expect('{');
    if (c.peek() == '}') return;
    while (true) {
      std::string key = c.str();
      c.expect(':');
      if (key == "__metadata__") {
        c.expect('{');
        if (c.peek() != '}') {
          while (true) {
            std::string k = c.str();
            c.expect(':');
            if (c.peek() == '"') meta_[k] = c.str();
            else c.skip_value();
            if (c.peek() == ',') { c.advance(); continue; }
            break;
          }
        }
        c.expect('}');
      } else {
        TensorInfo t;
        c.expect('{');
        while (true) {
          std::string f = c.str();
          c.expect(':');
          if (f == "dtype") {
            t.dtype = c.str();
          } else if (f == "shape") {
            c.expect('[');
            if (c.peek() != ']') {
              while (true) {
                t.shape.push_back(c.integer());
                if (c.peek() == ',') { c.advance(); continue; }
                break;
              }
            }
            c.expect(']');
          } else if (f == "data_offsets") {
            c.expect('[');
            t.begin = c.integer();
            c.expect(',');
            t.end = c.integer();
            c.expect(']');
          } else {
            c.skip_value();
          }
          if (c.peek() == ',') { c.advance(); continue; }
          break;
        }
        c.expect('}');
        if (t.begin < 0 || t.end < t.begin || (int64_t)(data_ - map_) + t.end > size_)
          throw std::runtime_error("safetensors: tensor " + key + " out of file bounds");
        int64_t numel = 1;
        for (int64_t d : t.shape) {
          if (d < 0 || (d > 0 && numel > INT64_MAX / d)) throw std::runtime_error("safetensors: bad shape of " + key);
          numel *= d;
        }
        const int es = dtype_size_or0(t.dtype);  // unknown dtypes fail on access instead
        if (es && (numel > INT64_MAX / 8 || numel * es != t.end - t.begin))  // copy_slice trusts shape x dtype
          throw std::runtime_error("safetensors: shape/dtype of " + key + " disagree with its data_offsets");
        tensors_[key] = t;
      }
      if (c.peek() == ',') { c.advance(); continue; }
      break;
    }
    c.expect('}');
  }

  std::string path_;
  int fd_ = -1;
  int64_t size_ = 0;
  const char* map_ = nullptr;
  const char* data_ = nullptr;
  std::map<std::string, TensorInfo> tensors_;
  std::map<std::string, std::string> meta_;
};

// ============================================================================ bindings
#ifndef LLMSS_HOST_TEST
template <typename T>
static py::array_t<T> to_np(const std::vector<T>& v) {
  py::array_t<T> a(v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

void register_runtime(py::module_& m) {
  py::class_<BlockAllocator>(m, "BlockAllocator")
      .def(py::init<int, int>(), py::arg("num_blocks"), py::arg("block_size"))
      .def("num_free", &BlockAllocator::num_free)
      .def("num_blocks", &BlockAllocator::num_blocks)
      .def("block_size", &BlockAllocator::block_size)
      .def("can_allocate", &BlockAllocator::can_allocate)
      .def("allocate", &BlockAllocator::allocate)
      .def("allocate_n", &BlockAllocator::allocate_n)
      .def("fork", &BlockAllocator::fork)
      .def("free", &BlockAllocator::free)
      .def("free_all", &BlockAllocator::free_all)
      .def("ref_count", &BlockAllocator::ref_count);

  py::class_<StepBatch>(m, "StepBatch")
      .def_readonly("kind", &StepBatch::kind)
      .def_readonly("num_decode", &StepBatch::num_decode)
      .def_readonly("max_blocks", &StepBatch::max_blocks)
      .def_property_readonly("sample", [](const StepBatch& b) {
        py::array_t<bool> a((ssize_t)b.sample.size());
        for (size_t i = 0; i < b.sample.size(); ++i) a.mutable_data()[i] = b.sample[i] != 0;
        return a;
      })
      .def_property_readonly("ids", [](const StepBatch& b) { return to_np(b.ids); })
      .def_property_readonly("query_lens", [](const StepBatch& b) { return to_np(b.query_lens); })
      .def_property_readonly("ctx_lens", [](const StepBatch& b) { return to_np(b.ctx_lens); })
      .def_property_readonly("positions", [](const StepBatch& b) { return to_np(b.positions); })
      .def_property_readonly("slots", [](const StepBatch& b) { return to_np(b.slots); })
      .def_property_readonly("block_table",
                             [](const StepBatch& b) {
                               auto a = to_np(b.block_table);
                               const ssize_t B = (ssize_t)b.ids.size();
                               a.resize({B, (ssize_t)b.max_blocks});
                               return a;
                             })
      .def_property_readonly("preempted", [](const StepBatch& b) { return to_np(b.preempted); });

  py::class_<Scheduler>(m, "Scheduler")
      .def(py::init<int, int, int, int, int, int>(), py::arg("num_blocks"), py::arg("block_size"),
           py::arg("max_num_seqs"), py::arg("max_batched_tokens"), py::arg("max_model_len"),
           py::arg("prefill_chunk") = 0)
      .def("add", &Scheduler::add)
      .def("on_token", &Scheduler::on_token)
      .def("on_tokens",
           [](Scheduler& sc, py::array_t<int64_t, py::array::c_style | py::array::forcecast> ids,
              py::array_t<bool, py::array::c_style | py::array::forcecast> fin) {
             if (ids.size() != fin.size()) throw std::invalid_argument("Scheduler.on_tokens: length mismatch");
             sc.on_tokens(ids.data(), fin.data(), ids.size());
           })
      .def("finish", &Scheduler::finish)
      .def("abort", &Scheduler::abort)
      .def("schedule", &Scheduler::schedule)
      .def("num_waiting", &Scheduler::num_waiting)
      .def("num_running", &Scheduler::num_running)
      .def("num_prefilling", &Scheduler::num_prefilling)
      .def("num_computed", &Scheduler::num_computed)
      .def("num_free_blocks", &Scheduler::num_free_blocks)
      .def("max_blocks_per_seq", &Scheduler::max_blocks_per_seq)
      .def("has_work", &Scheduler::has_work)
      .def("num_tokens", &Scheduler::num_tokens)
      .def("reserve", &Scheduler::reserve)
      .def("blocks", &Scheduler::blocks)
      .def("contains", &Scheduler::contains);

  py::class_<SafetensorsFile>(m, "SafetensorsFile")
      .def(py::init<const std::string&>())
      .def("keys", &SafetensorsFile::keys)
      .def("info",
           [](const SafetensorsFile& f, const std::string& name) {
             const auto& t = f.info(name);
             return py::make_tuple(t.dtype, t.shape, t.begin, t.end);
           })
      .def("metadata", &SafetensorsFile::metadata)
      .def("nbytes", &SafetensorsFile::nbytes)
      .def("copy_slice", &SafetensorsFile::copy_slice, py::arg("name"), py::arg("dim"), py::arg("start"),
           py::arg("stop"), py::arg("dst"), py::arg("threads") = 8);
}
#endif  // LLMSS_HOST_TEST
