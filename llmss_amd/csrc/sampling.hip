// Fused token sampler (reference: rank-0-only argmax / softmax+multinomial with
// HF TopP/TopK/Temperature warpers that are never applied because of an inverted condition,
// generate.py:109-126, consumer_server.py:130-147 - quirk Q1; here the documented intent is
// implemented: temperature -> top-k -> top-p -> sample).
//
// One workgroup (1024 threads) per row; logits are re-read from L2 per pass (a row is
// 64-256 KB). Thresholds by 4-pass 8-bit radix select on order-preserving float keys:
// counts for top-k, exp-mass for top-p. Sampling is Gumbel-max (argmax of x/T + Gumbel noise
// over the kept set), which draws exactly from the renormalised filtered softmax without a
// prefix sum. Noise is Philox-4x32-10 keyed by the per-row 64-bit seed and counted by token
// index, so every tensor-parallel rank - which holds the same all-gathered logits - draws the
// same token with no broadcast (reference broadcasts the sampled token every step, C7/C11).
#include "common.h"
#include <cstdlib>

__device__ __forceinline__ unsigned fkey(float f) {  // order-preserving (ascending) uint key
  unsigned u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

__device__ __forceinline__ unsigned philox(unsigned c0, unsigned c1, unsigned k0, unsigned k1) {
  unsigned c2 = 0, c3 = 0;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const unsigned long long p0 = (unsigned long long)0xD2511F53u * c0;
    const unsigned long long p1 = (unsigned long long)0xCD9E8D57u * c2;
    const unsigned h0 = p0 >> 32, l0 = (unsigned)p0, h1 = p1 >> 32, l1 = (unsigned)p1;
    const unsigned n0 = h1 ^ c1 ^ k0, n2 = h0 ^ c3 ^ k1;
    c0 = n0; c1 = l1; c2 = n2; c3 = l0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return c0;
}

template <typename T>
__device__ __forceinline__ float load_logit(const T* p, int i);
template <>
__device__ __forceinline__ float load_logit<bf16_t>(const bf16_t* p, int i) { return bf2f(p[i]); }
template <>
__device__ __forceinline__ float load_logit<float>(const float* p, int i) { return p[i]; }

// Find the largest key threshold thr such that the "weight" of elements with key >= thr is
// >= target. mode 0: weight = count (top-k), mode 1: weight = exp(x - mx) (top-p).
template <typename T>
__device__ unsigned radix_select(const T* row, int V, float scale, float mx, unsigned min_key, float target, int mode,
                                 float* hist, float* red) {
  unsigned prefix = 0, mask = 0;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0.f;
    __syncthreads();
    for (int i = threadIdx.x; i < V; i += blockDim.x) {
      const float x = load_logit(row, i) * scale;
      const unsigned k = fkey(x);
      if (k >= min_key && (k & mask) == prefix) {
        const float wgt = mode == 0 ? 1.f : __expf(x - mx);
        atomicAdd(&hist[(k >> shift) & 255], wgt);
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float cum = 0.f;
      int d = 255;
      for (; d > 0; --d) {
        if (cum + hist[d] >= target) break;
        cum += hist[d];
      }
      red[0] = __int_as_float(d);
      red[1] = target - cum;
    }
    __syncthreads();
    const int d = __float_as_int(red[0]);
    target = red[1];
    prefix |= (unsigned)d << shift;
    mask |= 255u << shift;
    __syncthreads();
  }
  return prefix;
}

template <typename T>
__global__ __launch_bounds__(1024) void sample_kernel(const T* __restrict__ logits, int64_t ld, int V,
                                                      const float* __restrict__ temperature,
                                                      const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                      const int64_t* __restrict__ seeds, int64_t* __restrict__ out,
                                                      int64_t* __restrict__ out2) {
  __shared__ float hist[256];
  __shared__ float red[32];
  __shared__ int redi[32];
  const int b = blockIdx.x;
  const T* row = logits + b * ld;
  const float temp = temperature ? temperature[b] : 0.f;
  const int k = top_k ? top_k[b] : 0;
  const float p = top_p ? top_p[b] : 1.f;
  const bool greedy = !(temp > 0.f) || k == 1;
  const float scale = greedy ? 1.f : 1.f / temp;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;

  // max
  float mx = -INFINITY;
  for (int i = threadIdx.x; i < V; i += blockDim.x) mx = fmaxf(mx, load_logit(row, i) * scale);
  mx = block_max(mx, red);

  unsigned thr = 0;
  if (!greedy) {
    if (k > 0 && k < V) thr = radix_select(row, V, scale, mx, 0u, (float)k, 0, hist, red);
    if (p < 1.f) {
      float z = 0.f;
      for (int i = threadIdx.x; i < V; i += blockDim.x) {
        const float x = load_logit(row, i) * scale;
        if (fkey(x) >= thr) z += __expf(x - mx);
      }
      __syncthreads();
      z = block_sum(z, red);
      const unsigned tp = radix_select(row, V, scale, mx, thr, p * z, 1, hist, red);
      thr = tp > thr ? tp : thr;
    }
  }
  // argmax of (x + gumbel) over kept tokens (greedy: plain argmax, lowest index on ties)
  const unsigned long long seed = seeds ? (unsigned long long)seeds[b] : 0ull;
  const unsigned s0 = (unsigned)seed, s1 = (unsigned)(seed >> 32);
  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int i = threadIdx.x; i < V; i += blockDim.x) {
    const float x = load_logit(row, i) * scale;
    float v = x;
    if (!greedy) {
      if (fkey(x) < thr) continue;
      const unsigned r = philox((unsigned)i, (unsigned)b * 0u, s0, s1);
      const float u = ((float)(r >> 8) + 0.5f) * (1.0f / 16777216.0f);
      v = x - __logf(-__logf(u));
    }
    if (v > best || (v == best && i < besti)) { best = v; besti = i; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
  }
  __syncthreads();
  if (lane == 0) { red[wid] = best; redi[wid] = besti; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float bb = red[0];
    int bi = redi[0];
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i)
      if (red[i] > bb || (red[i] == bb && redi[i] < bi)) { bb = red[i]; bi = redi[i]; }
    if (bi >= V) bi = 0;  // all -inf / NaN row
    out[b] = bi;
    if (out2) out2[b] = bi;
  }
}

// ---------------------------------------------------------------------------------------------
// v3 (bf16 logits, 16-B aligned rows, V <= 1024 * 8 * CPT). The row is read once into registers.
// Thresholds: ONE histogram pass over the distance to the row max (2048 bins of 1/32 logit; the
// last bin collects everything >= 64 below the max), then an exact rank selection among the few
// elements of the boundary bin only (gathered into LDS). Probability mass is accumulated as
// 2^-32 fixed-point integers, so every sum is order-independent: all TP ranks (same all-gathered
// logits) derive bit-identical thresholds and draw the same token without any broadcast - v1's
// float LDS atomics did not guarantee that. More than SV3_MAXC elements tied within 1/32 logit at
// the boundary (pathological) keeps the whole bin.
// ---------------------------------------------------------------------------------------------
constexpr int SV3_BINS = 2048;
constexpr int SV3_MAXC = 2048;
constexpr int SV3_SORT_MIN = 128;  // boundary bins with more candidates are sorted (sv3_sort), fewer ranked all-pairs

struct Sv3Smem {
  unsigned cnt[SV3_BINS];
  unsigned long long mass[SV3_BINS];
  float cv[SV3_MAXC];
  int ci[SV3_MAXC];
  unsigned long long wtot[16];
  float red[32];
  int redi[32];
  int ncand;
  int bin;
  unsigned long long excl;
  unsigned long long acc;
  float thr;
};

__device__ __forceinline__ int sv3_bin(float e, float mx) {
  const float d = (mx - e) * 32.f;
  return d < 2047.f ? (int)d : 2047;
}
__device__ __forceinline__ unsigned long long sv3_mass(float e, float mx) {
  return (unsigned long long)(__expf(e - mx) * 4294967296.f);
}

// First bin b < limit whose inclusive prefix of arr reaches target; sm.bin / sm.excl (prefix
// before b). 1024 threads x 2 bins. If the total never reaches target: bin = limit - 1.
template <typename T>
__device__ void sv3_find(const T* arr, unsigned long long target, int limit, Sv3Smem& sm) {
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const unsigned long long a0 = 2 * t < limit ? (unsigned long long)arr[2 * t] : 0ull;
  const unsigned long long a1 = 2 * t + 1 < limit ? (unsigned long long)arr[2 * t + 1] : 0ull;
  const unsigned long long loc = a0 + a1;
  unsigned long long inc = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  if (t == 0) { sm.bin = limit - 1; sm.excl = 0; }
  if (lane == 63) sm.wtot[wid] = inc;
  __syncthreads();
  unsigned long long off = 0;
  for (int w = 0; w < wid; ++w) off += sm.wtot[w];
  const unsigned long long e0 = off + inc - loc, e1 = e0 + a0;
  if (e0 < target && e0 + a0 >= target) { sm.bin = 2 * t; sm.excl = e0; }
  else if (e1 < target && e1 + a1 >= target) { sm.bin = 2 * t + 1; sm.excl = e1; }
  __syncthreads();
}

// Sort the boundary bin's n candidates (sm.cv / sm.ci) into rank order - value descending, index ascending, the
// strict order the selection uses - with a bitonic network over the next power of two (<= SV3_MAXC, padding
// -inf / INT_MAX sorts last). O(n log^2 n) work in log^2 barrier steps: the rank selections below then read
// position r - 1 (top-k) and an integer prefix scan (top-p) instead of comparing every candidate with every
// other one, which took 100-170 us per call on a flat top-p row (n ~ 1-2 K; bench/sampler_bench.py).
__device__ __attribute__((noinline)) void sv3_sort(Sv3Smem& sm, int n) {
  int P = 1;
  while (P < n) P <<= 1;
  for (int i = n + (int)threadIdx.x; i < P; i += blockDim.x) { sm.cv[i] = -INFINITY; sm.ci[i] = 0x7fffffff; }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < (P >> 1); t += blockDim.x) {
        const int i = 2 * t - (t & (j - 1)), l = i + j;
        const float vi = sm.cv[i], vl = sm.cv[l];
        const int ii = sm.ci[i], il = sm.ci[l];
        const bool l_first = vl > vi || (vl == vi && il < ii);
        if (l_first == ((i & k) == 0)) {
          sm.cv[i] = vl; sm.cv[l] = vi;
          sm.ci[i] = il; sm.ci[l] = ii;
        }
      }
      __syncthreads();
    }
  }
}

// LROW: the packed row lives in LDS instead of VGPRs. At CPT = 8 (vocab 32K-57K, e.g. GPT-2's
// padded 50304) a register-resident row exceeds the 128-VGPR budget of a 1024-thread block: the
// compiler spills to scratch and the kernel takes ~100 us per call even for argmax; every pass
// over the row re-reads it from LDS (ds_read_b128, conflict-free lane-linear chunks) instead.
constexpr int SV3_LROW_CHUNKS = 7168;  // 112 KiB row + ~40 KiB Sv3Smem < 160 KiB LDS

template <int CPT, bool LROW>
__global__ __launch_bounds__(1024) void sample_v3_kernel(const bf16_t* __restrict__ logits, int64_t ld, int V,
                                                         const float* __restrict__ temperature,
                                                         const int* __restrict__ top_k, const float* __restrict__ top_p,
                                                         const int64_t* __restrict__ seeds, int64_t* __restrict__ out,
                                                         int64_t* __restrict__ out2) {
  __shared__ Sv3Smem sm;
  __shared__ __attribute__((aligned(16))) u16x8 srow[LROW ? SV3_LROW_CHUNKS : 1];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int lane = tid & 63, wid = tid >> 6;
  const bf16_t* row = logits + b * ld;
  const float temp = temperature ? temperature[b] : 0.f;
  const int k = top_k ? top_k[b] : 0;
  const float p = top_p ? top_p[b] : 1.f;
  const bool greedy = !(temp > 0.f) || k == 1;
  const float scale = greedy ? 1.f : 1.f / temp;

  // the row stays packed (bf16) in registers; X(i) = scaled logit of element slot i, -inf past V
  u16x8 raw[LROW ? 1 : CPT];
#pragma unroll
  for (int c = 0; c < CPT; ++c) {
    const int ch = tid + c * 1024;
    const u16x8 v = ch * 8 < V ? *reinterpret_cast<const u16x8*>(row + ch * 8) : u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if constexpr (LROW) {
      if (ch < SV3_LROW_CHUNKS) srow[ch] = v;
    } else {
      raw[c] = v;
    }
  }
  if constexpr (LROW) __syncthreads();
#define CHUNK(c) (LROW ? srow[tid + (c) * 1024] : raw[LROW ? 0 : (c)])
// element loops: FOR_ELEMS(i) { ... X(i) ... } END_ELEMS - one chunk read per 8 elements; the chunk loop
// stays rolled for an LDS row (else the compiler hoists every pass's 64 LDS values into VGPRs)
constexpr int UNR = LROW ? 1 : CPT;
#define FOR_ELEMS(i)                                 \
  _Pragma("unroll UNR") for (int c_ = 0; c_ < CPT; ++c_) { \
    const u16x8 rc_ = CHUNK(c_);                     \
    _Pragma("unroll") for (int j_ = 0; j_ < 8; ++j_) { \
      const int i = c_ * 8 + j_;
#define END_ELEMS }}
#define X(i) (((tid + ((i) >> 3) * 1024) * 8 + ((i) & 7) < V) ? bf2f(rc_[(i) & 7]) * scale : -INFINITY)
  float thr = -INFINITY;
  if (!greedy) {
    float mx = -INFINITY;
    FOR_ELEMS(i) mx = fmaxf(mx, X(i)); END_ELEMS
    mx = block_max(mx, sm.red);
    const bool do_k = k > 0 && k < V, do_p = p < 1.f;
    if (do_k || do_p) {
      for (int i = tid; i < SV3_BINS; i += 1024) { sm.cnt[i] = 0u; sm.mass[i] = 0ull; }
      __syncthreads();
FOR_ELEMS(i) {
        const float xi = X(i);
        if (xi > -INFINITY) {
          const int bn = sv3_bin(xi, mx);
          atomicAdd(&sm.cnt[bn], 1u);
          if (do_p) atomicAdd(&sm.mass[bn], sv3_mass(xi, mx));
        }
      } END_ELEMS
      __syncthreads();
    }
    int bk = SV3_BINS;  // top-k boundary bin (bins > bk are cut)
    unsigned long long kept_bk = 0;
    if (do_k) {
      sv3_find(sm.cnt, (unsigned long long)k, SV3_BINS, sm);
      bk = sm.bin;
      const int r = k - (int)sm.excl;  // 1-based rank of the k-th largest inside bin bk
      if (tid == 0) { sm.ncand = 0; sm.acc = 0; }
      __syncthreads();
FOR_ELEMS(i) {
        const float xi = X(i);
        if (xi > -INFINITY && sv3_bin(xi, mx) == bk) {
          const int slot = atomicAdd(&sm.ncand, 1);
          if (slot < SV3_MAXC) { sm.cv[slot] = xi; sm.ci[slot] = (tid + (i >> 3) * 1024) * 8 + (i & 7); }
        }
      } END_ELEMS
      __syncthreads();
      const int n = sm.ncand;
      if (n > SV3_MAXC) {  // pathological tie mass: keep the whole bin
        thr = mx - (float)(bk + 1) / 32.f;
        thr = nextafterf(thr, INFINITY);
      } else if (n > SV3_SORT_MIN) {
        sv3_sort(sm, n);
        thr = sm.cv[r - 1];  // the k-th largest (1 <= r <= n: bk holds it)
      } else {  // a few candidates: all-pairs ranks in one pass beat the sort's barrier steps
        for (int c = tid; c < n; c += 1024) {
          const float v = sm.cv[c];
          const int vi = sm.ci[c];
          int rank = 0;
          for (int c2 = 0; c2 < n; ++c2) {
            const float v2 = sm.cv[c2];
            rank += (v2 > v || (v2 == v && sm.ci[c2] < vi)) ? 1 : 0;
          }
          if (rank == r - 1) sm.thr = v;
        }
        __syncthreads();
        thr = sm.thr;
      }
      if (do_p) {  // kept mass inside the boundary bin
        for (int c = tid; c < min(n, SV3_MAXC); c += 1024)
          if (sm.cv[c] >= thr) atomicAdd(&sm.acc, sv3_mass(sm.cv[c], mx));
        __syncthreads();
        kept_bk = sm.acc;
      }
    }
    if (do_p) {
      // kept-set mass Z: full bins above bk + the kept part of bin bk
      const int limit = do_k ? bk : SV3_BINS;
      sv3_find(sm.mass, ~0ull, limit, sm);  // only for the total below `limit`
      unsigned long long z = 0;
      for (int w = 0; w < 16; ++w) z += sm.wtot[w];
      __syncthreads();
      if (do_k && tid == 0) sm.mass[bk] = kept_bk;
      __syncthreads();
      z += do_k ? kept_bk : 0ull;
      const unsigned long long target = (unsigned long long)((double)p * (double)z);
      const int lim2 = do_k ? bk + 1 : SV3_BINS;
      sv3_find(sm.mass, target < 1ull ? 1ull : target, lim2, sm);
      const int bp = sm.bin;
      const unsigned long long above = sm.excl;
      if (tid == 0) sm.ncand = 0;
      __syncthreads();
FOR_ELEMS(i) {
        const float xi = X(i);
        if (xi > -INFINITY && xi >= thr && sv3_bin(xi, mx) == bp) {
          const int slot = atomicAdd(&sm.ncand, 1);
          if (slot < SV3_MAXC) { sm.cv[slot] = xi; sm.ci[slot] = (tid + (i >> 3) * 1024) * 8 + (i & 7); }
        }
      } END_ELEMS
      __syncthreads();
      const int n = sm.ncand;
      float tp = -INFINITY;
      if (n > SV3_MAXC) {
        tp = nextafterf(mx - (float)(bp + 1) / 32.f, INFINITY);
      } else if (n > SV3_SORT_MIN) {
        // rank order, then the first candidate whose inclusive mass prefix (above + masses ranked before it +
        // its own) reaches the target; integer sums, so every rank finds the same one. The histogram is no
        // longer needed: its mass array holds the sorted candidates' masses.
        sv3_sort(sm, n);
        for (int c = tid; c < n; c += 1024) sm.mass[c] = sv3_mass(sm.cv[c], mx);
        __syncthreads();
        sv3_find(sm.mass, target - above, n, sm);
        const int c = sm.bin;
        tp = sm.excl + sm.mass[c] >= target - above ? sm.cv[c] : -INFINITY;
      } else {  // a few candidates: the same selection with all-pairs sums
        if (tid == 0) sm.thr = -INFINITY;
        __syncthreads();
        for (int c = tid; c < n; c += 1024) {
          const float v = sm.cv[c];
          const int vi = sm.ci[c];
          unsigned long long before = 0;
          for (int c2 = 0; c2 < n; ++c2) {
            const float v2 = sm.cv[c2];
            if (v2 > v || (v2 == v && sm.ci[c2] < vi)) before += sv3_mass(v2, mx);
          }
          const unsigned long long lo = above + before, hi = lo + sv3_mass(v, mx);
          if (lo < target && hi >= target) sm.thr = v;
        }
        __syncthreads();
        tp = sm.thr;
      }
      thr = fmaxf(thr, tp);
    }
  }
  // Gumbel-max over the kept set (greedy: plain argmax, lowest index on ties)
  const unsigned long long seed = seeds ? (unsigned long long)seeds[b] : 0ull;
  const unsigned s0 = (unsigned)seed, s1 = (unsigned)(seed >> 32);
  float best = -INFINITY;
  int besti = 0x7fffffff;
FOR_ELEMS(i) {
    const int idx = (tid + (i >> 3) * 1024) * 8 + (i & 7);
    float v = X(i);
    if (!(v > -INFINITY)) continue;
    if (!greedy) {
      if (v < thr) continue;
      const unsigned r = philox((unsigned)idx, 0u, s0, s1);
      const float u = ((float)(r >> 8) + 0.5f) * (1.0f / 16777216.0f);
      v = v - __logf(-__logf(u));
    }
    if (v > best || (v == best && idx < besti)) { best = v; besti = idx; }
  } END_ELEMS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
  }
  __syncthreads();
  if (lane == 0) { sm.red[wid] = best; sm.redi[wid] = besti; }
  __syncthreads();
  if (tid == 0) {
    float bb = sm.red[0];
    int bi = sm.redi[0];
    for (int i = 1; i < 16; ++i)
      if (sm.red[i] > bb || (sm.red[i] == bb && sm.redi[i] < bi)) { bb = sm.red[i]; bi = sm.redi[i]; }
    if (bi >= V) bi = 0;
    out[b] = bi;
    if (out2) out2[b] = bi;
  }
#undef X
#undef CHUNK
#undef FOR_ELEMS
#undef END_ELEMS
}

void launch_sample(const void* logits, int64_t ld, bool fp32_logits, int B, int V, const void* temperature,
                   const void* top_k, const void* top_p, const void* seeds, void* out, void* out2, hipStream_t st) {
  if (B == 0) return;
  const int chunks = (V + 7) / 8;
  if (!fp32_logits && ld % 8 == 0 && (uintptr_t)logits % 16 == 0 && chunks <= SV3_LROW_CHUNKS) {
#define SV3(CPT_, LROW_)                                                                                            \
  sample_v3_kernel<CPT_, LROW_><<<B, 1024, 0, st>>>((const bf16_t*)logits, ld, V, (const float*)temperature,      \
                                                    (const int*)top_k, (const float*)top_p, (const int64_t*)seeds, \
                                                    (int64_t*)out, (int64_t*)out2)
    // register-resident rows up to CPT 4 (LDS rows measured 2-10 % slower there, profiles/r5_sampler); CPT 8
    // would spill, so its row lives in LDS
    if (chunks <= 2048) SV3(2, false);
    else if (chunks <= 4096) SV3(4, false);
    else SV3(8, true);
#undef SV3
    HIP_CHECK_LAUNCH();
    return;
  }
  if (fp32_logits)
    sample_kernel<float><<<B, 1024, 0, st>>>((const float*)logits, ld, V, (const float*)temperature, (const int*)top_k,
                                             (const float*)top_p, (const int64_t*)seeds, (int64_t*)out, (int64_t*)out2);
  else
    sample_kernel<bf16_t><<<B, 1024, 0, st>>>((const bf16_t*)logits, ld, V, (const float*)temperature,
                                              (const int*)top_k, (const float*)top_p, (const int64_t*)seeds,
                                              (int64_t*)out, (int64_t*)out2);
  HIP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// Distributed (vocab-parallel) sampling for tensor parallelism. Reference: the LM head output is
// all-gathered as full [B, V] logits and rank 0 samples (layers.py:106-135, generate.py:109-144);
// the v3 path above still needs the gathered row. Here each rank reduces its [B, V/tp] shard to
// at most KC candidates per row (every element whose scaled logit is >= the shard's K-th largest,
// ties included), the ranks all-gather those [B, tp, KC] (value, global index) pairs - KBs instead
// of the full logits - and every rank runs the v3 selection (top-k boundary, fixed-point top-p
// mass, Philox Gumbel-max keyed by the GLOBAL token index) on the union. For greedy rows and rows
// with 1 <= top_k <= K the global kept set is inside that union, so the token equals the v3
// sampler's on the gathered row bit for bit (same mx, same masses, same noise).
// ---------------------------------------------------------------------------------------------
constexpr int CAND_THREADS = 1024;

// parallel "first digit from the top whose inclusive count reaches target" over 256 bins held in
// LDS (cnt), by the first 256 threads; writes the digit and the count strictly above it
__device__ void cand_find_digit(const unsigned* cnt, unsigned target, int* out_digit, unsigned* out_above,
                                unsigned* wsum) {
  const int t = threadIdx.x;
  unsigned v = 0, inc = 0;
  if (t < 256) {
    v = cnt[255 - t];  // descending digits
    inc = v;
    const int lane = t & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const unsigned u = __shfl_up(inc, o, 64);
      if (lane >= o) inc += u;
    }
    if (lane == 63) wsum[t >> 6] = inc;
  }
  __syncthreads();
  if (t < 256) {
    unsigned off = 0;
    for (int w = 0; w < (t >> 6); ++w) off += wsum[w];
    const unsigned excl = off + inc - v;
    if (excl < target && excl + v >= target) {
      *out_digit = 255 - t;
      *out_above = excl;
    }
  }
  __syncthreads();
}

template <int EPT>
__global__ __launch_bounds__(CAND_THREADS) void cand_topk_kernel(const bf16_t* __restrict__ logits, int64_t ld,
                                                                 int vl, int lo, int V,
                                                                 const float* __restrict__ temperature,
                                                                 const int* __restrict__ top_k, int K, int KC,
                                                                 float* __restrict__ pack, int64_t ldp) {
  __shared__ unsigned hist[256];
  __shared__ unsigned wsum[4];
  __shared__ int digit;
  __shared__ unsigned above;
  __shared__ int nout;
  const int b = blockIdx.x, t = threadIdx.x;
  // blockIdx.y = vocab shard of this launch (one GPU's [B, V] logits cut into gridDim.y shards of vl columns,
  // packed shard-major like the all-gathered packs of a vocab-parallel group); 0 for a TP rank's own shard
  lo += blockIdx.y * vl;
  pack += blockIdx.y * 2 * KC;
  const float temp = temperature ? temperature[b] : 0.f;
  const int k = top_k ? top_k[b] : 0;
  const bool greedy = !(temp > 0.f) || k == 1;
  const float scale = greedy ? 1.f : 1.f / temp;
  const bf16_t* row = logits + (int64_t)b * ld + (int64_t)blockIdx.y * vl;
  float x[EPT];
  unsigned key[EPT];
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    const int j = t + e * CAND_THREADS;
    const bool ok = j < vl && lo + j < V;
    x[e] = ok ? bf2f(row[j]) * scale : -INFINITY;
    key[e] = ok ? fkey(x[e]) : 0u;  // 0 = below every real key
  }
  // K-th largest key by 4 passes of 8-bit radix select (counts are exact integers)
  unsigned prefix = 0, mask = 0, target = (unsigned)K;
  for (int shift = 24; shift >= 0; shift -= 8) {
    if (t < 256) hist[t] = 0u;
    if (t == 0) { digit = 0; above = 0u; }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EPT; ++e)
      if (key[e] != 0u && (key[e] & mask) == prefix) atomicAdd(&hist[(key[e] >> shift) & 255], 1u);
    __syncthreads();
    cand_find_digit(hist, target, &digit, &above, wsum);
    const int d = digit;
    const unsigned a = above;
    __syncthreads();  // every thread has read digit / above before thread 0 resets them for the next pass
    target -= a;
    prefix |= (unsigned)d << shift;
    mask |= 255u << shift;
  }
  // prefix = K-th largest key (or 0 when the shard has fewer than K elements: keep all)
  if (t == 0) nout = 0;
  __syncthreads();
  const unsigned kth = prefix;
  // packed row: KC values then KC global indices (one tensor, one all-gather)
  float* ov = pack + (int64_t)b * ldp;
  int* oi = reinterpret_cast<int*>(ov + KC);
#pragma unroll
  for (int e = 0; e < EPT; ++e) {
    if (key[e] != 0u && key[e] >= kth) {
      const int s = atomicAdd(&nout, 1);
      if (s < KC) {
        ov[s] = x[e];
        oi[s] = lo + t + e * CAND_THREADS;
      }
    }
  }
  __syncthreads();
  if (nout > KC) {
    // more than KC keys tie at the boundary: the atomic slot order above kept an arbitrary subset
    // of the ties, which could drop the lowest-index one that greedy / top-k tie-breaking needs. Rewrite the
    // row deterministically: every key above the boundary (fewer than K <= KC of them), then the ties in
    // ascending vocabulary index (a ballot rank per wave + wave offsets, in (e, t) = index order).
    __shared__ int n_above, wtie[CAND_THREADS / 64], tie_base;
    if (t == 0) { n_above = 0; tie_base = 0; }
    __syncthreads();
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      if (key[e] != 0u && key[e] > kth) {
        const int s = atomicAdd(&n_above, 1);
        ov[s] = x[e];
        oi[s] = lo + t + e * CAND_THREADS;
      }
    }
    __syncthreads();
    const int room = KC - n_above;
    const int lane = t & 63, wv = t >> 6;
#pragma unroll
    for (int e = 0; e < EPT; ++e) {
      const bool tie = key[e] != 0u && key[e] == kth;
      const unsigned long long bal = __ballot(tie);
      if (lane == 0) wtie[wv] = __popcll(bal);
      __syncthreads();
      int off = tie_base;
      for (int w2 = 0; w2 < wv; ++w2) off += wtie[w2];
      const int rank = off + __popcll(bal & ((1ull << lane) - 1ull));
      if (tie && rank < room) {
        ov[n_above + rank] = x[e];
        oi[n_above + rank] = lo + t + e * CAND_THREADS;
      }
      __syncthreads();
      if (t == 0) {
        int tot = 0;
        for (int w2 = 0; w2 < CAND_THREADS / 64; ++w2) tot += wtie[w2];
        tie_base += tot;
      }
      __syncthreads();
    }
  }
  for (int s = nout + t; s < KC; s += CAND_THREADS) {  // unused slots
    ov[s] = -INFINITY;
    oi[s] = 0x7fffffff;
  }
}

constexpr int SCAND_MAX = 2048;  // gathered candidates per row (tp * KC)

__global__ __launch_bounds__(256) void sample_cand_kernel(const float* __restrict__ pack, int64_t ldp, int groups,
                                                          int KC, const float* __restrict__ temperature,
                                                          const int* __restrict__ top_k,
                                                          const float* __restrict__ top_p,
                                                          const int64_t* __restrict__ seeds,
                                                          int64_t* __restrict__ out, int64_t* __restrict__ out2) {
  __shared__ float v[SCAND_MAX];
  __shared__ int id[SCAND_MAX];
  __shared__ float sv[SCAND_MAX];  // sorted (value desc, index asc)
  __shared__ int sid[SCAND_MAX];
  __shared__ float cv[SCAND_MAX];  // candidates >= the top-k boundary (unordered)
  __shared__ int cid[SCAND_MAX];
  __shared__ unsigned hist[256];
  __shared__ unsigned wsum[4];
  __shared__ int digit_s, nkeep;
  __shared__ unsigned above_s;
  __shared__ float red[8];
  __shared__ int redi[8];
  __shared__ float thr_s;
  __shared__ int nvalid;
  const int b = blockIdx.x, t = threadIdx.x;
  const int N = groups * KC;
  const float temp = temperature ? temperature[b] : 0.f;
  const int k = top_k ? top_k[b] : 0;
  const float p = top_p ? top_p[b] : 1.f;
  const bool greedy = !(temp > 0.f) || k == 1;
  if (t == 0) nvalid = 0;
  __syncthreads();
  const float* row = pack + (int64_t)b * ldp;  // [groups][KC values | KC indices]
  int myvalid = 0;
  for (int i = t; i < N; i += 256) {
    const int g = i / KC, s = i - g * KC;
    v[i] = row[(int64_t)g * 2 * KC + s];
    id[i] = reinterpret_cast<const int*>(row)[(int64_t)g * 2 * KC + KC + s];
    myvalid += v[i] > -INFINITY ? 1 : 0;
  }
  // one LDS atomic per wave (a per-candidate atomic on one address serialised up to tp * KC updates per row)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) myvalid += __shfl_xor(myvalid, o, 64);
  if ((t & 63) == 0) atomicAdd(&nvalid, myvalid);
  __syncthreads();
  float thr = -INFINITY;
  if (!greedy) {
    float mx = -INFINITY;
    for (int i = t; i < N; i += 256) mx = fmaxf(mx, v[i]);
    mx = block_max(mx, red);
    // Only the candidates >= the k-th largest value take part in the top-k / top-p decision. Ranking every
    // candidate against every other (N^2 LDS reads, N = tp * KC = 1024 at TP=8) cost ~340 us per call; instead
    // (1) the k-th largest key by 4 passes of 8-bit radix select (exact counts, as cand_topk), (2) compact
    // the candidates at or above it (k plus ties: ~64), (3) exact ranks inside that small set.
    const int n = nvalid;
    const unsigned kk = (k > 0 && k <= n) ? (unsigned)k : 0u;  // 0: keep every real candidate
    unsigned kth = 0u;
    if (kk) {
      unsigned prefix = 0u, mask = 0u, target = kk;
      for (int shift = 24; shift >= 0; shift -= 8) {
        hist[t] = 0u;  // 256 threads, 256 bins
        if (t == 0) { digit_s = 0; above_s = 0u; }
        __syncthreads();
        for (int i = t; i < N; i += 256) {
          const unsigned key = v[i] > -INFINITY ? fkey(v[i]) : 0u;
          if (key != 0u && (key & mask) == prefix) atomicAdd(&hist[(key >> shift) & 255], 1u);
        }
        __syncthreads();
        cand_find_digit(hist, target, &digit_s, &above_s, wsum);
        const int d = digit_s;
        const unsigned a = above_s;
        __syncthreads();
        target -= a;
        prefix |= (unsigned)d << shift;
        mask |= 255u << shift;
      }
      kth = prefix;
    }
    if (t == 0) nkeep = 0;
    __syncthreads();
    for (int i = t; i < N; i += 256) {
      if (!(v[i] > -INFINITY) || fkey(v[i]) < kth) continue;
      const int s = atomicAdd(&nkeep, 1);
      cv[s] = v[i];
      cid[s] = id[i];
    }
    __syncthreads();
    const int m = nkeep;  // every candidate >= the k-th largest value (ties included), unordered
    // exact ranks (value desc, global index asc) inside the kept set -> sorted copy
    for (int i = t; i < m; i += 256) {
      const float a = cv[i];
      const int ai = cid[i];
      int r = 0;
      for (int j = 0; j < m; ++j) {
        const float c = cv[j];
        r += (c > a || (c == a && cid[j] < ai)) ? 1 : 0;
      }
      sv[r] = a;
      sid[r] = ai;
    }
    __syncthreads();
    if (t == 0) {
      const int n = m;  // sv[0, m) holds every candidate >= the top-k boundary, in order
      float th = -INFINITY;
      if (k > 0 && k <= n) th = sv[k - 1];  // top-k boundary value (ties at it are kept)
      if (p < 1.f) {
        unsigned long long z = 0;
        int m = 0;
        for (; m < n && sv[m] >= th; ++m) z += sv3_mass(sv[m], mx);
        unsigned long long target = (unsigned long long)((double)p * (double)z);
        if (target < 1ull) target = 1ull;
        unsigned long long cum = 0;
        float tp = sv[m > 0 ? m - 1 : 0];
        for (int r = 0; r < m; ++r) {
          const unsigned long long hi = cum + sv3_mass(sv[r], mx);
          if (cum < target && hi >= target) {
            tp = sv[r];
            break;
          }
          cum = hi;
        }
        th = fmaxf(th, tp);
      }
      thr_s = th;
    }
    __syncthreads();
    thr = thr_s;
  }
  const unsigned long long seed = seeds ? (unsigned long long)seeds[b] : 0ull;
  const unsigned s0 = (unsigned)seed, s1 = (unsigned)(seed >> 32);
  float best = -INFINITY;
  int besti = 0x7fffffff;
  for (int i = t; i < N; i += 256) {
    float x = v[i];
    const int idx = id[i];
    if (!(x > -INFINITY)) continue;
    if (!greedy) {
      if (x < thr) continue;
      const unsigned r = philox((unsigned)idx, 0u, s0, s1);
      const float u = ((float)(r >> 8) + 0.5f) * (1.0f / 16777216.0f);
      x = x - __logf(-__logf(u));
    }
    if (x > best || (x == best && idx < besti)) { best = x; besti = idx; }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(besti, o, 64);
    if (ob > best || (ob == best && oi < besti)) { best = ob; besti = oi; }
  }
  __syncthreads();
  if ((t & 63) == 0) { red[t >> 6] = best; redi[t >> 6] = besti; }
  __syncthreads();
  if (t == 0) {
    float bb = red[0];
    int bi = redi[0];
    for (int i = 1; i < 4; ++i)
      if (red[i] > bb || (red[i] == bb && redi[i] < bi)) { bb = red[i]; bi = redi[i]; }
    if (bi == 0x7fffffff) bi = 0;
    out[b] = bi;
    if (out2) out2[b] = bi;
  }
}

void launch_cand_topk(const void* logits, int64_t ld, int B, int vl, int lo, int V, const void* temperature,
                      const void* top_k, int K, int KC, void* pack, int64_t ldp, hipStream_t st, int shards) {
  if (B == 0) return;
  if (K < 1 || KC < K) throw std::runtime_error("cand_topk: need 1 <= K <= KC");
  if (shards < 1 || (int64_t)shards * 2 * KC > ldp) throw std::runtime_error("cand_topk: pack row too narrow");
  const int ept = (vl + CAND_THREADS - 1) / CAND_THREADS;
#define CT(E_)                                                                                                    \
  cand_topk_kernel<E_><<<dim3(B, shards), CAND_THREADS, 0, st>>>((const bf16_t*)logits, ld, vl, lo, V,            \
                                                   (const float*)temperature, (const int*)top_k, K, KC, (float*)pack, ldp)
  if (ept <= 4) CT(4);
  else if (ept <= 8) CT(8);
  else if (ept <= 16) CT(16);
  else throw std::runtime_error("cand_topk: vocab shard wider than 16384 (use the gathered-logits sampler)");
#undef CT
  HIP_CHECK_LAUNCH();
}

void launch_sample_cand(const void* pack, int64_t ldp, int B, int groups, int KC, const void* temperature,
                        const void* top_k, const void* top_p, const void* seeds, void* out, void* out2, hipStream_t st) {
  if (B == 0) return;
  if (groups * KC > SCAND_MAX) throw std::runtime_error("sample_cand: too many candidates per row");
  sample_cand_kernel<<<B, 256, 0, st>>>((const float*)pack, ldp, groups, KC, (const float*)temperature,
                                        (const int*)top_k, (const float*)top_p, (const int64_t*)seeds, (int64_t*)out,
                                        (int64_t*)out2);
  HIP_CHECK_LAUNCH();
}
