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

void launch_sample(const void* logits, int64_t ld, bool fp32_logits, int B, int V, const void* temperature,
                   const void* top_k, const void* top_p, const void* seeds, void* out, void* out2, hipStream_t st) {
  if (B == 0) return;
  if (fp32_logits)
    sample_kernel<float><<<B, 1024, 0, st>>>((const float*)logits, ld, V, (const float*)temperature, (const int*)top_k,
                                             (const float*)top_p, (const int64_t*)seeds, (int64_t*)out, (int64_t*)out2);
  else
    sample_kernel<bf16_t><<<B, 1024, 0, st>>>((const bf16_t*)logits, ld, V, (const float*)temperature,
                                              (const int*)top_k, (const float*)top_p, (const int64_t*)seeds,
                                              (int64_t*)out, (int64_t*)out2);
  HIP_CHECK_LAUNCH();
}
