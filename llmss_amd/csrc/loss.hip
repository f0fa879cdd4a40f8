// Token-level cross-entropy of LM logits (reference: CrossEntropyLoss on shifted
// labels, gptj_modeling.py:612-622 / gpt_bigcode_modeling.py:896-902, an fp32 [B*(S-1), V]
// log-softmax materialised by ATen).
//
// loss[t] = logsumexp(logits[t, :V]) - logits[t, label[t]]   (fp32; label < 0 -> 0, not counted)
// One 256-thread workgroup per row streams the row ONCE with 16-B loads: an online
// (max, sum-of-exp) pair per lane, merged across lanes and waves - no second pass over V and no
// [T, V] probability tensor. Logits are bf16 (the decoder's output) or fp32.
#include "common.h"

template <typename T>
__device__ __forceinline__ void ce_load8(const T* p, float (&v)[8]);
template <>
__device__ __forceinline__ void ce_load8<bf16_t>(const bf16_t* p, float (&v)[8]) {
  const u16x8 x = *reinterpret_cast<const u16x8*>(p);
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = bf2f(x[i]);
}
template <>
__device__ __forceinline__ void ce_load8<float>(const float* p, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p), b = *reinterpret_cast<const f32x4*>(p + 4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = a[i];
    v[4 + i] = b[i];
  }
}

__device__ __forceinline__ void lse_merge(float& m, float& s, float m2, float s2) {
  if (m2 == -INFINITY) return;  // empty partner (a lane that saw no element): avoid inf - inf
  if (m == -INFINITY) {
    m = m2;
    s = s2;
    return;
  }
  const float mx = fmaxf(m, m2);
  s = s * exp2f(m - mx) + s2 * exp2f(m2 - mx);  // log2 domain
  m = mx;
}

template <typename T>
__global__ __launch_bounds__(256) void ce_loss_kernel(const T* __restrict__ logits, int64_t ld, const int64_t* __restrict__ labels,
                                                      int V, float* __restrict__ loss) {
  constexpr float kL2e = 1.4426950408889634f, kLn2 = 0.6931471805599453f;
  __shared__ float red_m[4], red_s[4];
  const int t = blockIdx.x;
  const T* row = logits + (int64_t)t * ld;
  float m = -INFINITY, s = 0.f;
  const int V8 = V & ~7;
  for (int c = threadIdx.x * 8; c < V8; c += 256 * 8) {
    float v[8];
    ce_load8<T>(row + c, v);
    float cm = v[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) cm = fmaxf(cm, v[i]);
    cm *= kL2e;
    float cs = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) cs += exp2f(v[i] * kL2e - cm);
    lse_merge(m, s, cm, cs);
  }
  for (int c = V8 + threadIdx.x; c < V; c += 256) {  // tail (V % 8)
    float x;
    if constexpr (sizeof(T) == 2) x = bf2f(row[c]);
    else x = row[c];
    lse_merge(m, s, x * kL2e, 1.f);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    lse_merge(m, s, m2, s2);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) {
    red_m[w] = m;
    red_s[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = red_m[0], S = red_s[0];
    for (int i = 1; i < 4; ++i) lse_merge(M, S, red_m[i], red_s[i]);
    const int64_t lab = labels[t];
    float out = 0.f;
    if (lab >= 0 && lab < V) {
      float x;
      if constexpr (sizeof(T) == 2) x = bf2f(row[lab]);
      else x = row[lab];
      out = (M + log2f(S)) * kLn2 - x;
    }
    loss[t] = out;
  }
}

void launch_ce_loss(const void* logits, int64_t ld, bool fp32, const void* labels, int T, int V, void* loss,
                    hipStream_t st) {
  if (T == 0) return;
  if (ld % 8) throw std::runtime_error("ce_loss: row stride must be a multiple of 8 elements");
  if (fp32)
    ce_loss_kernel<float><<<T, 256, 0, st>>>((const float*)logits, ld, (const int64_t*)labels, V, (float*)loss);
  else
    ce_loss_kernel<bf16_t><<<T, 256, 0, st>>>((const bf16_t*)logits, ld, (const int64_t*)labels, V, (float*)loss);
  HIP_CHECK_LAUNCH();
}
