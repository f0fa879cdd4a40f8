// fp8 (OCP e4m3fn, gfx950-native - not the MI300 fnuz variant) weight quantisation at load time:
// one scale per output row (channel), q = saturate(w / scale), scale = absmax / 448.
// Used by the W8A16 path of the skinny GEMM (weights dequantised in registers, halving the
// HBM bytes that bound decode) for the Llama-2-70B TP=8 fp8 configuration.
#include "common.h"

__global__ __launch_bounds__(256) void quant_fp8_rows_kernel(const bf16_t* __restrict__ w, unsigned char* __restrict__ q,
                                                             float* __restrict__ scale, int64_t K) {
  __shared__ float red[16];
  const int64_t r = blockIdx.x;
  const bf16_t* wr = w + r * K;
  float amax = 0.f;
  for (int64_t k = threadIdx.x * 8; k < K; k += blockDim.x * 8) {
    u16x8 v = *reinterpret_cast<const u16x8*>(wr + k);
#pragma unroll
    for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f(v[j])));
  }
  amax = block_max(amax, red);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[r] = s;
  for (int64_t k = threadIdx.x * 8; k < K; k += blockDim.x * 8) {
    u16x8 v = *reinterpret_cast<const u16x8*>(wr + k);
    unsigned lo = 0, hi = 0;
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(bf2f(v[j]) * inv, -448.f), 448.f);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], lo, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], hi, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
    *reinterpret_cast<uint2*>(q + r * K + k) = make_uint2(lo, hi);
  }
}

void launch_quant_fp8_rows(const void* w, void* q, void* scale, int64_t N, int64_t K, hipStream_t st) {
  if (K % 8) throw std::runtime_error("quant_fp8_rows: K must be a multiple of 8");
  if (N == 0) return;
  quant_fp8_rows_kernel<<<(unsigned)N, 256, 0, st>>>((const bf16_t*)w, (unsigned char*)q, (float*)scale, K);
  HIP_CHECK_LAUNCH();
}

// Per-token activation quantisation for W8A8 GEMMs (x rows with a leading dimension): one pass, the
// row stays in registers between the absmax reduction and the conversion (K <= 8192; longer rows take
// the two-pass kernel above). Writes q [M, K] (dense) and scale [M].
template <int CH>
__global__ __launch_bounds__(256) void quant_fp8_act_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                           unsigned char* __restrict__ q, float* __restrict__ scale,
                                                           int K) {
  __shared__ float red[16];
  const int64_t r = blockIdx.x;
  const bf16_t* xr = x + r * ldx;
  u16x8 v[CH];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int k = (c * 256 + threadIdx.x) * 8;
    if (k < K) {
      v[c] = *reinterpret_cast<const u16x8*>(xr + k);
#pragma unroll
      for (int j = 0; j < 8; ++j) amax = fmaxf(amax, fabsf(bf2f(v[c][j])));
    }
  }
  amax = block_max(amax, red);
  const float s = amax > 0.f ? amax / 448.f : 1.f;
  const float inv = 1.f / s;
  if (threadIdx.x == 0) scale[r] = s;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int k = (c * 256 + threadIdx.x) * 8;
    if (k < K) {
      float f[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(bf2f(v[c][j]) * inv, -448.f), 448.f);
      unsigned lo = 0, hi = 0;
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], lo, false);
      lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], hi, false);
      hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
      *reinterpret_cast<uint2*>(q + r * (int64_t)K + k) = make_uint2(lo, hi);
    }
  }
}

void launch_quant_fp8_rows_ld(const void* x, int64_t ldx, void* q, void* scale, int64_t M, int64_t K, hipStream_t st) {
  if (K % 8 || ldx % 8) throw std::runtime_error("quant_fp8_rows_ld: K and the row stride must be multiples of 8");
  if (M == 0) return;
  auto X = (const bf16_t*)x;
  auto Q = (unsigned char*)q;
  auto S = (float*)scale;
  if (K <= 2048) quant_fp8_act_kernel<1><<<(unsigned)M, 256, 0, st>>>(X, ldx, Q, S, (int)K);
  else if (K <= 4096) quant_fp8_act_kernel<2><<<(unsigned)M, 256, 0, st>>>(X, ldx, Q, S, (int)K);
  else if (K <= 8192) quant_fp8_act_kernel<4><<<(unsigned)M, 256, 0, st>>>(X, ldx, Q, S, (int)K);
  else if (ldx == K) quant_fp8_rows_kernel<<<(unsigned)M, 256, 0, st>>>(X, Q, S, K);
  else throw std::runtime_error("quant_fp8_rows_ld: rows longer than 8192 must be contiguous");
  HIP_CHECK_LAUNCH();
}

// w[r, :] = q[r, :] * scale[r] -> bf16. Prefill with fp8 weights (M > 128) is compute-bound, so the
// weight is expanded once per call into a bf16 scratch and the big-tile bf16 GEMM runs on it
// (100 MB of fp8 -> ~40 us, vs ~0.75 ms for the GEMM it feeds at 8K tokens).
__global__ __launch_bounds__(256) void dequant_fp8_rows_kernel(const unsigned char* __restrict__ q,
                                                               const float* __restrict__ scale,
                                                               bf16_t* __restrict__ w, int64_t N, int64_t K) {
  const int64_t n8 = N * K / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i * 8;
    const float s = scale[e / K];
    const uint2 v = *reinterpret_cast<const uint2*>(q + e);
    const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8(v.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8(v.x, true);
    const f32x2 c = __builtin_amdgcn_cvt_pk_f32_fp8(v.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8(v.y, true);
    u16x8 o = {f2bf(a[0] * s), f2bf(a[1] * s), f2bf(b[0] * s), f2bf(b[1] * s),
               f2bf(c[0] * s), f2bf(c[1] * s), f2bf(d[0] * s), f2bf(d[1] * s)};
    *reinterpret_cast<u16x8*>(w + e) = o;
  }
}

void launch_dequant_fp8_rows(const void* q, const void* scale, void* w, int64_t N, int64_t K, hipStream_t st) {
  if (K % 8) throw std::runtime_error("dequant_fp8_rows: K must be a multiple of 8");
  if (N == 0) return;
  const int64_t n8 = N * K / 8;
  const int blocks = (int)std::min<int64_t>((n8 + 255) / 256, 256 * 16);
  dequant_fp8_rows_kernel<<<blocks, 256, 0, st>>>((const unsigned char*)q, (const float*)scale, (bf16_t*)w, N, K);
  HIP_CHECK_LAUNCH();
}
