// Fused residual-add + LayerNorm / RMSNorm (reference applies
// nn.LayerNorm after a separate residual add, gptj_modeling.py:295-310,
// gpt_bigcode_modeling.py:366-407; the optional external dropout_add_ln_fwd kernel at
// utils/layers.py:217-253 is the same fusion, which the reference never calls).
//
//   r = x (+ residual)            -> stored to residual_out (bf16) when a residual is given
//   y = norm(r) * w (+ b)         -> bf16
//
// One workgroup per row; every lane owns MAXC 16-byte chunks of the row in registers, so the
// row is read from HBM once and the two-pass (mean, then centred variance) statistics are
// computed from registers. Memory bound: 16-B vector loads/stores only (guide G13).
#include "common.h"
#include <stdexcept>
#include <string>

// PART: x is not a bf16 tensor but S fp32 split-K partial slabs of the preceding GEMM
// (part[s*slab + row*H + col]) plus an optional bf16 bias - the split-K reduction is fused here.
// PS: 0 = bf16 input; > 0 = that many partial slabs (compile-time: every load is issued before
// the first add - a runtime trip count would serialise one memory round trip per slab); -1 = S.
template <int MAXC, bool RMS, bool HAS_RES, bool HAS_BIAS, int PS>
__global__ __launch_bounds__(256) void add_norm_kernel(const bf16_t* __restrict__ x, int64_t x_stride,
                                                       const bf16_t* res_in, bf16_t* res_out,
                                                       const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                       bf16_t* __restrict__ y, int64_t y_stride, int H, float eps,
                                                       const float* __restrict__ part, int S, int64_t slab,
                                                       const bf16_t* __restrict__ xbias, unsigned char* __restrict__ q8,
                                                       float* __restrict__ s8, int xcw) {
  __shared__ float red[32];
  __shared__ float red2[32];
  const int row = blockIdx.x;
  const int nchunk = H >> 3;
  float v[MAXC][8];
  const bf16_t* xr = x + row * x_stride;
  // norm weight / bias issued first, beside the row loads (not a dependent round trip after them)
  u16x8 wv[MAXC], bv[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = min((int)threadIdx.x + c * (int)blockDim.x, nchunk - 1);
    wv[c] = *reinterpret_cast<const u16x8*>(w + ch * 8);
    if constexpr (HAS_BIAS) bv[c] = *reinterpret_cast<const u16x8*>(b + ch * 8);
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = threadIdx.x + c * blockDim.x;
    if (ch < nchunk) {
      if constexpr (PS != 0) {
        const float* pr = part + (int64_t)row * H + ch * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
        if constexpr (PS > 0) {
          f32x4 p[PS][2];
#pragma unroll
          for (int sp = 0; sp < PS; ++sp) {
            p[sp][0] = *reinterpret_cast<const f32x4*>(pr + sp * slab);
            p[sp][1] = *reinterpret_cast<const f32x4*>(pr + sp * slab + 4);
          }
#pragma unroll
          for (int sp = 0; sp < PS; ++sp)
#pragma unroll
            for (int j = 0; j < 4; ++j) { v[c][j] += p[sp][0][j]; v[c][4 + j] += p[sp][1][j]; }
        } else {  // runtime S: the slabs in groups of SG, every load of a group issued before its adds (one memory
                  // round trip per group, not per slab; the adds stay in slab order 0..S-1)
          constexpr int SG = MAXC == 1 ? 8 : (MAXC == 2 ? 4 : 2);
          for (int s0 = 0; s0 < S; s0 += SG) {
            f32x4 p[SG][2];
#pragma unroll
            for (int g = 0; g < SG; ++g) {
              const int sp = min(s0 + g, S - 1);
              p[g][0] = *reinterpret_cast<const f32x4*>(pr + sp * slab);
              p[g][1] = *reinterpret_cast<const f32x4*>(pr + sp * slab + 4);
            }
#pragma unroll
            for (int g = 0; g < SG; ++g)
              if (s0 + g < S)
#pragma unroll
                for (int j = 0; j < 4; ++j) { v[c][j] += p[g][0][j]; v[c][4 + j] += p[g][1][j]; }
          }
        }
        if (xbias) {
          u16x8 bb = *reinterpret_cast<const u16x8*>(xbias + ch * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] += bf2f(bb[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(f2bf(v[c][j]));  // the GEMM output is bf16 in the unfused path
      } else {
        // xcw > 0: column-chunked input [C][T][xcw] (the decoder's column-chunked all-reduce schedule)
        const bf16_t* xp = xcw > 0 ? x + (int64_t)(ch * 8 / xcw) * gridDim.x * xcw + (int64_t)row * xcw + (ch * 8) % xcw
                                   : xr + ch * 8;
        u16x8 a = *reinterpret_cast<const u16x8*>(xp);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(a[j]);
      }
      if constexpr (HAS_RES) {
        u16x8 r = *reinterpret_cast<const u16x8*>(res_in + (int64_t)row * H + ch * 8);
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          v[c][j] += bf2f(r[j]);
          o[j] = f2bf(v[c][j]);
          v[c][j] = bf2f(o[j]);  // normalise exactly what is stored in the residual stream
        }
        *reinterpret_cast<u16x8*>(res_out + (int64_t)row * H + ch * 8) = o;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  // ONE block reduction of (sum, sum of squares): var = E[x^2] - E[x]^2 in fp32 (relative error ~1e-7 x
  // (1 + mean^2 / var), negligible for residual-stream rows) instead of a second pass over the centred row
  float mean = 0.f, var;
  {
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int c = 0; c < MAXC; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) {  // padded chunks hold zeros
        s += v[c][j];
        ss += v[c][j] * v[c][j];
      }
    if constexpr (RMS) {
      var = block_sum(ss, red) / H;  // mean of squares
    } else {
      const f32x2 tot = block_sum2(s, ss, red);
      mean = tot[0] / H;
      var = fmaxf(tot[1] / H - mean * mean, 0.f);
    }
  }
  const float rstd = rsqrtf(var + eps);
  u16x8 ov[MAXC];
  float amax = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = threadIdx.x + c * blockDim.x;
    if (ch < nchunk) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = (v[c][j] - mean) * rstd * bf2f(wv[c][j]);
        if constexpr (HAS_BIAS) t += bf2f(bv[c][j]);
        o[j] = f2bf(t);
        amax = fmaxf(amax, fabsf(bf2f(o[j])));
      }
      ov[c] = o;
      *reinterpret_cast<u16x8*>(y + row * y_stride + ch * 8) = o;
    }
  }
  if (q8) {  // per-token fp8-e4m3 twin of the bf16 output for a W8A8 consumer (== quant_fp8_rows_ld of y)
    amax = block_max(amax, red2);
    const float sc = amax > 0.f ? amax / 448.f : 1.f;
    const float inv = 1.f / sc;
    if (threadIdx.x == 0) s8[row] = sc;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = threadIdx.x + c * blockDim.x;
      if (ch < nchunk) {
        float f[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) f[j] = fminf(fmaxf(bf2f(ov[c][j]) * inv, -448.f), 448.f);
        unsigned lo = 0, hi = 0;
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], lo, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], hi, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
        *reinterpret_cast<uint2*>(q8 + (int64_t)row * H + ch * 8) = make_uint2(lo, hi);
      }
    }
  }
}

template <bool RMS, bool HAS_RES, bool HAS_BIAS, int PART = 0>
static void launch_norm_t(const bf16_t* x, int64_t xs, const bf16_t* ri, bf16_t* ro, const bf16_t* w,
                          const bf16_t* b, bf16_t* y, int64_t ys, int T, int H, float eps, hipStream_t st,
                          const float* part = nullptr, int S = 0, int64_t slab = 0, const bf16_t* xbias = nullptr,
                          unsigned char* q8 = nullptr, float* s8 = nullptr, int xcw = 0) {
  const int nchunk = H / 8;
  int threads = nchunk <= 256 ? ((nchunk + 63) / 64) * 64 : 256;
  const int maxc = (nchunk + threads - 1) / threads;
  dim3 grid(T), block(threads);
  if (maxc == 1)
    add_norm_kernel<1, RMS, HAS_RES, HAS_BIAS, PART><<<grid, block, 0, st>>>(x, xs, ri, ro, w, b, y, ys, H, eps, part, S, slab, xbias, q8, s8, xcw);
  else if (maxc == 2)
    add_norm_kernel<2, RMS, HAS_RES, HAS_BIAS, PART><<<grid, block, 0, st>>>(x, xs, ri, ro, w, b, y, ys, H, eps, part, S, slab, xbias, q8, s8, xcw);
  else if (maxc <= 4)
    add_norm_kernel<4, RMS, HAS_RES, HAS_BIAS, PART><<<grid, block, 0, st>>>(x, xs, ri, ro, w, b, y, ys, H, eps, part, S, slab, xbias, q8, s8, xcw);
  else if (maxc <= 8)
    add_norm_kernel<8, RMS, HAS_RES, HAS_BIAS, PART><<<grid, block, 0, st>>>(x, xs, ri, ro, w, b, y, ys, H, eps, part, S, slab, xbias, q8, s8, xcw);
  else
    throw std::runtime_error("add_norm: hidden size too large (max 16384)");
  HIP_CHECK_LAUNCH();
}

void launch_add_norm(const void* x, int64_t x_stride, const void* res_in, void* res_out, const void* w,
                     const void* b, void* y, int64_t y_stride, int T, int H, float eps, bool rms,
                     hipStream_t st, void* q8v, void* s8v, int xcw) {
  auto Q8 = (unsigned char*)q8v;
  auto S8 = (float*)s8v;
  if (H % 8 != 0) throw std::runtime_error("add_norm: hidden size must be a multiple of 8");
  if (xcw < 0 || xcw % 8 || (xcw && H % xcw)) throw std::runtime_error("add_norm: chunk width must divide H, multiple of 8");
  if (T == 0) return;
  auto X = (const bf16_t*)x;
  auto RI = (const bf16_t*)res_in;
  auto RO = (bf16_t*)res_out;
  auto W = (const bf16_t*)w;
  auto B = (const bf16_t*)b;
  auto Y = (bf16_t*)y;
  const bool has_res = res_in != nullptr, has_b = b != nullptr;
  if (rms) {
    if (has_res) launch_norm_t<true, true, false>(X, x_stride, RI, RO, W, B, Y, y_stride, T, H, eps, st, nullptr, 0, 0, nullptr, Q8, S8, xcw);
    else launch_norm_t<true, false, false>(X, x_stride, RI, RO, W, B, Y, y_stride, T, H, eps, st, nullptr, 0, 0, nullptr, Q8, S8, xcw);
  } else {
    if (has_res) {
      if (has_b) launch_norm_t<false, true, true>(X, x_stride, RI, RO, W, B, Y, y_stride, T, H, eps, st, nullptr, 0, 0, nullptr, Q8, S8, xcw);
      else launch_norm_t<false, true, false>(X, x_stride, RI, RO, W, B, Y, y_stride, T, H, eps, st, nullptr, 0, 0, nullptr, Q8, S8, xcw);
    } else {
      if (has_b) launch_norm_t<false, false, true>(X, x_stride, RI, RO, W, B, Y, y_stride, T, H, eps, st, nullptr, 0, 0, nullptr, Q8, S8, xcw);
      else launch_norm_t<false, false, false>(X, x_stride, RI, RO, W, B, Y, y_stride, T, H, eps, st, nullptr, 0, 0, nullptr, Q8, S8, xcw);
    }
  }
}

// residual-add + norm whose input is the split-K partial sum of the preceding row-parallel GEMM
void launch_add_norm_partial(const void* part, int S, int64_t slab, const void* xbias, const void* res_in,
                             void* res_out, const void* w, const void* b, void* y, int64_t y_stride, int T, int H,
                             float eps, bool rms, hipStream_t st, void* q8v, void* s8v) {
  auto Q8 = (unsigned char*)q8v;
  auto S8 = (float*)s8v;
  if (H % 8 != 0) throw std::runtime_error("add_norm: hidden size must be a multiple of 8");
  if (!res_in) throw std::runtime_error("add_norm_partial: needs a residual");
  if (T == 0) return;
  auto P = (const float*)part;
  auto XB = (const bf16_t*)xbias;
  auto RI = (const bf16_t*)res_in;
  auto RO = (bf16_t*)res_out;
  auto W = (const bf16_t*)w;
  auto B = (const bf16_t*)b;
  auto Y = (bf16_t*)y;
#define LNP(PS_)                                                                                                   \
  do {                                                                                                             \
    if (rms) launch_norm_t<true, true, false, PS_>(nullptr, 0, RI, RO, W, B, Y, y_stride, T, H, eps, st, P, S, slab, XB, Q8, S8); \
    else if (b) launch_norm_t<false, true, true, PS_>(nullptr, 0, RI, RO, W, B, Y, y_stride, T, H, eps, st, P, S, slab, XB, Q8, S8); \
    else launch_norm_t<false, true, false, PS_>(nullptr, 0, RI, RO, W, B, Y, y_stride, T, H, eps, st, P, S, slab, XB, Q8, S8); \
  } while (0)
  switch (S) {
    case 2: LNP(2); break;
    case 4: LNP(4); break;
    case 8: LNP(8); break;
    default: LNP(-1); break;
  }
#undef LNP
}
