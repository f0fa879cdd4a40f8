// Shared helpers for the gfx950 (CDNA4 / MI355X) kernels of llmss_amd.
//
// Conventions used by every kernel in this directory:
//   * activations and weights are bf16 stored as raw 16-bit words (ushort); math is fp32;
//   * memory-bound kernels move 16 B per lane (8 bf16) per access (guide G13);
//   * wave = 64 lanes, blocks are multiples of 64 threads;
//   * every launcher takes the caller's hipStream_t so the whole decode step can be captured
//     into one HIP graph by the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>
#include <algorithm>
#include <stdexcept>
#include <string>

#define LLMSS_WAVE 64

typedef unsigned short bf16_t;
typedef unsigned short __attribute__((ext_vector_type(8))) u16x8;
typedef unsigned short __attribute__((ext_vector_type(4))) u16x4;
typedef short __attribute__((ext_vector_type(8))) s16x8;
typedef short __attribute__((ext_vector_type(4))) s16x4;
typedef float __attribute__((ext_vector_type(4))) f32x4;
typedef float __attribute__((ext_vector_type(16))) f32x16;
typedef float __attribute__((ext_vector_type(2))) f32x2;
typedef unsigned int __attribute__((ext_vector_type(4))) u32x4;
typedef unsigned int __attribute__((ext_vector_type(2))) u32x2;

#define LDS_AS __attribute__((address_space(3)))

__device__ __forceinline__ float bf2f(bf16_t x) { return __uint_as_float(((unsigned)x) << 16); }

__device__ __forceinline__ bf16_t f2bf(float f) {
  __hip_bfloat16 h = __float2bfloat16(f);  // v_cvt_pk_bf16_f32 on gfx950 (RNE, NaN-preserving)
  return *reinterpret_cast<bf16_t*>(&h);
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x <= 1024. `red` must hold >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = warp_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ float block_max(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  v = warp_max(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, red[i]);
  return t;
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  float u = k0 * (x + k1 * x * x * x);
  // tanh(u) = 1 - 2/(exp(2u)+1); saturates correctly at +-inf
  float t = 1.f - 2.f / (__expf(2.f * u) + 1.f);
  return 0.5f * x * (1.f + t);
}

__device__ __forceinline__ float gelu_erf(float x) { return 0.5f * x * (1.f + erff(x * 0.7071067811865476f)); }

__device__ __forceinline__ float silu(float x) { return x / (1.f + __expf(-x)); }

enum Act : int { ACT_NONE = 0, ACT_GELU_TANH = 1, ACT_GELU = 2, ACT_RELU = 3, ACT_SILU_GLU = 4 };

__device__ __forceinline__ float apply_act(float x, int act) {
  switch (act) {
    case ACT_GELU_TANH: return gelu_tanh(x);
    case ACT_GELU: return gelu_erf(x);
    case ACT_RELU: return fmaxf(x, 0.f);
    default: return x;
  }
}

// XCD-aware bijective remap of a linear workgroup id (guide T1): blocks b and b+8 share an XCD
// under round-robin dispatch, so give each XCD a contiguous run of tile ids.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7, xcd = orig & 7, idx = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

// Split-K tiled GEMMs: linear block id -> (m0, n0, split z). Items are ordered z-major, then
// N-tile, with the M-tiles of one N-tile adjacent, and each XCD receives a contiguous item range
// (dispatch is round-robin over the linear id). An XCD therefore works on whole weight columns and
// one K-slice: its L2 fetches each weight tile once for every M-tile and only its K-slice of the
// activations. Measured on the TP=8 QKV shape (M=512, N=1536, K=4096): the M-major order fetched
// 59 MB from the fabric for 16.6 MB of unique operands.
struct TileWork {
  int m0, n0, z;
};
__device__ __forceinline__ TileWork tile_work(int ntm, int ntn, int bm, int bn) {
  const int G = gridDim.x * gridDim.y;
  const int w = xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, G);
  const int per = ntm * ntn;
  const int z = w / per, t = w - z * per;
  const int nt = t / ntm;
  return {(t - nt * ntm) * bm, nt * bn, z};
}

#define HIP_CHECK_LAUNCH()                                                               \
  do {                                                                                   \
    hipError_t e__ = hipGetLastError();                                                  \
    if (e__ != hipSuccess) throw std::runtime_error(std::string("HIP launch failed: ") + \
                                                    hipGetErrorString(e__));             \
  } while (0)
