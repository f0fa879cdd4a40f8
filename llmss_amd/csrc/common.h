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

// Block-wide sums of two values with one pair of barriers. `red` must hold >= 32 floats.
__device__ __forceinline__ f32x2 block_sum2(float a, float b, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = (blockDim.x + 63) >> 6;
  a = warp_sum(a);
  b = warp_sum(b);
  __syncthreads();
  if (lane == 0) {
    red[wid] = a;
    red[16 + wid] = b;
  }
  __syncthreads();
  f32x2 t = {0.f, 0.f};
  for (int i = 0; i < nw; ++i) {
    t[0] += red[i];
    t[1] += red[16 + i];
  }
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

// Buffer resource descriptor whose words the compiler can PROVE wave-uniform (guide T20): the base pointer
// halves and the byte count go through readfirstlane, so the descriptor lives in SGPRs and buffer loads /
// stores are not wrapped in waterfall loops (one readfirstlane loop per memory op otherwise). `bytes` is
// clamped to the 32-bit record count; callers keep every per-lane part in voffset.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p, int64_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)(bytes < 0x7fffffff ? bytes : 0x7fffffff));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, n,
                                           0x00020000);
}

// Reductions over lane pairs (lane, lane ^ 16) / (lane, lane ^ 32) by the gfx950 permlane swaps (VALU,
// no LDS round trip like ds_bpermute-based __shfl_xor): swapping two copies of x leaves x and its
// partner's x in the two registers, in some order - symmetric ops need no fix-up. Inline asm (with the
// 2 wait states the swap needs after a VALU write of its operands): through the builtins hipcc treats
// the two results as one value and drops the partner.
template <bool P32>
__device__ __forceinline__ f32x2 swap_pair(float x) {
  unsigned a = __builtin_bit_cast(unsigned, x), b = a;
  if constexpr (P32) asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  else asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return f32x2{__builtin_bit_cast(float, a), __builtin_bit_cast(float, b)};
}
__device__ __forceinline__ float xor16_max(float x) { const f32x2 r = swap_pair<false>(x); return fmaxf(r[0], r[1]); }
__device__ __forceinline__ float xor32_max(float x) { const f32x2 r = swap_pair<true>(x); return fmaxf(r[0], r[1]); }
__device__ __forceinline__ float xor16_sum(float x) { const f32x2 r = swap_pair<false>(x); return r[0] + r[1]; }
__device__ __forceinline__ float xor32_sum(float x) { const f32x2 r = swap_pair<true>(x); return r[0] + r[1]; }

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

// QKV-projection epilogue (decode / prompt chunks): instead of the separate RoPE + paged-KV-write kernel
// (embed_rope.hip rope_cache_kernel, whose semantics this reproduces), the GEMM's LDS-staged epilogue
// rounds each (token m, 8 columns) group to bf16 as the unfused output would be, rotates q / k columns
// (neox: the partner column d +- rot/2 is read from the same tile row - the host only takes this path
// with head-aligned tiles; gptj: pairs inside the group), stores the row to the qkv buffer and the k / v
// groups to their paged-cache rows (bf16 caches). D == 0: not a QKV projection.
//
//
// mxq / mxs (SwiGLU GEMMs only, D == 0): instead of bf16 rows, write the SwiGLU output as MX-fp8 for a W8A8 consumer
// (gemm_mid MXA): e4m3 bytes [M][N/2] with row stride ldy, and one e8m0 scale per row and 32 outputs [M][N/64] -
// the scale 2^e with the smallest e that puts the block's |max| (after bf16 rounding, as the unfused output) at or
// below 448 (OCP MX).
struct QkvEpi {
  const int64_t* pos;
  const float* cos_t;
  const float* sin_t;
  bf16_t* kc;
  bf16_t* vc;
  const int64_t* slot;
  int nh, nkv, D, rot, block_size, style, do_rope;
  unsigned char* mxq;
  unsigned char* mxs;
};

// e8m0 exponent e of an MX block with absolute maximum amax (> 0): the smallest e with amax / 2^e <= 448, clamped to
// the exponents whose inverse 2^-e is a normal float
__device__ __forceinline__ int mx_block_exp(float amax) {
  const uint32_t b = __float_as_uint(amax / 448.f);
  int e = (int)((b >> 23) & 255) - 127 + ((b & 0x7fffffu) != 0u);
  return e < -126 ? -126 : (e > 126 ? 126 : e);
}

// fp32 epilogue image of a tile with BN columns in LDS. The C-layout writes (lane li, g -> row 4g + i,
// column li: ds_write_b32, banks mod 32 per 32-lane half) and the row-piece reads (ds_read_b128, banks
// mod 64 per 16-lane group) are both conflict-free when rows are unpadded and the 16-B slot of a float
// is XOR-ed with 4 on rows with bit 2 set (BN % 32 == 0); other widths pad rows by 4 floats. The
// previous padded image with 4-byte reads cost 4-8x the ideal LDS cycles on the read side
// (SQ_LDS_BANK_CONFLICT 21 % of gemm_big's LDS-active cycles, all in the epilogue).
template <int BN>
struct EpiImg {
  static constexpr bool SWZ = BN % 32 == 0;
  static constexpr int LDW = SWZ ? BN : BN + 4;
  __device__ static __forceinline__ int at(int r, int c) { return r * LDW + (SWZ ? (c ^ (((r >> 2) & 1) << 4)) : c); }
  __device__ static __forceinline__ f32x4 ld4(const float* ct, int r, int c) {  // c % 4 == 0
    return *reinterpret_cast<const f32x4*>(ct + at(r, c));
  }
  // 8 floats of row r from column c (c % 8 == 0) as two ds_read_b128. Lanes whose bit 3 is set take
  // the upper half first, so the lanes of a 16-lane group that hit the same slot pair split across
  // the two instructions.
  __device__ static __forceinline__ void ld8(const float* ct, int r, int c, float (&x)[8]) {
    const int key = (threadIdx.x >> 3) & 1;
    const f32x4 a = ld4(ct, r, c + 4 * key), b = ld4(ct, r, c + 4 * (key ^ 1));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      x[i] = key ? b[i] : a[i];
      x[4 + i] = key ? a[i] : b[i];
    }
  }
};

// One LDS row chunk of the QKV epilogue: each thread owns ITEMS (row, 8-column) groups of the chunk and
// processes them G at a time in three phases - (1) every group's position and cache slot, (2) every
// group's cos / sin rows, (3) rotate, round, store - so each thread pays two dependent memory round trips
// per G groups instead of per group (the loads sit behind no per-group branch: addresses are clamped).
template <int BN, int NTHR, int R>
__device__ __forceinline__ void qkv_store_chunk(const QkvEpi& e, const float* ct, int rows, int r0, int m0,
                                                int n0, int M, int N, bf16_t* __restrict__ Y, int64_t ldy,
                                                const bf16_t* __restrict__ bias) {
  constexpr int VPR = BN / 8, ITEMS = (R * VPR + NTHR - 1) / NTHR, G = ITEMS < 4 ? ITEMS : 4;
  const int D = e.D, nq = e.nh * D, nk = e.nkv * D, rh = e.rot >> 1;
  const bool rope = e.do_rope != 0;
#pragma unroll
  for (int i0 = 0; i0 < ITEMS; i0 += G) {
    int rr[G], cc[G], mm[G];
    bool ok[G];
    int64_t p[G], sl[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {  // phase 1: positions and slots
      const int v = threadIdx.x + (i0 + j) * NTHR;
      rr[j] = v / VPR;
      cc[j] = (v - rr[j] * VPR) * 8;
      mm[j] = m0 + r0 + rr[j];
      ok[j] = i0 + j < ITEMS && rr[j] < rows && mm[j] < M && n0 + cc[j] < N;
      const int mc = min(mm[j], M - 1);
      p[j] = rope ? e.pos[mc] : 0;
      sl[j] = e.kc ? e.slot[mc] : -1;
    }
    f32x4 cs[G][2], sn[G][2];
#pragma unroll
    for (int j = 0; j < G; ++j) {  // phase 2: cos / sin of each group's rotation angles
      if (rope) {
        const int n = n0 + cc[j], d = n % D;
        const bool lo = d < rh;
        int a = e.style == 1 ? (d >> 1) : (lo ? d : d - rh);
        a = (n < nq + nk && d < e.rot) ? a : 0;  // columns that do not rotate read a valid (unused) entry
        const float* cp = e.cos_t + p[j] * rh + a;
        const float* sp = e.sin_t + p[j] * rh + a;
        cs[j][0] = *reinterpret_cast<const f32x4*>(cp);
        sn[j][0] = *reinterpret_cast<const f32x4*>(sp);
        if (e.style != 1 && rh >= 8) {  // neox uses 8 angles per group (rh % 8 == 0: host-checked)
          cs[j][1] = *reinterpret_cast<const f32x4*>(cp + 4);
          sn[j][1] = *reinterpret_cast<const f32x4*>(sp + 4);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {  // phase 3: bias, bf16 rounding, rotation, stores
      if (!ok[j]) continue;
      const int c = cc[j], n = n0 + c, d = n % D, m = mm[j];
      float x[8], y[8];
      EpiImg<BN>::ld8(ct, rr[j], c, x);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        x[i] = bf2f(f2bf(x[i] + (bias ? bf2f(bias[n + i]) : 0.f)));
        y[i] = x[i];
      }
      const bool is_v = n >= nq + nk;
      if (rope && !is_v && d < e.rot) {
        if (e.style == 1) {  // gptj: interleaved pairs (2i, 2i + 1), angle d / 2 + i
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            y[2 * i] = x[2 * i] * cs[j][0][i] - x[2 * i + 1] * sn[j][0][i];
            y[2 * i + 1] = x[2 * i + 1] * cs[j][0][i] + x[2 * i] * sn[j][0][i];
          }
        } else {  // neox: halves [0, rh) and [rh, rot) rotate against each other
          const bool lo = d < rh;
          const int sh = lo ? rh : -rh;
          float xs[8];
          EpiImg<BN>::ld8(ct, rr[j], c + sh, xs);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float xp = bf2f(f2bf(xs[i] + (bias ? bf2f(bias[n + sh + i]) : 0.f)));
            const float cv = cs[j][i >> 2][i & 3], sv = sn[j][i >> 2][i & 3];
            y[i] = lo ? x[i] * cv - xp * sv : x[i] * cv + xp * sv;
          }
        }
      }
      u16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = f2bf(y[i]);
      *reinterpret_cast<u16x8*>(Y + (int64_t)m * ldy + n) = o;
      if (n >= nq && sl[j] >= 0) {
        const int h = (n - (is_v ? nq + nk : nq)) / D;
        const int64_t row = ((sl[j] / e.block_size) * e.nkv + h) * (int64_t)e.block_size + sl[j] % e.block_size;
        *reinterpret_cast<u16x8*>((is_v ? e.vc : e.kc) + row * D + d) = o;
      }
    }
  }
}

// Stores rows [r0, r0 + rows) of a tile's fp32 epilogue image (EpiImg<BN> layout at `ct`, row 0 = tile row r0)
// cooperatively over NTHR threads: fp32 split-K slab rows (part), the QKV RoPE / KV-write epilogue (qe.D), SwiGLU
// pairs (glu) or bf16 rows with bias / activation. Shared by tile_store_lds and the decode GEMM (gemm_dec.hip),
// which builds the image from K-split waves.
template <int BN, int NTHR, int R>
__device__ __forceinline__ void img_store_rows(const float* ct, int rows, int r0, int m0, int n0, int M, int N,
                                               float* __restrict__ part, bf16_t* __restrict__ Y, int64_t ldy,
                                               const bf16_t* __restrict__ bias, int act, int glu, const QkvEpi& qe) {
  using Img = EpiImg<BN>;
  if (qe.D) {  // QKV projection: RoPE + paged KV write (N % 8 == 0, ldy % 8 == 0: host-checked)
    qkv_store_chunk<BN, NTHR, R>(qe, ct, rows, r0, m0, n0, M, N, Y, ldy, bias);
  } else if (part) {  // fp32 slab rows: 4 floats (16 B) per thread-step
    constexpr int VPR = BN / 4;
    for (int v = threadIdx.x; v < rows * VPR; v += NTHR) {
      const int r = v / VPR, c = (v - r * VPR) * 4;
      const int m = m0 + r0 + r, n = n0 + c;
      if (m >= M || n >= N) continue;
      const f32x4 val = Img::ld4(ct, r, c);
      float* dst = part + (int64_t)m * N + n;
      if (n + 3 < N && (N & 3) == 0) *reinterpret_cast<f32x4*>(dst) = val;
      else
        for (int j = 0; j < 4 && n + j < N; ++j) dst[j] = val[j];
    }
  } else if (glu && qe.mxq) {  // SwiGLU -> MX-fp8 (BN % 64 == 0: 4 consecutive threads hold one 32-output block)
    constexpr int VPR = BN / 16;
    static_assert(BN % 16 == 0, "SwiGLU tile");
    if constexpr (VPR % 4 == 0) {
      // rows * VPR is a multiple of 64 (rows % 16 == 0), so a wave's 64 lanes run the same trip count: the block
      // maximum's lane shuffles see every lane of the block
      for (int v = threadIdx.x; v < rows * VPR; v += NTHR) {
        const int r = v / VPR, oc = (v - r * VPR) * 8;
        const int p = oc >> 4, j = oc & 15;
        const int cg = 32 * p + j, m = m0 + r0 + r, ng = n0 + cg;
        const bool ok = m < M && ng < N;
        float gx[8], ux[8], h[8];
        Img::ld8(ct, r, cg, gx);
        Img::ld8(ct, r, cg + 16, ux);
        float amax = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float gv = gx[e], uv = ux[e];
          if (bias && ok) { gv += bf2f(bias[ng + e]); uv += bf2f(bias[ng + 16 + e]); }
          h[e] = bf2f(f2bf(silu(gv) * uv));
          amax = fmaxf(amax, fabsf(h[e]));
        }
        amax = fmaxf(amax, __shfl_xor(amax, 1, 64));
        amax = fmaxf(amax, __shfl_xor(amax, 2, 64));
        const int ex = amax > 0.f ? mx_block_exp(amax) : 0;
        const float inv = __uint_as_float((uint32_t)(127 - ex) << 23);
        unsigned lo = 0, hi = 0;
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(h[0] * inv, h[1] * inv, lo, false);
        lo = __builtin_amdgcn_cvt_pk_fp8_f32(h[2] * inv, h[3] * inv, lo, true);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(h[4] * inv, h[5] * inv, hi, false);
        hi = __builtin_amdgcn_cvt_pk_fp8_f32(h[6] * inv, h[7] * inv, hi, true);
        const int64_t oc_g = n0 / 2 + oc;  // output column
        if (ok) {
          *reinterpret_cast<uint2*>(qe.mxq + (int64_t)m * ldy + oc_g) = make_uint2(lo, hi);
          if ((v & 3) == 0) qe.mxs[(int64_t)m * (ldy / 32) + oc_g / 32] = (unsigned char)(ex + 127);
        }
      }
    }
  } else if (glu) {  // out col 16p + j = silu(gate col 32p + j) * up col 32p + 16 + j, 8 per thread-step
    constexpr int VPR = BN / 16;
    for (int v = threadIdx.x; v < rows * VPR; v += NTHR) {
      const int r = v / VPR, oc = (v - r * VPR) * 8;
      const int p = oc >> 4, j = oc & 15;
      const int cg = 32 * p + j, m = m0 + r0 + r, ng = n0 + cg;
      if (m >= M || ng >= N) continue;  // N % 32 == 0: the whole gate|up pair exists
      u16x8 o;
      float gx[8], ux[8];
      Img::ld8(ct, r, cg, gx);
      Img::ld8(ct, r, cg + 16, ux);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float gv = gx[e], uv = ux[e];
        if (bias) { gv += bf2f(bias[ng + e]); uv += bf2f(bias[ng + 16 + e]); }
        o[e] = f2bf(silu(gv) * uv);
      }
      bf16_t* dst = Y + (int64_t)m * ldy + n0 / 2 + oc;
      if (ng + 16 + 7 < N && (ldy & 7) == 0) *reinterpret_cast<u16x8*>(dst) = o;
      else
        for (int e = 0; e < 8 && ng + 16 + e < N; ++e) dst[e] = o[e];
    }
  } else {  // bf16 rows: 8 values (16 B) per thread-step
    constexpr int VPR = BN / 8;
    for (int v = threadIdx.x; v < rows * VPR; v += NTHR) {
      const int r = v / VPR, c = (v - r * VPR) * 8;
      const int m = m0 + r0 + r, n = n0 + c;
      if (m >= M || n >= N) continue;
      u16x8 o;
      float xv[8];
      Img::ld8(ct, r, c, xv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float x = xv[e];
        if (bias && n + e < N) x += bf2f(bias[n + e]);
        o[e] = f2bf(apply_act(x, act));
      }
      bf16_t* dst = Y + (int64_t)m * ldy + n;
      if (n + 7 < N && (ldy & 7) == 0) *reinterpret_cast<u16x8*>(dst) = o;
      else
        for (int e = 0; e < 8 && n + e < N; ++e) dst[e] = o[e];
    }
  }
}

// Cooperative GEMM epilogue through LDS. A wave's accumulators (MT x NT mfma_f32_16x16x32 tiles in
// the C layout: lane (li = lane & 15, g = lane >> 4) holds rows 4g..4g+3 of column li) are written
// row-major into a padded fp32 image in LDS, then every thread stores 16 B row-contiguous pieces:
// fp32 split-K slabs (part != nullptr, [M][N] of this slice) or bf16 Y with bias / activation /
// SwiGLU (16-row interleaved gate|up) applied on the way. Replaces per-lane 2-/4-byte stores of
// every accumulator element, whose issue cost dominated small tiles (an 8-k-step 128x128 tile spent
// ~10 us in the store tail). The tile is processed in row chunks that fit LDSB bytes; the caller
// must have drained every load into / read from that LDS region.
template <int BM, int BN, int MT, int NT, int NTHR, int LDSB>
__device__ __forceinline__ void tile_store_lds(const f32x4 (&acc)[MT][NT], char* lds, int wrow0, int wcol0, int m0,
                                               int n0, int M, int N, float* __restrict__ part,
                                               bf16_t* __restrict__ Y, int64_t ldy, const bf16_t* __restrict__ bias,
                                               int act, int glu, const QkvEpi& qe = QkvEpi{}) {
  using Img = EpiImg<BN>;
  constexpr int RMAX = LDSB / (Img::LDW * 4);
  constexpr int R = (RMAX >= BM ? BM : RMAX) / 16 * 16;
  static_assert(R >= 16, "LDS too small for a 16-row epilogue chunk");
  float* ct = reinterpret_cast<float*>(lds);
  const int lane = threadIdx.x & 63, li = lane & 15, g = lane >> 4;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // every wave is done reading the operand stages
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  for (int r0 = 0; r0 < BM; r0 += R) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int rb = wrow0 + mt * 16;  // a 16-row block is entirely inside or outside the chunk
      if (rb < r0 || rb >= r0 + R) continue;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) ct[Img::at(rb - r0 + 4 * g + i, wcol0 + nt * 16 + li)] = acc[mt][nt][i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int rows = BM - r0 < R ? BM - r0 : R;  // the last chunk may be shorter
    img_store_rows<BN, NTHR, R>(ct, rows, r0, m0, n0, M, N, part, Y, ldy, bias, act, glu, qe);
    if (r0 + R < BM) {  // the next chunk overwrites the image
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
  }
}

// In-launch split-K combine (guide "Projection GEMM at M = 256" item 2, write-through form; the
// hand-off is row 1 of MI355X_MICROARCH "Valid forms"): every K-slice workgroup of a tile stores
// its accumulators write-through (sc1, aux 16) into its slab of the tile's workspace region, EVERY
// wave drains its stores, then one lane takes a ticket on the tile's counter (relaxed agent atomic).
// The workgroup that draws ticket S-1 reads all S slabs back with sc1 loads (every load of the
// handed-off bytes is sc1, so no acquire fence), summing in slice order 0..S-1 - bit-identical to
// the separate splitk_reduce kernel whatever the arrival order - and finishes the tile; it also
// resets the counter for the next launch (counters start zeroed). Returns true in that workgroup.
// Slab layout: per wave, per (mt, nt) accumulator tile, 64 lanes x 16 B = one 1-KiB row, so each
// store / load wave-instruction moves a whole contiguous KiB. The slabs are read G at a time (all
// loads of a group issued before any add) so the reducer pays ceil(S / G) round trips, not S, and
// no load sits behind a per-element condition (a select after the load instead).
template <int MT, int NT>
__device__ __forceinline__ bool splitk_combine(f32x4 (&acc)[MT][NT], float* ws, int* cnt, int tile, int S, int z,
                                               int wid, int nwaves, int lane, int* lds_word) {
  constexpr int G = MT * NT * 4 <= 32 ? 4 : (MT * NT * 4 <= 64 ? 2 : 1);
  const int tile_f = nwaves * MT * NT * 256;  // floats per slab
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(ws + (int64_t)tile * S * tile_f, (short)0,
                                                    (int)((uint32_t)S * (uint32_t)tile_f * 4u), 0x00020000);
  const uint32_t base = (uint32_t)((wid * MT * NT * 64 + lane) * 16);
  const uint32_t slab_b = (uint32_t)tile_f * 4u;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[mt][nt]), rs,
                                             base + (uint32_t)((mt * NT + nt) * 1024), (uint32_t)z * slab_b, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains before the ticket
  __syncthreads();
  if (threadIdx.x == 0) *lds_word = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*lds_word != S - 1) return false;
  if (threadIdx.x == 0) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int s0 = 0; s0 < S; s0 += G) {
    u32x4 v[G][MT][NT];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const uint32_t so = (uint32_t)min(s0 + j, S - 1) * slab_b;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          v[j][mt][nt] = __builtin_amdgcn_raw_buffer_load_b128(rs, base + (uint32_t)((mt * NT + nt) * 1024), so, 16);
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const bool use = s0 + j < S;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const f32x4 p = __builtin_bit_cast(f32x4, v[j][mt][nt]);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[mt][nt][i] += use ? p[i] : 0.f;
        }
    }
  }
  return true;
}

#define HIP_CHECK_LAUNCH()                                                            \
  do {                                                                                   \
    hipError_t e__ = hipGetLastError();                                                  \
    if (e__ != hipSuccess) throw std::runtime_error(std::string("HIP launch failed: ") + \
                                                    hipGetErrorString(e__));             \
  } while (0)
