// Tensor-parallel linear layers on MFMA (reference: F.linear -> cuBLAS
// in FastLinear/TensorParallel{Column,Row}Linear, utils/layers.py:39-179, with bias and
// activation as separate ATen kernels).
//
//   Y[M, N] = epilogue( X[M, K] . W[N, K]^T )    X, W bf16 (W optionally fp8-e4m3 + per-row scale)
//   epilogue: (* w_scale[n]) (+ bias[n]) then act (gelu_tanh | gelu | relu) or SwiGLU
//   SwiGLU ("silu_glu"): W rows are interleaved in 16-row groups at load time, group 2p = gate
//   rows [16p, 16p+16), group 2p+1 = up rows [16p, 16p+16); the kernel writes
//   Y[:, 16p + i] = silu(gate) * up, so the [M, 2F] intermediate never reaches HBM.
//
// Kernel family (launch_gemm picks one per call; explicit hints and the autotuned plan table,
// ops/autotune.py, override the static planner):
//  * gemm_stream / gemm_stream2 (M <= 16, fp8 decode candidates): weight streaming straight into
//    VGPRs (non-temporal), X staged once per chunk in LDS, 3-deep register ring, split-K slabs.
//  * gemm_tiled<BM, BN, NS, WNT, F8> (decode / mid M): 64x64, 64x128 or 128x128 tiles, 4 waves,
//    both operands by global_load_lds into XOR-swizzled 128-B-row LDS images, an NS-stage ring
//    (2-6) waited with counted vmcnt across raw barriers, split-K over grid.y with fp32 slabs that
//    the NEXT kernel sums (add_norm, rope) or splitk_reduce; F8 = fp8 weight tiles (W8A16).
//  * gemm_streamk: persistent stream-K variant of the tiled kernel (in-kernel last-arriver combine).
//  * gemm_big<F8> (prefill, M >= ~1K): 256x256 tile, 8 waves, 128 KiB double buffer whose K-tile
//    t+2 is restaged while t is still being multiplied; F8 = W8A8 on the MX-fp8 matrix cores.
//  * gemm_f8f8: tiled W8A8 for fp8 shapes too small for the 256x256 tile.
// Split-K partial slabs never leave a call unless gemm_partial_slabs() says so (one source of
// truth shared with the Python wrapper).
#include "common.h"

#include <mutex>
#include <unordered_map>

// -------------------------------------------------------------------------------------------
// helpers
// -------------------------------------------------------------------------------------------
// 16 fp8-e4m3 (one 16-B word) -> two bf16x8 fragments
__device__ __forceinline__ void fp8x16_to_bf16(const u32x4& w, s16x8& f0, s16x8& f1) {
  const unsigned wd[4] = {w[0], w[1], w[2], w[3]};
  short o[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    f32x2 lo = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], false);
    f32x2 hi = __builtin_amdgcn_cvt_pk_f32_fp8(wd[q], true);
    o[4 * q + 0] = (short)f2bf(lo[0]);
    o[4 * q + 1] = (short)f2bf(lo[1]);
    o[4 * q + 2] = (short)f2bf(hi[0]);
    o[4 * q + 3] = (short)f2bf(hi[1]);
  }
  f0 = s16x8{o[0], o[1], o[2], o[3], o[4], o[5], o[6], o[7]};
  f1 = s16x8{o[8], o[9], o[10], o[11], o[12], o[13], o[14], o[15]};
}

__device__ __forceinline__ float epi_value(float v, int n, const float* wscale, const bf16_t* bias, int act) {
  if (wscale) v *= wscale[n];
  if (bias) v += bf2f(bias[n]);
  return apply_act(v, act);
}

// -------------------------------------------------------------------------------------------
// weight-streaming GEMM (M <= 128: decode / small batches)
// grid (ceil(N / (64*NT)), SPLITK), block 256 = 4 waves; wave w owns NT 16-column tiles.
// Per K-chunk of KC: X[0:16*MT, chunk] is staged ONCE per workgroup into LDS by 16-byte
// global_load_lds (lane-linear image, XOR swizzle applied on the source address: rule 21), and
// shared by the 4 waves; each wave streams its W rows straight into VGPRs (non-temporal: read
// once per step), 32 B per lane = a full 128-B line per 4 lanes. W for chunk c+1 and X for chunk
// c+1 are issued before the MFMAs of chunk c (register ring of 2 named buffers, static indexing).
// -------------------------------------------------------------------------------------------
template <int MT, int NT, int KC, bool FP8W>
struct StreamCfg {
  static constexpr int ROWS = MT * 16;
  static constexpr int RB = KC * 2;                     // LDS row bytes
  static constexpr int XBYTES = ROWS * RB;              // one X chunk
  static constexpr int NG = KC / 64;                    // 64-k groups per chunk
  static constexpr int WV = FP8W ? 1 : 2;               // u32x4 per lane per (nt, group)
  static constexpr int SW = (KC / 8 - 1) < 15 ? (KC / 8 - 1) : 15;  // swizzle mask (chunks)
  static constexpr int XINST = XBYTES / 1024 / 4;       // glds per wave per chunk
  static_assert(XBYTES % 4096 == 0, "X chunk must be a multiple of 4 KiB (4 waves x 1 KiB)");
};

template <int MT, int NT, int KC, bool FP8W>
__device__ __forceinline__ void stream_stage_x(const bf16_t* __restrict__ X, int64_t ldx, int M, int K, int kc0,
                                               char* xbuf, int w, int lane) {
  using C = StreamCfg<MT, NT, KC, FP8W>;
#pragma unroll
  for (int i = 0; i < C::XINST; ++i) {
    const int inst = i * 4 + w;
    const int o = inst * 1024 + lane * 16;
    const int row = o / C::RB;
    const int pc = (o % C::RB) >> 4;
    const int gc = pc ^ (row & C::SW);
    const int k = min(kc0 + gc * 8, K - 8);
    const bf16_t* src = X + (int64_t)min(row, M - 1) * ldx + k;
    __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(xbuf + inst * 1024), 16, 0, 0);
  }
}

template <int MT, int NT, int KC, bool FP8W>
__device__ __forceinline__ void stream_load_w(const char* const (&wrow)[NT], int kc0, int K, int g,
                                              u32x4 (&wr)[NT][KC / 64][FP8W ? 1 : 2]) {
  constexpr int WB = FP8W ? 1 : 2;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int q = 0; q < KC / 64; ++q) {
      int k = kc0 + 64 * q + 16 * g;
      k = k < K ? k : 0;  // tail lanes read a valid address; their fragments are zeroed at use
      const u32x4* p = reinterpret_cast<const u32x4*>(wrow[nt] + (int64_t)k * WB);
      wr[nt][q][0] = __builtin_nontemporal_load(p);
      if constexpr (!FP8W) wr[nt][q][1] = __builtin_nontemporal_load(p + 1);
    }
}

// 8 fp8-e4m3 (two dwords) -> one bf16x8 fragment
__device__ __forceinline__ s16x8 fp8x8_to_bf16(unsigned w0, unsigned w1) {
  const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8(w0, false), b = __builtin_amdgcn_cvt_pk_f32_fp8(w0, true);
  const f32x2 c = __builtin_amdgcn_cvt_pk_f32_fp8(w1, false), d = __builtin_amdgcn_cvt_pk_f32_fp8(w1, true);
  return s16x8{(short)f2bf(a[0]), (short)f2bf(a[1]), (short)f2bf(b[0]), (short)f2bf(b[1]),
               (short)f2bf(c[0]), (short)f2bf(c[1]), (short)f2bf(d[0]), (short)f2bf(d[1])};
}

template <int MT, int NT, int KC, bool FP8W, bool TAIL>
__device__ __forceinline__ void stream_compute(const char* xbuf, const u32x4 (&wr)[NT][KC / 64][FP8W ? 1 : 2],
                                               f32x4 (&acc)[MT][NT], int kc0, int K, int li, int g) {
  using C = StreamCfg<MT, NT, KC, FP8W>;
  const s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int q = 0; q < C::NG; ++q) {
    const bool ok = !TAIL || (kc0 + 64 * q + 16 * g < K);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      s16x8 b[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        if constexpr (FP8W) b[nt] = fp8x8_to_bf16(wr[nt][q][0][2 * s], wr[nt][q][0][2 * s + 1]);
        else b[nt] = *reinterpret_cast<const s16x8*>(&wr[nt][q][s]);
        if (TAIL && !ok) b[nt] = z;
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int r = mt * 16 + li;
        const int c = 8 * q + 2 * g + s;
        s16x8 a = *reinterpret_cast<const s16x8*>(xbuf + r * C::RB + ((c ^ (r & C::SW)) << 4));
        if (TAIL && !ok) a = z;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[nt], acc[mt][nt], 0, 0, 0);
      }
    }
  }
}

template <int MT, int NT, int KC, bool FP8W>
__global__ __launch_bounds__(256, 2) void gemm_stream_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                             const void* __restrict__ Wv, int64_t ldw,
                                                             const float* __restrict__ wscale,
                                                             const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                             int64_t ldy, float* __restrict__ part, int M, int N, int K,
                                                             int act, int glu) {
  using C = StreamCfg<MT, NT, KC, FP8W>;
  __shared__ __attribute__((aligned(16))) char xs[2 * C::XBYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (64 * NT) + w * (16 * NT);
  const int split = blockIdx.y, nsplit = gridDim.y;
  const int nck = (K + KC - 1) / KC;
  const int cb = (int)((int64_t)nck * split / nsplit), ce = (int)((int64_t)nck * (split + 1) / nsplit);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int WB = FP8W ? 1 : 2;
  const char* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    wrow[nt] = (const char*)Wv + (int64_t)min(n0 + nt * 16 + li, N - 1) * ldw * WB;  // + k*WB per load

  u32x4 wA[NT][KC / 64][FP8W ? 1 : 2], wB[NT][KC / 64][FP8W ? 1 : 2];
  const bool tail_k = (K % KC) != 0;
  if (cb < ce) {
    stream_stage_x<MT, NT, KC, FP8W>(X, ldx, M, K, cb * KC, xs, w, lane);
    stream_load_w<MT, NT, KC, FP8W>(wrow, cb * KC, K, g, wA);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  for (int c = cb; c < ce; c += 2) {
    // ---- even chunk: compute from wA / buffer 0, prefetch chunk c+1 into wB / buffer 1
    if (c + 1 < ce) {
      stream_stage_x<MT, NT, KC, FP8W>(X, ldx, M, K, (c + 1) * KC, xs + C::XBYTES, w, lane);
      stream_load_w<MT, NT, KC, FP8W>(wrow, (c + 1) * KC, K, g, wB);
    }
    if (tail_k && c == nck - 1) stream_compute<MT, NT, KC, FP8W, true>(xs, wA, acc, c * KC, K, li, g);
    else stream_compute<MT, NT, KC, FP8W, false>(xs, wA, acc, c * KC, K, li, g);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (c + 1 >= ce) break;
    // ---- odd chunk: compute from wB / buffer 1, prefetch chunk c+2 into wA / buffer 0
    if (c + 2 < ce) {
      stream_stage_x<MT, NT, KC, FP8W>(X, ldx, M, K, (c + 2) * KC, xs, w, lane);
      stream_load_w<MT, NT, KC, FP8W>(wrow, (c + 2) * KC, K, g, wA);
    }
    if (tail_k && c + 1 == nck - 1) stream_compute<MT, NT, KC, FP8W, true>(xs + C::XBYTES, wB, acc, (c + 1) * KC, K, li, g);
    else stream_compute<MT, NT, KC, FP8W, false>(xs + C::XBYTES, wB, acc, (c + 1) * KC, K, li, g);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  // ---- epilogue (C layout: col = lane&15 -> n, row = 4*(lane>>4)+i -> m) --------------------
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * g + i;
      if (m >= M) continue;
      if (nsplit > 1) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = n0 + nt * 16 + li;
          if (n < N) part[((int64_t)split * M + m) * N + n] = acc[mt][nt][i] * (wscale ? wscale[n] : 1.f);
        }
      } else if (glu) {
#pragma unroll
        for (int p = 0; p < NT / 2; ++p) {
          const int ng = n0 + 2 * p * 16 + li, nu = ng + 16;
          if (nu < N) {
            const float gv = epi_value(acc[mt][2 * p][i], ng, wscale, bias, ACT_NONE);
            const float uv = epi_value(acc[mt][2 * p + 1][i], nu, wscale, bias, ACT_NONE);
            Y[(int64_t)m * ldy + n0 / 2 + p * 16 + li] = f2bf(silu(gv) * uv);
          }
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = n0 + nt * 16 + li;
          if (n < N) Y[(int64_t)m * ldy + n] = f2bf(epi_value(acc[mt][nt][i], n, wscale, bias, act));
        }
      }
    }
  }
}

// -------------------------------------------------------------------------------------------
// weight-streaming GEMM, v2: register-staged X + 3-deep W register ring (2 chunks in flight).
// v1 stages X with global_load_lds; while an LDS-DMA is in flight hipcc drains vmcnt(0) at every
// use of an ordinary load (guide §5 'Pipelining across barriers'), which caps v1 at ONE W chunk
// in flight per wave. Here every load is an ordinary global_load, issued in the order
// X(c+1), W(c+2) before the MFMAs of chunk c, so the compiler's counted vmcnt waits only for what
// each consumer needs: the ds_write of X(c+1) waits for X(c+1), not for W(c+2).
// Same tile/K mapping as v1 (verified by tests/test_kernel_emulation.py), same epilogue.
// -------------------------------------------------------------------------------------------
template <int MT, int NT, int KC, bool FP8W>
struct Stream2Cfg {
  static constexpr int ROWS = MT * 16;
  static constexpr int RB = KC * 2;
  static constexpr int XBYTES = ROWS * RB;
  static constexpr int CPR = KC / 8;                      // 16-B chunks per X row
  static constexpr int XPT = ROWS * CPR / 256;            // X chunks per thread per K-chunk
  static constexpr int SW = (CPR - 1) < 15 ? (CPR - 1) : 15;
  static_assert((ROWS * CPR) % 256 == 0, "X chunk must split evenly over 256 threads");
};

template <int MT, int NT, int KC, bool FP8W>
__device__ __forceinline__ void stream2_load_x(const bf16_t* __restrict__ X, int64_t ldx, int M, int K, int kc0,
                                               u32x4 (&xr)[Stream2Cfg<MT, NT, KC, FP8W>::XPT]) {
  using C = Stream2Cfg<MT, NT, KC, FP8W>;
#pragma unroll
  for (int i = 0; i < C::XPT; ++i) {
    const int id = threadIdx.x + i * 256;
    const int row = id / C::CPR, c = id % C::CPR;
    const int k = min(kc0 + c * 8, K - 8);
    xr[i] = *reinterpret_cast<const u32x4*>(X + (int64_t)min(row, M - 1) * ldx + k);
  }
}

template <int MT, int NT, int KC, bool FP8W>
__device__ __forceinline__ void stream2_store_x(char* xbuf, const u32x4 (&xr)[Stream2Cfg<MT, NT, KC, FP8W>::XPT]) {
  using C = Stream2Cfg<MT, NT, KC, FP8W>;
#pragma unroll
  for (int i = 0; i < C::XPT; ++i) {
    const int id = threadIdx.x + i * 256;
    const int row = id / C::CPR, c = id % C::CPR;
    *reinterpret_cast<u32x4*>(xbuf + row * C::RB + ((c ^ (row & C::SW)) << 4)) = xr[i];
  }
}

template <int MT, int NT, int KC, bool FP8W>
__global__ __launch_bounds__(256, 2) void gemm_stream2_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                              const void* __restrict__ Wv, int64_t ldw,
                                                              const float* __restrict__ wscale,
                                                              const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                              int64_t ldy, float* __restrict__ part, int M, int N,
                                                              int K, int act, int glu) {
  using C = Stream2Cfg<MT, NT, KC, FP8W>;
  __shared__ __attribute__((aligned(16))) char xs[2 * C::XBYTES];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (64 * NT) + w * (16 * NT);
  const int split = blockIdx.y, nsplit = gridDim.y;
  const int nck = (K + KC - 1) / KC;
  const int cb = (int)((int64_t)nck * split / nsplit), ce = (int)((int64_t)nck * (split + 1) / nsplit);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr int WB = FP8W ? 1 : 2;
  const char* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wrow[nt] = (const char*)Wv + (int64_t)min(n0 + nt * 16 + li, N - 1) * ldw * WB;

  u32x4 w0[NT][KC / 64][FP8W ? 1 : 2], w1[NT][KC / 64][FP8W ? 1 : 2], w2[NT][KC / 64][FP8W ? 1 : 2];
  u32x4 xr[C::XPT];
  const bool tail_k = (K % KC) != 0;
  if (cb < ce) {
    stream2_load_x<MT, NT, KC, FP8W>(X, ldx, M, K, cb * KC, xr);
    stream_load_w<MT, NT, KC, FP8W>(wrow, cb * KC, K, g, w0);
    if (cb + 1 < ce) stream_load_w<MT, NT, KC, FP8W>(wrow, (cb + 1) * KC, K, g, w1);
    stream2_store_x<MT, NT, KC, FP8W>(xs, xr);
    __syncthreads();
  }
  // Steady state: branch-free steps (every prefetch valid), so hipcc's vmcnt bookkeeping stays
  // exact and it waits only for the chunk being consumed (a load under an `if` makes the counts
  // path-dependent and the compiler then drains vmcnt(0) before re-issuing - measured).
#define STREAM2_STEADY(CUR, NXT2)                                                                             \
  {                                                                                                          \
    stream2_load_x<MT, NT, KC, FP8W>(X, ldx, M, K, (c + 1) * KC, xr);                                        \
    stream_load_w<MT, NT, KC, FP8W>(wrow, (c + 2) * KC, K, g, NXT2);                                         \
    __builtin_amdgcn_sched_barrier(0); /* keep the prefetch ahead of the MFMAs (hipcc sinks it) */           \
    stream_compute<MT, NT, KC, FP8W, false>(xs + ((c - cb) & 1) * C::XBYTES, CUR, acc, c * KC, K, li, g);    \
    __builtin_amdgcn_sched_barrier(0);                                                                       \
    stream2_store_x<MT, NT, KC, FP8W>(xs + ((c + 1 - cb) & 1) * C::XBYTES, xr);                              \
    __syncthreads();                                                                                         \
    ++c;                                                                                                     \
  }
#define STREAM2_REM(CUR, NXT2)                                                                                \
  {                                                                                                          \
    if (c >= ce) break;                                                                                      \
    if (c + 1 < ce) stream2_load_x<MT, NT, KC, FP8W>(X, ldx, M, K, (c + 1) * KC, xr);                        \
    if (c + 2 < ce) stream_load_w<MT, NT, KC, FP8W>(wrow, (c + 2) * KC, K, g, NXT2);                         \
    const char* xb = xs + ((c - cb) & 1) * C::XBYTES;                                                        \
    if (tail_k && c == nck - 1) stream_compute<MT, NT, KC, FP8W, true>(xb, CUR, acc, c * KC, K, li, g);      \
    else stream_compute<MT, NT, KC, FP8W, false>(xb, CUR, acc, c * KC, K, li, g);                            \
    if (c + 1 < ce) stream2_store_x<MT, NT, KC, FP8W>(xs + ((c + 1 - cb) & 1) * C::XBYTES, xr);              \
    __syncthreads();                                                                                         \
    ++c;                                                                                                     \
  }
  int c = cb;
  for (; c + 4 < ce;) {  // 3 chunks per iteration; chunks c+2..c+4 exist -> all prefetches valid
    STREAM2_STEADY(w0, w2)
    STREAM2_STEADY(w1, w0)
    STREAM2_STEADY(w2, w1)
  }
  do {  // remaining <= 4 chunks (ring rotation continues at w0); also handles the K tail chunk
    STREAM2_REM(w0, w2)
    STREAM2_REM(w1, w0)
    STREAM2_REM(w2, w1)
    STREAM2_REM(w0, w2)
  } while (0);
#undef STREAM2_STEADY
#undef STREAM2_REM

#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * g + i;
      if (m >= M) continue;
      if (nsplit > 1) {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = n0 + nt * 16 + li;
          if (n < N) part[((int64_t)split * M + m) * N + n] = acc[mt][nt][i] * (wscale ? wscale[n] : 1.f);
        }
      } else if (glu) {
#pragma unroll
        for (int p = 0; p < NT / 2; ++p) {
          const int ng = n0 + 2 * p * 16 + li, nu = ng + 16;
          if (nu < N) {
            const float gv = epi_value(acc[mt][2 * p][i], ng, wscale, bias, ACT_NONE);
            const float uv = epi_value(acc[mt][2 * p + 1][i], nu, wscale, bias, ACT_NONE);
            Y[(int64_t)m * ldy + n0 / 2 + p * 16 + li] = f2bf(silu(gv) * uv);
          }
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const int n = n0 + nt * 16 + li;
          if (n < N) Y[(int64_t)m * ldy + n] = f2bf(epi_value(acc[mt][nt][i], n, wscale, bias, act));
        }
      }
    }
  }
}

// split-K reduction + epilogue: part [S, M, N] fp32 (w_scale already applied). The slabs are read in groups of 8 with
// every load of a group issued before its adds (one memory round trip per group, not per slab; adds in slab order).
__device__ __forceinline__ float slab_sum(const float* __restrict__ part, int S, int64_t stride, int64_t off) {
  constexpr int SG = 8;
  float v = 0.f;
  for (int s0 = 0; s0 < S; s0 += SG) {
    float x[SG];
#pragma unroll
    for (int g = 0; g < SG; ++g) x[g] = part[(int64_t)min(s0 + g, S - 1) * stride + off];
#pragma unroll
    for (int g = 0; g < SG; ++g) v += s0 + g < S ? x[g] : 0.f;
  }
  return v;
}

__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                            int64_t ldy, int act, int glu) {
  const int m = blockIdx.y;
  const int nout = glu ? N / 2 : N;
  const int64_t stride = (int64_t)M * N;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nout; c += gridDim.x * blockDim.x) {
    if (glu) {
      const int p = c >> 4, i = c & 15;
      const int ng = 32 * p + i, nu = ng + 16;
      float gv = slab_sum(part, S, stride, (int64_t)m * N + ng), uv = slab_sum(part, S, stride, (int64_t)m * N + nu);
      if (bias) { gv += bf2f(bias[ng]); uv += bf2f(bias[nu]); }
      Y[(int64_t)m * ldy + c] = f2bf(silu(gv) * uv);
    } else {
      float v = slab_sum(part, S, stride, (int64_t)m * N + c);
      if (bias) v += bf2f(bias[c]);
      Y[(int64_t)m * ldy + c] = f2bf(apply_act(v, act));
    }
  }
}

// -------------------------------------------------------------------------------------------
// tiled GEMM (prefill / large M), bf16 weights. Tile BM x BN x 64, 4 waves in 2x2, each wave
// (BM/2) x (BN/2) = MTW x NTW mfma_f32_16x16x32 accumulators. Both operands staged by 16-byte
// global_load_lds into an XOR-swizzled image (chunk ^= row & 7: conflict-free ds_read_b128),
// double-buffered; XCD-aware tile order (T1). The tile is chosen per call so small-N tensor-
// parallel shards still produce >= ~256 workgroups (128x128, 64x128 or 64x64).
// -------------------------------------------------------------------------------------------
constexpr int TBK = 64;

// F8: B (weights) is fp8-e4m3, one byte per element: its LDS image is [BN][64 B] with the 16-B chunk
// q of row r stored at q ^ ((r >> 2) & 3) (ds_read_b64 fragment reads conflict-free, bank-simulated).
template <int BN, bool F8, int NW = 4>
struct TiledB {
  static constexpr int ROWB = F8 ? 64 : 128;  // LDS bytes per B row per 64-k stage
  static constexpr int BYTES = BN * ROWB;
  static constexpr int LOADS = F8 ? BN / (16 * NW) : BN / (8 * NW);  // glds per wave per stage
};

template <int BM, int BN, bool WNT = false, bool F8 = false, int NW = 4>
__device__ __forceinline__ void tiled_stage(const bf16_t* __restrict__ A, int64_t lda, int M, const void* __restrict__ Bv,
                                            int64_t ldb, int N, int K, int m0, int n0, int k0, char* sA, char* sB,
                                            int w, int lane) {
  // one wave-instruction = 1 KiB = 8 rows x 128 B; A needs BM/8 of them, B BN/8 (NW waves share)
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split evenly over the waves");
#pragma unroll
  for (int it = 0; it < BM / (8 * NW); ++it) {
    const int inst = it * NW + w;
    const int row = inst * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (row & 7);
    const int kc = min(k0 + c * 8, K - 8);
    const bf16_t* ga = A + (int64_t)min(m0 + row, M - 1) * lda + kc;
    __builtin_amdgcn_global_load_lds((const void*)ga, (LDS_AS void*)(sA + inst * 1024), 16, 0, 0);
  }
  if constexpr (F8) {
    const unsigned char* B = reinterpret_cast<const unsigned char*>(Bv);
#pragma unroll
    for (int it = 0; it < BN / (16 * NW); ++it) {  // one wave-instruction = 16 rows x 64 B
      const int inst = it * NW + w;
      const int row = inst * 16 + (lane >> 2);
      const int gq = (lane & 3) ^ ((row >> 2) & 3);
      const int kc = min(k0 + gq * 16, K - 16);
      const unsigned char* gb = B + (int64_t)min(n0 + row, N - 1) * ldb + kc;
      __builtin_amdgcn_global_load_lds((const void*)gb, (LDS_AS void*)(sB + inst * 1024), 16, 0, WNT ? 2 : 0);
    }
  } else {
    const bf16_t* B = reinterpret_cast<const bf16_t*>(Bv);
#pragma unroll
    for (int it = 0; it < BN / (8 * NW); ++it) {
      const int inst = it * NW + w;
      const int row = inst * 8 + (lane >> 3);
      const int c = (lane & 7) ^ (row & 7);
      const int kc = min(k0 + c * 8, K - 8);
      const bf16_t* gb = B + (int64_t)min(n0 + row, N - 1) * ldb + kc;
      // weights read once per step (single M tile): non-temporal (aux = 2), guide 'nt-weights'
      __builtin_amdgcn_global_load_lds((const void*)gb, (LDS_AS void*)(sB + inst * 1024), 16, 0, WNT ? 2 : 0);
    }
  }
}

template <int MTW, int NTW, bool MASK, bool F8 = false>
__device__ __forceinline__ void tiled_compute(const char* sA, const char* sB, f32x4 (&acc)[MTW][NTW], int wr, int wc,
                                              int li, int g, int k0, int K) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = 4 * s + g;
    const bool valid = !MASK || (k0 + c * 8 < K);
    const s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    s16x8 a[MTW], b[NTW];
#pragma unroll
    for (int t = 0; t < MTW; ++t) {
      const int ra = wr * (MTW * 16) + t * 16 + li;
      a[t] = *reinterpret_cast<const s16x8*>(sA + ra * 128 + ((c ^ (ra & 7)) << 4));
      if (MASK && !valid) a[t] = z;
    }
#pragma unroll
    for (int t = 0; t < NTW; ++t) {
      const int rb = wc * (NTW * 16) + t * 16 + li;
      if constexpr (F8) {  // k bytes [32 s + 8 g, +8) = half (g & 1) of 16-B chunk 2 s + g / 2
        const int pq = (2 * s + (g >> 1)) ^ ((rb >> 2) & 3);
        const u32x2 raw = *reinterpret_cast<const u32x2*>(sB + rb * 64 + pq * 16 + (g & 1) * 8);
        b[t] = fp8x8_to_bf16(raw[0], raw[1]);
      } else {
        b[t] = *reinterpret_cast<const s16x8*>(sB + rb * 128 + ((c ^ (rb & 7)) << 4));
      }
      if (MASK && !valid) b[t] = z;
    }
#pragma unroll
    for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
      for (int nt = 0; nt < NTW; ++nt)
        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
  }
}

// s_waitcnt vmcnt(N) with expcnt / lgkmcnt left alone (gfx9 encoding: vmcnt[3:0] + [15:14])
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// wait until at most min(younger, MAXY) stages of LOADS instructions each are outstanding
template <int LOADS, int MAXY>
__device__ __forceinline__ void wait_vmcnt_upto(int younger) {
  if constexpr (MAXY <= 0) {
    wait_vmcnt<0>();
  } else {
    if (younger >= MAXY) wait_vmcnt<LOADS * MAXY>();
    else wait_vmcnt_upto<LOADS, MAXY - 1>(younger);
  }
}

// Barrier that lets global_load_lds stay in flight across it: __syncthreads()' release fence
// would emit vmcnt(0) and drain the prefetch (guide: "Pipelining across barriers").
__device__ __forceinline__ void lds_barrier() {
  // lgkmcnt(0) through the builtin (vmcnt / expcnt at their maxima), which the compiler's wait-count
  // pass accounts for: after an inline-asm wait it still believes earlier LDS reads are pending and
  // adds an lgkmcnt(0) in front of the next MFMA that uses their registers
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// NW = 4: waves 2 (M) x 2 (N); NW = 8 (256-row tiles, one workgroup per CU): waves 4 (M) x 2 (N),
// each 64 x BN/2 - mid-M shapes (TP-sharded decode at M = 256-512) are per-CU load-latency bound,
// so a wider tile moves fewer bytes per output through each CU's load path (guide: "Projection GEMM
// at M = 256").
template <int BM, int BN, int NS, bool WNT, bool F8 = false, int NW = 4>
__global__ __launch_bounds__(64 * NW) void gemm_tiled_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                         const void* __restrict__ B, int64_t ldb,
                                                         const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                         int64_t ldy, float* __restrict__ part, int M, int N, int K,
                                                         int act, int glu, const float* __restrict__ wscale,
                                                         int* __restrict__ cnt, QkvEpi qe) {
  constexpr int MTW = BM / (8 * NW), NTW = BN / 32;  // 16x16 tiles per wave (waves NW/2 x 2)
  constexpr int A_BYTES = BM * TBK * 2, B_BYTES = TiledB<BN, F8, NW>::BYTES, STAGE = A_BYTES + B_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const TileWork tw = tile_work(ntm, ntn, BM, BN);
  const int m0 = tw.m0, n0 = tw.n0, zk = tw.z;

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int a = 0; a < MTW; ++a)
#pragma unroll
    for (int b = 0; b < NTW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K (grid.y): slice z covers k-tiles [t0, t1); partial sums go to part[z] (fp32)
  const int nk_all = (K + TBK - 1) / TBK;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int t0 = zk * per, t1 = min(nk_all, t0 + per);
  if constexpr (NS == 2) {
    if (t0 < t1) {
      tiled_stage<BM, BN, WNT, F8, NW>(A, lda, M, B, ldb, N, K, m0, n0, t0 * TBK, smem, smem + A_BYTES, w, lane);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    for (int t = t0; t < t1; ++t) {
      const int cur = (t - t0) & 1;
      char* nA = smem + (cur ^ 1) * STAGE;
      char* cA = smem + cur * STAGE;
      if (t + 1 < t1) tiled_stage<BM, BN, WNT, F8, NW>(A, lda, M, B, ldb, N, K, m0, n0, (t + 1) * TBK, nA, nA + A_BYTES, w, lane);
      if (t + 1 == nk_all && (K % TBK)) tiled_compute<MTW, NTW, true, F8>(cA, cA + A_BYTES, acc, wr, wc, li, g, t * TBK, K);
      else tiled_compute<MTW, NTW, false, F8>(cA, cA + A_BYTES, acc, wr, wc, li, g, t * TBK, K);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
  } else {
    // NS-stage ring: stage t+NS-1 is issued while stage t is computed; the wait before compute
    // only covers stage t (the younger stages' LOADS instructions each stay in flight): no drain.
    constexpr int LOADS = BM / (8 * NW) + TiledB<BN, F8, NW>::LOADS;  // global_load_lds per wave per stage
#pragma unroll
    for (int j = 0; j < NS - 1; ++j)
      if (t0 + j < t1)
        tiled_stage<BM, BN, WNT, F8, NW>(A, lda, M, B, ldb, N, K, m0, n0, (t0 + j) * TBK, smem + j * STAGE,
                            smem + j * STAGE + A_BYTES, w, lane);
    int cur = 0;
    for (int t = t0; t < t1; ++t) {
      wait_vmcnt_upto<LOADS, NS - 2>(t1 - 1 - t);  // stages younger than t still in flight
      lds_barrier();  // stage t visible; every wave is past compute(t-1), so its buffer is free
      char* cA = smem + cur * STAGE;
      const int nxt = cur == 0 ? NS - 1 : cur - 1;  // (cur + NS - 1) % NS
      if (t + NS - 1 < t1) {
        char* nA = smem + nxt * STAGE;
        tiled_stage<BM, BN, WNT, F8, NW>(A, lda, M, B, ldb, N, K, m0, n0, (t + NS - 1) * TBK, nA, nA + A_BYTES, w, lane);
      }
      if (t + 1 == nk_all && (K % TBK)) tiled_compute<MTW, NTW, true, F8>(cA, cA + A_BYTES, acc, wr, wc, li, g, t * TBK, K);
      else tiled_compute<MTW, NTW, false, F8>(cA, cA + A_BYTES, acc, wr, wc, li, g, t * TBK, K);
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
  }
  // cnt: split-K slices combine in this launch (common.h splitk_combine); the last arriver of the
  // tile finishes it with the normal bf16 epilogue, the others are done
  if (cnt) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!splitk_combine<MTW, NTW>(acc, part, cnt, (n0 / BN) * ntm + m0 / BM, gridDim.y, zk, w, NW, lane,
                                  reinterpret_cast<int*>(smem)))
      return;
    part = nullptr;
  }
  if constexpr (!F8) {
    // QKV projection (RoPE + paged KV write) runs in the LDS-staged epilogue
    // (unsplit / combined plans only)
    if (qe.D) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tile_store_lds<BM, BN, MTW, NTW, 64 * NW, NS * STAGE>(acc, smem, wr * (MTW * 16), wc * (NTW * 16), m0, n0, M,
                                                             N, nullptr, Y, ldy, bias, act, glu, qe);
      return;
    }
  }
  // epilogue (C layout: col = lane&15 -> n, row = 4*(lane>>4)+i -> m)
  const int wn0 = n0 + wc * (NTW * 16);
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * (MTW * 16) + mt * 16 + 4 * g + i;
      if (m >= M) continue;
      if (part) {
        float* pr = part + ((int64_t)zk * M + m) * N;
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int n = wn0 + nt * 16 + li;
          if (n < N) pr[n] = F8 ? acc[mt][nt][i] * wscale[n] : acc[mt][nt][i];
        }
      } else if (glu) {
#pragma unroll
        for (int p = 0; p < NTW / 2; ++p) {
          const int ng = wn0 + 2 * p * 16 + li, nu = ng + 16;
          if (nu < N) {
            float gv = acc[mt][2 * p][i], uv = acc[mt][2 * p + 1][i];
            if constexpr (F8) { gv *= wscale[ng]; uv *= wscale[nu]; }
            if (bias) { gv += bf2f(bias[ng]); uv += bf2f(bias[nu]); }
            Y[(int64_t)m * ldy + wn0 / 2 + p * 16 + li] = f2bf(silu(gv) * uv);
          }
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int n = wn0 + nt * 16 + li;
          if (n < N) {
            float v = acc[mt][nt][i];
            if constexpr (F8) v *= wscale[n];
            if (bias) v += bf2f(bias[n]);
            Y[(int64_t)m * ldy + n] = f2bf(apply_act(v, act));
          }
        }
      }
    }
  }
}

// -------------------------------------------------------------------------------------------
// W8A8 big-tile GEMM (fp8 prefill, M >= ~1024; bf16 prompt batches take gemm_pp_kernel below):
// 256x256 tile of 128-element fp8 K-tiles, 8 waves (2 x 4), each wave 128x64 = 8x4 accumulators on the
// MX-fp8 16x16x128 MFMA. LDS = 2 buffers x {A rows 0-127, A rows 128-255, B rows 0-127, B rows 128-255}
// of 16 KiB = 128 KiB -> one workgroup per CU.
// Per K-tile t: (1) counted vmcnt(8) retires stage t while stage t+1 stays in flight, raw
// barrier; (2) every wave reads ALL its fragments of tile t into VGPRs (24 ds_read_b128) and
// runs the first half of its MFMAs; (3) barrier (lgkmcnt(0): all reads of buffer t&1 done) and
// stage t+2 is issued into that same buffer, then the second half of MFMAs. Prefetch distance
// is therefore ~1.5 K-tiles of MFMA time and no barrier ever drains the DMA queue (guide:
// "Pipelining across barriers", 3-buffer-equivalent depth in 2 buffers).
// Requires K % 64 == 0; rows beyond M / N are clamped on load and masked on store.
// -------------------------------------------------------------------------------------------
// M-tiles per tile group of the big-tile kernel's launch order (gemm_big_set_group; measured 4)
static int g_big_group_m = 4;
void gemm_big_set_group(int g) { g_big_group_m = g >= 1 && g <= 64 ? g : 4; }

// one MX-fp8 16x16x128 MFMA from two 16-B fragment halves per operand (unit E8M0 block scales)
__device__ __forceinline__ f32x4 mfma_f8x2(s16x8 a0, s16x8 a1, s16x8 b0, s16x8 b1, f32x4 c) {
  typedef int __attribute__((ext_vector_type(4))) i32x4_t;
  typedef int __attribute__((ext_vector_type(8))) i32x8_t;
  const i32x4_t al = __builtin_bit_cast(i32x4_t, a0), ah = __builtin_bit_cast(i32x4_t, a1);
  const i32x4_t bl = __builtin_bit_cast(i32x4_t, b0), bh = __builtin_bit_cast(i32x4_t, b1);
  const i32x8_t av = __builtin_shufflevector(al, ah, 0, 1, 2, 3, 4, 5, 6, 7);
  const i32x8_t bv = __builtin_shufflevector(bl, bh, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(av, bv, c, 0, 0, 0, 127, 0, 127);
}

// F8: both operands fp8-e4m3 (W8A8): a 128-element fp8 K-tile has exactly the byte layout of the
// 64-element bf16 one, so staging / LDS image / fragment addresses are shared; each (m, n) takes one
// MX-fp8 16x16x128 MFMA per K-tile (the two 16-B chunks 2g, 2g+1 of the lane's row), and the
// per-token x per-channel scales are applied in the epilogue.
template <bool F8>
__global__ __launch_bounds__(512, 1) void gemm_big_kernel(const void* __restrict__ A, int64_t lda,
                                                          const void* __restrict__ B, int64_t ldb,
                                                          const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                          int64_t ldy, int M, int N, int K, int act, int glu,
                                                          const float* __restrict__ xs, const float* __restrict__ ws,
                                                          int group_m) {
  constexpr int ES = F8 ? 1 : 2;  // operand bytes per element
  constexpr int HALF = 16384, BUF = 4 * HALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 2, wc = w & 3;
  const int ntn = (N + 255) / 256, ntm = (M + 255) / 256;
  // XCD-contiguous tile ranges, grouped GM M-tiles high: the 32 workgroups an XCD runs at once cover a
  // 4 x 8 block of tiles, so its L2 fills 4 A + 8 B panels per round instead of ~1 A + 32 B panels
  // (PMC: 4 TB/s of L2 fills and 47 % of wave cycles waiting before this)
  const int GM = group_m;
  const int tile = xcd_remap(blockIdx.x, ntn * ntm);
  const int grp = tile / (GM * ntn), gidx = tile - grp * (GM * ntn);
  const int gm = min(GM, ntm - grp * GM);
  const int m0 = (grp * GM + gidx % gm) * 256, n0 = (gidx / gm) * 256;
  const int nk = K * ES / 128;  // 128-byte K-tiles

  // staging: half h (0,1: A rows 128h.., 2,3: B rows 128(h-2)..), 2 x 1-KiB glds per wave; lane ->
  // row inst*8 + lane/8, LDS chunk lane&7 holding global chunk (lane&7) ^ (row&7) (swizzle on source)
  const char* src[4] = {(const char*)A, (const char*)A, (const char*)B, (const char*)B};
  const int64_t ld[4] = {lda * ES, lda * ES, ldb * ES, ldb * ES};  // bytes
  int64_t soff[4][2];
  int lofs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = i * 8 + w;
    const int row = inst * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ (row & 7);
    lofs[i] = inst * 1024;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const bool isA = h < 2;
      const int lim = isA ? M : N;
      const int r = min((isA ? m0 : n0) + (h & 1) * 128 + row, lim - 1);
      soff[h][i] = (int64_t)r * ld[h] + gc * 16;
    }
  }
  auto stage = [&](int t, char* buf) {
#pragma unroll
    for (int h = 0; h < 4; ++h)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        __builtin_amdgcn_global_load_lds((const void*)(src[h] + soff[h][i] + (int64_t)t * 128),
                                         (LDS_AS void*)(buf + h * HALF + lofs[i]), 16, 0, 0);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes within a buffer): A half wr, B half wc>>1 (+64 rows for odd wc)
  int aoff[8][2], boff[4][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    // bf16: k-half s; fp8: the lane's two 16-B chunks g, g + 4 (the same k permutation for A and B, the
    // conflict-free bf16 read pattern; chunks 2g, 2g + 1 hit the same banks)
    const int c = 4 * s + g;
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int r = m * 16 + li;
      aoff[m][s] = wr * HALF + r * 128 + ((c ^ (r & 7)) << 4);
    }
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int r = (wc & 1) * 64 + n * 16 + li;
      boff[n][s] = (2 + (wc >> 1)) * HALF + r * 128 + ((c ^ (r & 7)) << 4);
    }
  }

  stage(0, smem);
  if (nk > 1) stage(1, smem + BUF);
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * BUF;
    if (t + 1 < nk) wait_vmcnt<8>();
    else wait_vmcnt<0>();
    lds_barrier();  // stage t landed for every wave
    s16x8 a[8][2], b[4][2];
    {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int n = 0; n < 4; ++n) b[n][s] = *reinterpret_cast<const s16x8*>(cur + boff[n][s]);
#pragma unroll
      for (int m = 0; m < 8; ++m) a[m][s] = *reinterpret_cast<const s16x8*>(cur + aoff[m][s]);
    }
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {  // first half: n-tiles 0, 1
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n) acc[m][n] = mfma_f8x2(a[m][0], a[m][1], b[n][0], b[n][1], acc[m][n]);
    } else {
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][0], b[n][0], acc[m][n], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    }
    lds_barrier();  // every wave's reads of this buffer are complete -> restage it
    if (t + 2 < nk) stage(t + 2, cur);
    __builtin_amdgcn_s_setprio(1);
    if constexpr (F8) {  // second half: n-tiles 2, 3
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 2; n < 4; ++n) acc[m][n] = mfma_f8x2(a[m][0], a[m][1], b[n][0], b[n][1], acc[m][n]);
    } else {
#pragma unroll
      for (int m = 0; m < 8; ++m)
#pragma unroll
        for (int n = 0; n < 4; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[m][1], b[n][1], acc[m][n], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }

  // epilogue (C layout: col = lane&15 -> n, row = 4*(lane>>4)+i -> m)
  const int wn0 = n0 + wc * 64;
#pragma unroll
  for (int m = 0; m < 8; ++m) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = m0 + wr * 128 + m * 16 + 4 * g + i;
      if (row >= M) continue;
      const float sx = F8 ? xs[row] : 1.f;
      if (glu) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int ng = wn0 + 2 * p * 16 + li, nu = ng + 16;
          if (nu < N) {
            float gv = acc[m][2 * p][i], uv = acc[m][2 * p + 1][i];
            if constexpr (F8) { gv *= sx * ws[ng]; uv *= sx * ws[nu]; }
            if (bias) { gv += bf2f(bias[ng]); uv += bf2f(bias[nu]); }
            Y[(int64_t)row * ldy + wn0 / 2 + p * 16 + li] = f2bf(silu(gv) * uv);
          }
        }
      } else {
#pragma unroll
        for (int n = 0; n < 4; ++n) {
          const int col = wn0 + n * 16 + li;
          if (col < N) {
            float v = acc[m][n][i];
            if constexpr (F8) v *= sx * ws[col];
            if (bias) v += bf2f(bias[col]);
            Y[(int64_t)row * ldy + col] = f2bf(apply_act(v, act));
          }
        }
      }
    }
  }
}

// -------------------------------------------------------------------------------------------
// Ping-pong prefill GEMM (bf16, M >= ~1024): the shipped bf16 big-tile kernel (profiles/r5_gemm_pp).
// 256x256x64 tile, 8 waves = two groups of 4 (waves 0-3 / 4-7; one wave of each group per SIMD). Waves
// 4-7 pass one extra barrier before the K-loop, so on every SIMD one wave's compute segment runs beside
// its partner's load segment (guide "The 256^2 8-phase template", MI355X_MICROARCH "Two waves per SIMD").
//   * LDS = 2 buffers x 4 slots of 16 KiB: slot 0 = A half 0, 1 = B half 0, 2 = B half 1, 3 = A half 1.
//     A half h holds block rows {128 r + 64 h + i}, B half h block columns {64 c + 32 h + j}, so each
//     wave's contiguous 128x64 output splits into four 64x32 quadrants Q(mq, nq) reading A slot mq and
//     B slot nq. Rows are 128 B (one K-tile), chunk-XOR swizzled on the source address (rule 21).
//   * 4 phases per K-tile: Q(0,0) [reads A0 + B0: 12 ds_read_b128], Q(0,1) [B1: 4], Q(1,1) [A1: 8],
//     Q(1,0) [B0 still in registers]. Phase = load segment (2 LDS-DMA of slot p of the NEXT K-tile, then
//     the fragment reads, then a counted vmcnt) | barrier | 16 MFMA 16x16x32 | barrier.
//   * RAW: a slot is read one phase after the vmcnt that retires it (vmcnt 4/4/6/4 in steady state,
//     2/0 on the last K-tile); WAR: a slot is restaged >= 4 phases after its last read.
//   * waves 4-7 run at s_setprio 1 (the arbitration loser of each pair, MI355X_MICROARCH item 4).
// Measured vs the previous 2-barrier kernel at M = 8192 (Llama-2-7B shapes, random data, one process):
// +4-13 %; the no-stagger control equals the old kernel. Ablations (profiles/r5_gemm_pp/README.md): the
// LDS-DMA + fragment-read traffic through the LDS costs ~25 % each on top of the MFMA/barrier skeleton.
// K % 8 == 0: a partial last K-tile reads zeros (zpage) for the chunks past K; rows beyond M / N are clamped on load
// and masked on store.
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ void pp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

template <bool KTAIL>
__global__ __launch_bounds__(512, 1) void gemm_pp_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                         const bf16_t* __restrict__ B, int64_t ldb,
                                                         const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                         int64_t ldy, int M, int N, int K, int act, int glu,
                                                         int group_m, const char* __restrict__ zpage) {
  constexpr int SLOT = 16384, BUF = 4 * SLOT;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 2, wc = w & 3;
  const int ntn = (N + 255) / 256, ntm = (M + 255) / 256;
  const int GM = group_m;  // XCD-contiguous tile ranges, GM M-tiles per group (as gemm_big)
  const int tile = xcd_remap(blockIdx.x, ntn * ntm);
  const int grp = tile / (GM * ntn), gidx = tile - grp * (GM * ntn);
  const int gm = min(GM, ntm - grp * GM);
  const int m0 = (grp * GM + gidx % gm) * 256, n0 = (gidx / gm) * 256;
  const int nk = (K + 63) / 64;

  // staging: slot h, instruction i (0, 1) = 8 local rows x 128 B, local row lr = (8 i + w) * 8 + lane / 8;
  // LDS chunk lane & 7 holds global chunk (lane & 7) ^ (lr & 7)
  const char* src[4] = {(const char*)A, (const char*)B, (const char*)B, (const char*)A};
  int64_t soff[4][2];
  int lofs[2], kcol[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = i * 8 + w;
    const int lr = inst * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ (lr & 7);
    lofs[i] = inst * 1024;
    kcol[i] = gc * 8;
    const int ar0 = min(m0 + (lr >> 6) * 128 + (lr & 63), M - 1);
    const int ar1 = min(m0 + (lr >> 6) * 128 + 64 + (lr & 63), M - 1);
    const int bc0 = min(n0 + (lr >> 5) * 64 + (lr & 31), N - 1);
    const int bc1 = min(n0 + (lr >> 5) * 64 + 32 + (lr & 31), N - 1);
    soff[0][i] = (int64_t)ar0 * lda * 2 + gc * 16;
    soff[3][i] = (int64_t)ar1 * lda * 2 + gc * 16;
    soff[1][i] = (int64_t)bc0 * ldb * 2 + gc * 16;
    soff[2][i] = (int64_t)bc1 * ldb * 2 + gc * 16;
  }
  auto stage = [&](int t, int h, char* buf) {
    const bool last = KTAIL && t == nk - 1;  // wave-uniform; KTAIL: K % 64 != 0 (Llama-2-7B TP=8 down, K = 1376)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const char* p = src[h] + soff[h][i] + (int64_t)t * 128;
      if (last) p = t * 64 + kcol[i] >= K ? zpage : p;  // chunks past K (of A and B) land as zeros
      __builtin_amdgcn_global_load_lds((const void*)p, (LDS_AS void*)(buf + h * SLOT + lofs[i]), 16, 0, 0);
    }
  };
  // fragment offsets inside a slot: A rows wr*64 + mt*16 + li, B rows wc*32 + nt*16 + li; k-half s -> chunk 4s+g
  // (the conflict-free ds_read_b128 image of gemm_big)
  int aoff[4][2], boff[2][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = 4 * s + g;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
      const int r = wr * 64 + mt * 16 + li;
      aoff[mt][s] = r * 128 + ((c ^ (r & 7)) << 4);
    }
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      const int r = wc * 32 + nt * 16 + li;
      boff[nt][s] = r * 128 + ((c ^ (r & 7)) << 4);
    }
  }
  f32x4 acc[8][4];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 fa[4][2], fb0[2][2], fb1[2][2];
  auto rdA = [&](const char* slot) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[mt][s] = *reinterpret_cast<const s16x8*>(slot + aoff[mt][s]);
  };
  auto rdB = [&](const char* slot, s16x8 (&fb)[2][2]) {
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb[nt][s] = *reinterpret_cast<const s16x8*>(slot + boff[nt][s]);
  };
  auto quad = [&](int mq, int nq, const s16x8 (&fb)[2][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mq * 4 + mt][nq * 2 + nt] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt][s], fb[nt][s], acc[mq * 4 + mt][nq * 2 + nt], 0, 0, 0);
  };
  // one phase: LDS-DMA of slot h of the next K-tile, fragment reads, vmcnt(n) retiring what the next phase
  // reads, barrier, the quadrant's 16 MFMAs, barrier
  auto phase = [&](auto rd, int t, int h, bool more, int n_more, int n_last, int mq, int nq,
                   const s16x8 (&fb)[2][2]) {
    if (more) stage(t + 1, h, smem + ((t + 1) & 1) * BUF);
    rd();
    switch (more ? n_more : n_last) {
      case 0: wait_vmcnt<0>(); break;
      case 2: wait_vmcnt<2>(); break;
      case 4: wait_vmcnt<4>(); break;
      case 6: wait_vmcnt<6>(); break;
      default: break;
    }
    pp_barrier();
    quad(mq, nq, fb);
    pp_barrier();
  };

#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, smem);
  wait_vmcnt<4>();  // slots 0, 1 (A0, B0) of K-tile 0
  pp_barrier();
  if (w >= 4) {
    __builtin_amdgcn_s_setprio(1);
    pp_barrier();  // the stagger: waves 4-7 run one barrier behind waves 0-3
  }
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t & 1) * BUF;
    const bool more = t + 1 < nk;
    phase([&] { rdA(cur); rdB(cur + SLOT, fb0); }, t, 0, more, 4, 2, 0, 0, fb0);
    phase([&] { rdB(cur + 2 * SLOT, fb1); }, t, 1, more, 4, 0, 0, 1, fb1);
    phase([&] { rdA(cur + 3 * SLOT); }, t, 2, more, 6, -1, 1, 1, fb1);
    phase([&] {}, t, 3, more, 4, -1, 1, 0, fb0);
  }
  if (w < 4) pp_barrier();  // balances the stagger barrier
  __builtin_amdgcn_s_setprio(0);
  wait_vmcnt<0>();
  tile_store_lds<256, 256, 8, 4, 512, 2 * BUF>(acc, smem, wr * 128, wc * 64, m0, n0, M, N, nullptr, Y, ldy, bias,
                                               act, glu);
}

// -------------------------------------------------------------------------------------------
// stream-K tiled GEMM (mid-size M: TP-sharded decode at M = 128-512, mid prefill). Split-K grids
// leave CUs unevenly loaded (e.g. 352 blocks on 256 CUs: some CUs run two, the rest one) and pay
// a reduce launch. Here a persistent grid of G workgroups splits the flattened (tile, k-step)
// iteration space into G equal contiguous ranges; the LDS ring of the tiled kernel runs straight
// across tile boundaries. A tile whose k-range spans several workgroups is combined in-kernel:
// every segment stores its fp32 accumulators (register layout, 16 B per lane, coalesced), then
// draws a ticket (agent-scope release fence + relaxed atomic, guide 'splitk-seam' recipe); the
// last arriver acquires, adds the other segments and runs the epilogue. Counters reset themselves.
// -------------------------------------------------------------------------------------------
__device__ __forceinline__ int sk_block_of(int64_t x, int64_t U, int G) {  // block whose range holds unit x
  int g = (int)((x * G) / U);
  while (g + 1 < G && (int64_t)(g + 1) * U / G <= x) ++g;
  while (g > 0 && (int64_t)g * U / G > x) --g;
  return g;
}

template <int MTW, int NTW>
__device__ __forceinline__ void tile_epilogue(const f32x4 (&acc)[MTW][NTW], bf16_t* __restrict__ Y, int64_t ldy,
                                              const bf16_t* __restrict__ bias, int M, int N, int m0, int n0, int wr,
                                              int wc, int li, int g, int act, int glu) {
  const int wn0 = n0 + wc * (NTW * 16);
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * (MTW * 16) + mt * 16 + 4 * g + i;
      if (m >= M) continue;
      if (glu) {
#pragma unroll
        for (int p = 0; p < NTW / 2; ++p) {
          const int ng = wn0 + 2 * p * 16 + li, nu = ng + 16;
          if (nu < N) {
            float gv = acc[mt][2 * p][i], uv = acc[mt][2 * p + 1][i];
            if (bias) { gv += bf2f(bias[ng]); uv += bf2f(bias[nu]); }
            Y[(int64_t)m * ldy + wn0 / 2 + p * 16 + li] = f2bf(silu(gv) * uv);
          }
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int n = wn0 + nt * 16 + li;
          if (n < N) {
            float v = acc[mt][nt][i];
            if (bias) v += bf2f(bias[n]);
            Y[(int64_t)m * ldy + n] = f2bf(apply_act(v, act));
          }
        }
      }
    }
  }
}

template <int BM, int BN, int NS, bool WNT>
__global__ __launch_bounds__(256) void gemm_streamk_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                           const bf16_t* __restrict__ B, int64_t ldb,
                                                           const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                           int64_t ldy, float* __restrict__ part,
                                                           int* __restrict__ counters, int maxseg, int M, int N, int K,
                                                           int act, int glu) {
  constexpr int MTW = BM / 32, NTW = BN / 32;
  constexpr int A_BYTES = BM * TBK * 2, B_BYTES = BN * TBK * 2, STAGE = A_BYTES + B_BYTES;
  constexpr int LOADS = BM / 32 + BN / 32;
  constexpr int TILE_F = BM * BN;  // fp32 per partial tile
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE + 16];  // + ticket broadcast (one LDS object)
  int* s_ticket = reinterpret_cast<int*>(smem + NS * STAGE);
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const int tiles = ntn * ntm, nk = (K + TBK - 1) / TBK;
  const int U = tiles * nk;  // host guarantees < 2^31
  const int G = gridDim.x;
  const int u0 = (int)((int64_t)blockIdx.x * U / G), u1 = (int)((int64_t)(blockIdx.x + 1) * U / G);
  if (u0 >= u1) return;

  // (tile, k-step) of the next unit to stage, advanced incrementally: no divisions in the k-loop
  int pf_t = u0 / nk, pf_k = u0 - (u0 / nk) * nk;
  int pf_m0 = (pf_t / ntn) * BM, pf_n0 = (pf_t % ntn) * BN;
  auto stage_next = [&](char* buf) {
    tiled_stage<BM, BN, WNT>(A, lda, M, B, ldb, N, K, pf_m0, pf_n0, pf_k * TBK, buf, buf + A_BYTES, w, lane);
    if (++pf_k == nk) {
      pf_k = 0;
      ++pf_t;
      pf_m0 = (pf_t / ntn) * BM;
      pf_n0 = (pf_t % ntn) * BN;
    }
  };

  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int a = 0; a < MTW; ++a)
#pragma unroll
    for (int b = 0; b < NTW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (u0 + j < u1) stage_next(smem + j * STAGE);
  int cur = 0;
  int t = u0 / nk, kk = u0 - (u0 / nk) * nk;  // unit being computed
  for (int u = u0; u < u1; ++u) {
    wait_vmcnt_upto<LOADS, NS - 2>(min(u1 - 1 - u, NS));
    lds_barrier();
    char* cA = smem + cur * STAGE;
    if (u + NS - 1 < u1) stage_next(smem + (cur == 0 ? NS - 1 : cur - 1) * STAGE);
    if (kk == nk - 1 && (K % TBK)) tiled_compute<MTW, NTW, true>(cA, cA + A_BYTES, acc, wr, wc, li, g, kk * TBK, K);
    else tiled_compute<MTW, NTW, false>(cA, cA + A_BYTES, acc, wr, wc, li, g, kk * TBK, K);
    cur = cur == NS - 1 ? 0 : cur + 1;

    if (u + 1 != u1 && kk != nk - 1) {  // segment continues
      ++kk;
      continue;
    }
    // ---- segment end: tile t, this workgroup's k-steps up to kk
    const int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;
    const int tu0 = t * nk;
    const bool whole = u0 <= tu0 && kk == nk - 1;
    if (whole) {
      tile_epilogue<MTW, NTW>(acc, Y, ldy, bias, M, N, m0, n0, wr, wc, li, g, act, glu);
    } else {
      const int gfirst = sk_block_of(tu0, U, G), glast = sk_block_of((int64_t)tu0 + nk - 1, U, G);
      const int nseg = glast - gfirst + 1, seg = (int)blockIdx.x - gfirst;
      float* pt = part + (int64_t)t * maxseg * TILE_F;
#pragma unroll
      for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt)
          *reinterpret_cast<f32x4*>(pt + (int64_t)seg * TILE_F + (((w * MTW + mt) * NTW + nt) * 64 + lane) * 4) =
              acc[mt][nt];
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        *s_ticket = __hip_atomic_fetch_add(&counters[t], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (*s_ticket == nseg - 1) {  // last arriver: combine and finish the tile
        if (threadIdx.x == 0) {
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          counters[t] = 0;  // ready for the next launch
        }
        __syncthreads();
        for (int s2 = 0; s2 < nseg; ++s2) {
          if (s2 == seg) continue;
#pragma unroll
          for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
            for (int nt = 0; nt < NTW; ++nt) {
              const f32x4 o = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(
                  pt + (int64_t)s2 * TILE_F + (((w * MTW + mt) * NTW + nt) * 64 + lane) * 4));
#pragma unroll
              for (int i = 0; i < 4; ++i) acc[mt][nt][i] += o[i];
            }
        }
        tile_epilogue<MTW, NTW>(acc, Y, ldy, bias, M, N, m0, n0, wr, wc, li, g, act, glu);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stores / reads above must not count as ring stages
#pragma unroll
    for (int a = 0; a < MTW; ++a)
#pragma unroll
      for (int b = 0; b < NTW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    ++t;
    kk = 0;
  }
}

// -------------------------------------------------------------------------------------------
// W8A8 GEMM on the MX-fp8 matrix cores (BASELINE: Llama-2-70B TP=8 fp8, "CDNA4 fp8 MFMA").
// Y = (Xq . Wq^T) * xs[m] * ws[n] (+ bias, act / SwiGLU): Xq = per-token fp8-e4m3 activations
// (quant_fp8_rows on X), Wq = per-channel fp8-e4m3 weights. The 16x16x128 f8f6f4 MFMA with unit
// block scales (E8M0 127) runs at the fp8 peak (2x bf16; the unscaled 16x16x32 fp8 form runs at
// the bf16 rate). Tiles: BM x BN x 128 bytes staged by glds into the same XOR-swizzled 128-B-row
// LDS image as the bf16 tiles; lane (r = l&15, g = l>>4) takes 32 bytes = k [32g, 32g+32) of its
// row as 2 x ds_read_b128. Used where fp8 GEMMs are compute-bound (prefill, M > 128).
// -------------------------------------------------------------------------------------------
typedef int __attribute__((ext_vector_type(8))) i32x8;
constexpr int TBK8 = 128;  // k (bytes) per stage

template <int BM, int BN>
__device__ __forceinline__ void f8_stage(const unsigned char* __restrict__ A, int64_t lda, int M,
                                         const unsigned char* __restrict__ B, int64_t ldb, int N, int K, int m0, int n0,
                                         int k0, char* sA, char* sB, int w, int lane) {
#pragma unroll
  for (int it = 0; it < BM / 32; ++it) {
    const int inst = it * 4 + w;
    const int row = inst * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (row & 7);
    const int kc = min(k0 + c * 16, K - 16);
    __builtin_amdgcn_global_load_lds((const void*)(A + (int64_t)min(m0 + row, M - 1) * lda + kc),
                                     (LDS_AS void*)(sA + inst * 1024), 16, 0, 0);
  }
#pragma unroll
  for (int it = 0; it < BN / 32; ++it) {
    const int inst = it * 4 + w;
    const int row = inst * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (row & 7);
    const int kc = min(k0 + c * 16, K - 16);
    __builtin_amdgcn_global_load_lds((const void*)(B + (int64_t)min(n0 + row, N - 1) * ldb + kc),
                                     (LDS_AS void*)(sB + inst * 1024), 16, 0, 0);
  }
}

template <int MTW, int NTW, bool MASK>
__device__ __forceinline__ void f8_compute(const char* sA, const char* sB, f32x4 (&acc)[MTW][NTW], int wr, int wc,
                                           int li, int g, int k0, int K) {
  // the lane's k-bytes: chunks g and g + 4 of the 128-byte step (one k permutation for A and B; the chunk
  // pattern of the bf16 reads, free of bank conflicts on the swizzled image)
  const bool v0 = !MASK || (k0 + 16 * g < K), v1 = !MASK || (k0 + 64 + 16 * g < K);
  i32x8 a[MTW], b[NTW];
#pragma unroll
  for (int t = 0; t < MTW; ++t) {
    const int r = wr * (MTW * 16) + t * 16 + li;
    const u32x4 lo = *reinterpret_cast<const u32x4*>(sA + r * 128 + ((g ^ (r & 7)) << 4));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(sA + r * 128 + (((g + 4) ^ (r & 7)) << 4));
    a[t] = i32x8{(int)(v0 ? lo[0] : 0u), (int)(v0 ? lo[1] : 0u), (int)(v0 ? lo[2] : 0u), (int)(v0 ? lo[3] : 0u),
                 (int)(v1 ? hi[0] : 0u), (int)(v1 ? hi[1] : 0u), (int)(v1 ? hi[2] : 0u), (int)(v1 ? hi[3] : 0u)};
  }
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const int r = wc * (NTW * 16) + t * 16 + li;
    const u32x4 lo = *reinterpret_cast<const u32x4*>(sB + r * 128 + ((g ^ (r & 7)) << 4));
    const u32x4 hi = *reinterpret_cast<const u32x4*>(sB + r * 128 + (((g + 4) ^ (r & 7)) << 4));
    b[t] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  }
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt)
#pragma unroll
    for (int nt = 0; nt < NTW; ++nt)
      acc[mt][nt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[mt], b[nt], acc[mt][nt], 0, 0, 0, 127, 0, 127);
}

template <int BM, int BN, int NS>
__global__ __launch_bounds__(256) void gemm_f8f8_kernel(const unsigned char* __restrict__ A, int64_t lda,
                                                        const float* __restrict__ xs,
                                                        const unsigned char* __restrict__ B, int64_t ldb,
                                                        const float* __restrict__ ws,
                                                        const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                        int64_t ldy, float* __restrict__ part, int M, int N, int K,
                                                        int act, int glu) {
  constexpr int MTW = BM / 32, NTW = BN / 32;
  constexpr int A_BYTES = BM * TBK8, B_BYTES = BN * TBK8, STAGE = A_BYTES + B_BYTES;
  constexpr int LOADS = BM / 32 + BN / 32;
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const TileWork tw = tile_work(ntm, ntn, BM, BN);
  const int m0 = tw.m0, n0 = tw.n0, zk = tw.z;
  f32x4 acc[MTW][NTW];
#pragma unroll
  for (int a = 0; a < MTW; ++a)
#pragma unroll
    for (int b = 0; b < NTW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk_all = (K + TBK8 - 1) / TBK8;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int t0 = zk * per, t1 = min(nk_all, t0 + per);
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (t0 + j < t1)
      f8_stage<BM, BN>(A, lda, M, B, ldb, N, K, m0, n0, (t0 + j) * TBK8, smem + j * STAGE, smem + j * STAGE + A_BYTES,
                       w, lane);
  int cur = 0;
  for (int t = t0; t < t1; ++t) {
    wait_vmcnt_upto<LOADS, NS - 2>(t1 - 1 - t);
    lds_barrier();
    char* cA = smem + cur * STAGE;
    if (t + NS - 1 < t1) {
      char* nA = smem + (cur == 0 ? NS - 1 : cur - 1) * STAGE;
      f8_stage<BM, BN>(A, lda, M, B, ldb, N, K, m0, n0, (t + NS - 1) * TBK8, nA, nA + A_BYTES, w, lane);
    }
    if (t + 1 == nk_all && (K % TBK8)) f8_compute<MTW, NTW, true>(cA, cA + A_BYTES, acc, wr, wc, li, g, t * TBK8, K);
    else f8_compute<MTW, NTW, false>(cA, cA + A_BYTES, acc, wr, wc, li, g, t * TBK8, K);
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  // epilogue: per-token x per-channel scales, then the usual bias / act / SwiGLU (or split-K slabs)
  const int wn0 = n0 + wc * (NTW * 16);
#pragma unroll
  for (int mt = 0; mt < MTW; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * (MTW * 16) + mt * 16 + 4 * g + i;
      if (m >= M) continue;
      const float sx = xs[m];
      if (part) {
        float* pr = part + ((int64_t)zk * M + m) * N;
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int n = wn0 + nt * 16 + li;
          if (n < N) pr[n] = acc[mt][nt][i] * sx * ws[n];
        }
      } else if (glu) {
#pragma unroll
        for (int p = 0; p < NTW / 2; ++p) {
          const int ng = wn0 + 2 * p * 16 + li, nu = ng + 16;
          if (nu < N) {
            float gv = acc[mt][2 * p][i] * sx * ws[ng], uv = acc[mt][2 * p + 1][i] * sx * ws[nu];
            if (bias) { gv += bf2f(bias[ng]); uv += bf2f(bias[nu]); }
            Y[(int64_t)m * ldy + wn0 / 2 + p * 16 + li] = f2bf(silu(gv) * uv);
          }
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < NTW; ++nt) {
          const int n = wn0 + nt * 16 + li;
          if (n < N) {
            float v = acc[mt][nt][i] * sx * ws[n];
            if (bias) v += bf2f(bias[n]);
            Y[(int64_t)m * ldy + n] = f2bf(apply_act(v, act));
          }
        }
      }
    }
  }
}

// decode GEMM (csrc/gemm_dec.hip): hint tile bit 1024 (nt_hint bit 18), tile bits = the BN code, depth bits = ring
// depth code (2 / 3 / 4 / 4 stages per wave), split_hint = K split over the grid (fp32 slabs for the consumer)
void launch_gemm_dec(int code, int depth, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw,
                     const bf16_t* bias, bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act, int glu,
                     int split, hipStream_t st, const QkvEpi* qe, int* cnt);
bool gemm_dec_bn(int code, int* bn);
// the decode GEMM's in-launch combine (hint bit 256 with a split) fits the workspace: [tile][split][64 * bn] fp32
static bool dec_combine_fits(int N, int tsel, int s, int64_t ws_bytes) {
  int bn;
  if (!(tsel & 256) || s <= 1 || !gemm_dec_bn(tsel & 15, &bn)) return false;
  return (int64_t)((N + bn - 1) / bn) * s * 64 * bn * 4 <= ws_bytes;
}
static constexpr int kDecHint = 1024;
static int dec_split(int M, int N, int K, int split_hint, int64_t ws_bytes) {
  int s = std::max(1, std::min(split_hint, (K + 63) / 64));
  if ((int64_t)s * M * N * 4 > ws_bytes) s = 1;
  return s;
}
bool gemm_mid_dims(int tsel, int* bm, int* bn, int* threads);
void launch_gemm_mid(int tsel, int depth, bool wnt, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw,
                     const bf16_t* bias, bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act, int glu,
                     int split, hipStream_t st, int* cnt = nullptr,
                     const QkvEpi* qe = nullptr, const float* xs = nullptr, const float* wsc = nullptr,
                     bool ilv = false, const unsigned char* asc = nullptr);

// tile: 1 = 128x128, 2 = 64x128, 3 = 64x64; ring depth 2-4; split-K over grid.y; 8-13: the gemm_mid tiles
// (buffer-descriptor staging, csrc/gemm_mid.hip, fp8 MFMA variant; K % 128 == 0; ilv: its software-pipelined
// k-loop, >= 3 stages)
// MX-fp8 activations (gemm_mid tiles only): asc = e8m0 scales [M][K / 32] of xq (xs unused: nullptr), and mxq / mxs =
// a SwiGLU output written as MX-fp8 instead of bf16 y (e4m3 [M][N / 2] with row stride ldy, scales [M][N / 64]; the
// output tile must hold whole 32-output blocks, BN % 64 == 0, and finish in the launch: no split)
// partial_out: a split plan without activation / GLU leaves its fp32 slabs [split, M, N] (scales applied, no
// bias) in `workspace` for the consumer (rope_cache / add_norm sum them) and returns the split; else 0.
int launch_gemm_f8f8(const void* xq, int64_t ldx, const void* xs, const void* wq, int64_t ldw, const void* wsc,
                     const void* bias, void* y, int64_t ldy, int M, int N, int K, int act, bool glu, int tile,
                     int depth, int split, void* workspace, int64_t ws_bytes, hipStream_t st, bool partial_out,
                     bool ilv, void* mxq, void* mxs, const void* asc) {
  if (M == 0 || N == 0) return 0;
  if (K % 16) throw std::runtime_error("gemm_f8f8: K must be a multiple of 16");
  if (glu && (N % 32)) throw std::runtime_error("gemm_f8f8: glu needs N % 32 == 0");
  if (!y && !partial_out && !mxq) throw std::runtime_error("gemm_f8f8: output required");
  int bm = tile == 1 ? 128 : 64, bn = tile == 3 ? 64 : 128, thr = 256;
  const bool mid = tile >= 7 && tile <= 15;
  if (mid) {
    if (K % 128) throw std::runtime_error("gemm_f8f8: gemm_mid tiles need K % 128 == 0");
    gemm_mid_dims(tile, &bm, &bn, &thr);
  }
  if ((asc || mxq) && !mid) throw std::runtime_error("gemm_f8f8: MX-fp8 activations need a gemm_mid tile (7-15)");
  if (asc && (xs || K % 128)) throw std::runtime_error("gemm_f8f8: MX scales replace xs; K % 128 == 0");
  if (mxq && (!mxs || !glu || bn % 64 || N % 128 || ldy != N / 2 || partial_out))
    throw std::runtime_error("gemm_f8f8: MX output needs SwiGLU, BN % 64 == 0, N % 128 == 0, dense rows, no slabs");
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int nk = (K + TBK8 - 1) / TBK8;
  if (tile == 4 || (tile == 0 && K % 128 == 0 && ((M + 255) / 256) * ((N + 255) / 256) >= 192)) {
    if (K % 128) throw std::runtime_error("gemm_f8f8: the 256x256 tile needs K % 128 == 0");
    gemm_big_kernel<true><<<((M + 255) / 256) * ((N + 255) / 256), 512, 0, st>>>(
        xq, ldx, wq, ldw, (const bf16_t*)bias, (bf16_t*)y, ldy, M, N, K, act, glu ? 1 : 0, (const float*)xs,
        (const float*)wsc, g_big_group_m);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if (tile == 0) {  // auto: 128x128 when it fills the chip, else 64x128 / 64x64, split to >= ~256 WGs
    tile = ((M + 127) / 128) * ((N + 127) / 128) >= 240 ? 1 : (((M + 63) / 64) * ((N + 127) / 128) >= 240 ? 2 : 3);
    return launch_gemm_f8f8(xq, ldx, xs, wq, ldw, wsc, bias, y, ldy, M, N, K, act, glu, tile, depth, split, workspace,
                            ws_bytes, st, partial_out, ilv, mxq, mxs, asc);
  }
  if (split <= 0) {
    split = 1;
    while (tiles * split * 2 <= 512 && nk / (2 * split) >= 4 && split < 8) split *= 2;
  }
  split = std::max(1, std::min(split, nk));
  if ((int64_t)split * M * N * 4 > ws_bytes) split = 1;
  if (mxq && split > 1) throw std::runtime_error("gemm_f8f8: an MX-fp8 SwiGLU output cannot be split over K");
  float* part = split > 1 ? (float*)workspace : nullptr;
  const int act_k = split > 1 ? 0 : act, g = glu ? 1 : 0, glu_k = split > 1 ? 0 : g;
  if (depth <= 0) depth = tile == 1 ? 3 : 4;
  if (tile == 1 && depth > 3) depth = 3;
  dim3 grid(tiles, split);
  auto A = (const unsigned char*)xq;
  auto Bw = (const unsigned char*)wq;
  auto XS = (const float*)xs;
  auto WSc = (const float*)wsc;
  auto Bi = (const bf16_t*)bias;
  auto Y = (bf16_t*)y;
#define LF(BM_, BN_, NS_) \
  gemm_f8f8_kernel<BM_, BN_, NS_><<<grid, 256, 0, st>>>(A, ldx, XS, Bw, ldw, WSc, Bi, Y, ldy, part, M, N, K, act_k, glu_k)
  if (mid) {
    QkvEpi mx{};
    mx.mxq = (unsigned char*)mxq;
    mx.mxs = (unsigned char*)mxs;
    launch_gemm_mid(tile, depth, M <= bm, (const bf16_t*)xq, ldx, (const bf16_t*)wq, ldw, Bi, Y, ldy, part, M, N, K,
                    act_k, glu_k, split, st, nullptr, mxq ? &mx : nullptr, XS, WSc, ilv,
                    (const unsigned char*)asc);
  } else if (tile == 1) {
    if (depth >= 3) LF(128, 128, 3); else LF(128, 128, 2);
  } else if (tile == 2) {
    if (depth >= 4) LF(64, 128, 4); else if (depth == 3) LF(64, 128, 3); else LF(64, 128, 2);
  } else {
    if (depth >= 4) LF(64, 64, 4); else if (depth == 3) LF(64, 64, 3); else LF(64, 64, 2);
  }
#undef LF
  HIP_CHECK_LAUNCH();
  if (split > 1 && partial_out && !glu && act == 0) return split;
  if (split > 1) {
    if (!y) throw std::runtime_error("gemm_f8f8: output required");
    const int nout = glu ? N / 2 : N;
    dim3 rgrid(std::min((nout + 255) / 256, 64), M);
    splitk_reduce_kernel<<<rgrid, 256, 0, st>>>(part, split, M, N, Bi, Y, ldy, act, g);
    HIP_CHECK_LAUNCH();
  }
  return 0;
}

// the split a W8A8 call with these arguments leaves as slabs under partial_out (0 = finished output)
int gemm_f8f8_partial_slabs(int M, int N, int K, bool glu, int act, int tile, int split, int64_t ws_bytes) {
  if (M == 0 || N == 0 || glu || act != 0) return 0;
  if (tile == 4 || (tile == 0 && K % 128 == 0 && ((M + 255) / 256) * ((N + 255) / 256) >= 192)) return 0;
  if (tile == 0)
    tile = ((M + 127) / 128) * ((N + 127) / 128) >= 240 ? 1 : (((M + 63) / 64) * ((N + 127) / 128) >= 240 ? 2 : 3);
  int bm = tile == 1 ? 128 : 64, bn = tile == 3 ? 64 : 128, thr;
  if (tile >= 7 && tile <= 15) gemm_mid_dims(tile, &bm, &bn, &thr);
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const int nk = (K + TBK8 - 1) / TBK8;
  if (split <= 0) {
    split = 1;
    while (tiles * split * 2 <= 512 && nk / (2 * split) >= 4 && split < 8) split *= 2;
  }
  split = std::max(1, std::min(split, nk));
  if ((int64_t)split * M * N * 4 > ws_bytes) split = 1;
  return split > 1 ? split : 0;
}

// -------------------------------------------------------------------------------------------
// host dispatch
// -------------------------------------------------------------------------------------------
template <int MT, int NT, int KC, bool FP8W, int VARIANT>
static void launch_stream_t(const bf16_t* X, int64_t ldx, const void* W, int64_t ldw, const float* ws, const bf16_t* bias,
                            bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act, int glu, int splitk,
                            hipStream_t st) {
  dim3 grid((N + 64 * NT - 1) / (64 * NT), splitk);
  if constexpr (VARIANT == 2)
    gemm_stream2_kernel<MT, NT, KC, FP8W><<<grid, 256, 0, st>>>(X, ldx, W, ldw, ws, bias, Y, ldy, part, M, N, K, act, glu);
  else
    gemm_stream_kernel<MT, NT, KC, FP8W><<<grid, 256, 0, st>>>(X, ldx, W, ldw, ws, bias, Y, ldy, part, M, N, K, act, glu);
  HIP_CHECK_LAUNCH();
}

template <bool FP8W>
static void launch_stream(int variant, int mt, int nt, const bf16_t* X, int64_t ldx, const void* W, int64_t ldw,
                          const float* ws, const bf16_t* bias, bf16_t* Y, int64_t ldy, float* part, int M, int N, int K,
                          int act, int glu, int splitk, hipStream_t st) {
  if (variant == 2) {  // v2 instantiations (3-deep W ring): NT <= 2, spill-free at 2 waves/SIMD
#define LS2(MT_, NT_, KC_) \
  launch_stream_t<MT_, NT_, KC_, FP8W, 2>(X, ldx, W, ldw, ws, bias, Y, ldy, part, M, N, K, act, glu, splitk, st)
    if (nt >= 2) {
      if (mt == 1) LS2(1, 2, 128); else if (mt == 2) LS2(2, 2, 128); else if (mt <= 4) LS2(4, 2, 128); else LS2(8, 2, 64);
    } else {
      if (mt == 1) LS2(1, 1, 256); else if (mt == 2) LS2(2, 1, 128); else if (mt <= 4) LS2(4, 1, 128); else LS2(8, 1, 128);
    }
#undef LS2
    return;
  }
#define LS(MT_, NT_, KC_) \
  launch_stream_t<MT_, NT_, KC_, FP8W, 1>(X, ldx, W, ldw, ws, bias, Y, ldy, part, M, N, K, act, glu, splitk, st)
  // only register-feasible (spill-free at 2 waves/SIMD) instantiations
  if constexpr (FP8W) {
    if (nt >= 2) {
      if (mt == 1) LS(1, 2, 256); else if (mt == 2) LS(2, 2, 128); else if (mt <= 4) LS(4, 2, 128); else LS(8, 2, 64);
    } else {
      if (mt == 1) LS(1, 1, 256); else if (mt == 2) LS(2, 1, 256); else if (mt <= 4) LS(4, 1, 256); else LS(8, 1, 128);
    }
  } else {
    if (nt >= 4 && mt <= 2) {
      if (mt == 1) LS(1, 4, 128); else LS(2, 4, 128);
    } else if (nt >= 2) {
      if (mt == 1) LS(1, 2, 256); else if (mt == 2) LS(2, 2, 256); else if (mt <= 4) LS(4, 2, 256); else LS(8, 2, 64);
    } else {
      if (mt == 1) LS(1, 1, 256); else if (mt == 2) LS(2, 1, 256); else if (mt <= 4) LS(4, 1, 256); else LS(8, 1, 128);
    }
  }
#undef LS
}

// Tile/split choice for the streaming kernel: columns per workgroup and K splits such that the
// grid reaches ~2 workgroups per CU (256 CUs) without splitting K below 4 chunks per slice.
void gemm_stream_plan(int M, int N, int K, int* nt_out, int* splitk_out) {
  int nt = (N >= 16384) ? 2 : 1;
  const int nblk = (N + 64 * nt - 1) / (64 * nt);
  const int kc = M > 64 ? 128 : 256;
  const int nck = (K + kc - 1) / kc;
  // measured (bench/gemm_bench.py --sweep, Llama-2-7B shapes): M <= 16 likes ~3 workgroups per
  // CU, larger M ~1 per CU (its X tile already costs LDS); N alone filling the chip -> no split
  const int target = nblk >= 256 ? nblk : (M <= 16 ? 768 : 256);
  int s = 1;
  while (nblk * s < target && s < 16 && nck / (2 * s) >= 4) s *= 2;
  *nt_out = nt;
  *splitk_out = s;
}

int gemm_skinny_splitk(int M, int N, int K) {
  int nt, s;
  gemm_stream_plan(M, N, K, &nt, &s);
  return s;
}

int launch_tiled(const bf16_t* X, int64_t ldx, const void* W, int64_t ldw, const bf16_t* B, bf16_t* Y, int64_t ldy,
                 int M, int N, int K, int act, int g, int tsel, int split_hint, void* workspace, int64_t ws_bytes,
                 bool partial_out, hipStream_t st, const float* wscale = nullptr, const QkvEpi* qe = nullptr);

int gemm_partial_slabs(int M, int N, int K, bool w_fp8, bool glu, int act, int nt_hint, int split_hint,
                       int64_t ws_bytes);
void gemm_tiled_plan(int M, int N, int K, int* tsel_io, int* split_io, bool glu);
void gemm_stream_plan(int M, int N, int K, int* nt_out, int* splitk_out);

// Returns the number of fp32 partial slabs [S, M, N] left in `workspace` (partial_out and the
// planner chose split-K: the consumer - add_norm - reduces them and adds `bias`), or 0 when Y
// holds the finished bf16 output.
// Autotuned plans: (M, N, K, glu, fp8) -> (nt_hint, split) measured by llmss_amd/ops/autotune.py
// for the shapes an engine will actually run (decode batch buckets x layer GEMMs). Consulted by
// every call without explicit hints and by gemm_plan, so split-K partial fusion stays consistent.
namespace {
std::mutex g_tuned_mu;
std::unordered_map<uint64_t, std::pair<int, int>> g_tuned;
// kind: 0 = bf16 [N, K] weights, 1 = fp8 weights, 3 = QKV
// RoPE / KV-write epilogue (launch_gemm_qkv)
uint64_t tune_key(int M, int N, int K, bool glu, int kind) {
  return ((uint64_t)(kind & 7) << 61) | ((uint64_t)(M & 0x7FFFF) << 42) | ((uint64_t)N << 22) |
         ((uint64_t)K << 2) | (glu ? 2u : 0u) | (kind == 1 ? 1u : 0u);
}
}  // namespace

void gemm_tuned_set(int M, int N, int K, bool glu, int kind, int nt_hint, int split) {
  std::lock_guard<std::mutex> lk(g_tuned_mu);
  g_tuned[tune_key(M, N, K, glu, kind)] = {nt_hint, split};
}
void gemm_tuned_clear() {
  std::lock_guard<std::mutex> lk(g_tuned_mu);
  g_tuned.clear();
}
bool gemm_tuned_get(int M, int N, int K, bool glu, int kind, int* nt_hint, int* split) {
  std::lock_guard<std::mutex> lk(g_tuned_mu);
  auto it = g_tuned.find(tune_key(M, N, K, glu, kind));
  if (it == g_tuned.end()) return false;
  *nt_hint = it->second.first;
  *split = it->second.second;
  return true;
}

int launch_gemm(const void* x, int64_t ldx, const void* w, int64_t ldw, bool w_fp8, const void* w_scale,
                const void* bias, void* y, int64_t ldy, int M, int N, int K, int act, bool glu, void* workspace,
                int64_t ws_bytes, int nt_hint, int split_hint, bool partial_out, hipStream_t st) {
  if (M == 0 || N == 0) return 0;
  if (nt_hint == 0 && split_hint == 0) gemm_tuned_get(M, N, K, glu, w_fp8 ? 1 : 0, &nt_hint, &split_hint);
  if (!y && (!partial_out || gemm_partial_slabs(M, N, K, w_fp8, glu, act, nt_hint, split_hint, ws_bytes) == 0))
    throw std::runtime_error("gemm: this configuration writes the output, but no output buffer was given");
  if (K % 16) throw std::runtime_error("gemm: K must be a multiple of 16");
  if (glu && (N % 32)) throw std::runtime_error("gemm: glu needs N % 32 == 0");
  auto X = (const bf16_t*)x;
  auto B = (const bf16_t*)bias;
  auto Y = (bf16_t*)y;
  auto WS = (const float*)w_scale;
  const int g = glu ? 1 : 0;
  // weight-streaming kernel: M <= 16, explicit stream hints, and fp8 prefill panels; fp8 decode
  // (16 < M <= 128) runs the tiled kernel with fp8 weight tiles (W8A16)
  const int tiled_hint = nt_hint >> 8;
  const bool stream = (nt_hint & 0xff) || (!tiled_hint && (M <= 16 || (w_fp8 && M > 128)));
  if (stream) {
    if (M > 128) {  // fp8 weights with many rows (prefill): 128-row panels through the streaming kernel
      for (int m0 = 0; m0 < M; m0 += 128) {
        const int mm = std::min(128, M - m0);
        launch_gemm((const bf16_t*)x + m0 * ldx, ldx, w, ldw, w_fp8, w_scale, bias, (bf16_t*)y + m0 * ldy, ldy, mm, N,
                    K, act, glu, workspace, ws_bytes, nt_hint, split_hint, false, st);
      }
      return 0;
    }
    int nt, splitk;
    gemm_stream_plan(M, N, K, &nt, &splitk);
    // nt_hint = nt + 16 * variant (variant 1: LDS-DMA X staging, 2: register-staged X + W ring)
    int variant = ((nt_hint >> 4) & 15) ? ((nt_hint >> 4) & 15) : 2;
    nt_hint &= 15;
    if (nt_hint > 0) nt = nt_hint;
    if (split_hint > 0) splitk = split_hint;
    if (glu && nt < 2) nt = 2;  // the SwiGLU epilogue pairs (gate, up) 16-column tiles inside a wave
    if ((int64_t)splitk * M * N * 4 > ws_bytes) splitk = 1;
    float* part = splitk > 1 ? (float*)workspace : nullptr;
    const int mt = (M + 15) / 16;
    const int act_k = splitk > 1 ? 0 : act, glu_k = splitk > 1 ? 0 : g;
    if (w_fp8) launch_stream<true>(variant, mt, nt, X, ldx, w, ldw, WS, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
    else launch_stream<false>(variant, mt, nt, X, ldx, w, ldw, nullptr, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
    if (splitk > 1 && partial_out && !glu && act == 0) return splitk;
    if (splitk > 1) {
      const int nout = glu ? N / 2 : N;
      dim3 grid(std::min((nout + 255) / 256, 64), M);
      splitk_reduce_kernel<<<grid, 256, 0, st>>>(part, splitk, M, N, B, Y, ldy, act, g);
      HIP_CHECK_LAUNCH();
    }
    return 0;
  }
  return launch_tiled(X, ldx, w, ldw, B, Y, ldy, M, N, K, act, g, nt_hint >> 8, split_hint, workspace,
                      ws_bytes, partial_out, st, w_fp8 ? WS : nullptr);
}

// Tiled-path plan. Tile: 64 rows for M <= 64 (64x64, or 64x128 when 64x64 gives > 256 tiles),
// else 128x128. K is split until the grid holds ~3 (64-row tiles) or ~1.5 (128x128) workgroups
// per CU, keeping >= 512 k per slice. Measured on the Llama-2-7B shapes at M = 64..512
// (bench/gemm_bench.py --sweep): within ~5% of the best (tile, split) of the sweep everywhere.
static int tiles_of(int M, int N, int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); }
// tsel: 1 = 128x128, 2 = 64x128, 3 = 64x64 (4 waves); 5 = 256x128, 6 = 256x64 (8 waves, 1 WG/CU);
// 4 = the big-tile kernel
bool gemm_mid_dims(int tsel, int* bm, int* bn, int* threads);

// tsel 8-12: gemm_mid (gemm_mid.hip: buffer-descriptor staging, 128x128 / 256x128 / 64x256 / 64x128 / 128x256)
static int tile_dims(int tsel, int* bm, int* bn) {
  int thr;
  if (gemm_mid_dims(tsel, bm, bn, &thr)) return 0;
  *bm = tsel >= 5 ? 256 : (tsel == 1 ? 128 : 64);
  *bn = (tsel == 3 || tsel == 6) ? 64 : 128;
  return 0;
}
void gemm_tiled_plan(int M, int N, int K, int* tsel_io, int* split_io, bool glu) {
  int tsel = *tsel_io;
  // SwiGLU output cannot be folded into the next kernel, so a split would cost its own reduce
  // launch: with >= 256 64x64 tiles, no split (measured equal or better at M <= 128)
  if (tsel == 0 && glu && M <= 128 && tiles_of(M, N, 64, 64) >= 256 && *split_io <= 0) {
    *tsel_io = 3 | 16;
    *split_io = 1;
    return;
  }
  if (tsel == 0) {
    if (tiles_of(M, N, 256, 256) >= 192) tsel = 4;
    else tsel = M <= 64 ? (tiles_of(M, N, 64, 64) > 256 ? 2 : 3) : 1;
  }
  int hint_bits = tsel & ~15;
  tsel &= 15;
  if (tsel >= 5) hint_bits &= ~128;  // no stream-K variant of the 8-wave tiles
  if (hint_bits & 128) {  // stream-K: output is final (no slabs); split_io carries workgroups per CU
    *tsel_io = tsel | hint_bits;
    if (*split_io <= 0) *split_io = 2;
    return;
  }
  if (tsel == 4) {  // big-tile kernel: no split-K, no stage option
    *tsel_io = 4;
    *split_io = 1;
    return;
  }
  int bm, bn;
  tile_dims(tsel, &bm, &bn);
  const int nt = tiles_of(M, N, bm, bn);
  int s = *split_io;
  if (s <= 0) {
    const int bound = bm == 64 ? 800 : (bm == 128 ? 537 : 300);
    s = 1;
    while (nt * s * 2 <= bound && s < 8 && K / (2 * s) >= 512) s *= 2;
  }
  s = std::max(1, std::min(s, (K + TBK - 1) / TBK));
  // 3-stage LDS ring when the grid is too small for block-level latency hiding (measured: o/down
  // projections and the LM head at M <= 128 gain 10-20%; wide grids lose occupancy to its LDS)
  if (*tsel_io == 0 && nt * s <= (bm == 64 ? 600 : 256)) tsel |= 16;
  *tsel_io = tsel | hint_bits;
  *split_io = s;
}

static bool wnt_ok(int tsel_raw, int M, int tsel) {
  int bm, bn;
  tile_dims(tsel & 15, &bm, &bn);
  return !(tsel_raw & 64) && M <= bm;
}

// per-tile arrival counters of the stream-K and split-K combines, one buffer per device: zeroed
// once, reset by every last arriver (consecutive GEMMs on one stream never overlap)
static std::mutex g_sk_mu;
static int* g_sk_counters[64] = {};
static int g_sk_capacity[64] = {};

// workspace slot (gemm_set_slot): GEMM chains that may run concurrently on different streams (the two
// half-batch decode chains, models/decoder.py) use disjoint counter ranges, as they use disjoint workspaces
static constexpr int kSlots = 4;
static thread_local int g_ws_slot = 0;
void gemm_set_slot(int s) { g_ws_slot = s & (kSlots - 1); }

static int* sk_counters(int n) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) throw std::runtime_error("gemm counters: bad device");
  std::lock_guard<std::mutex> lk(g_sk_mu);
  if (n <= g_sk_capacity[dev]) return g_sk_counters[dev] + (size_t)g_ws_slot * g_sk_capacity[dev];
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(nullptr, &cs);
  if (cs != hipStreamCaptureStatusNone) throw std::runtime_error("gemm counters must be allocated before capture");
  int cap = std::max(n, 1 << 16);
  int* p = nullptr;
  const size_t bytes = (size_t)cap * kSlots * sizeof(int);
  if (hipMalloc(&p, bytes) != hipSuccess) throw std::runtime_error("gemm counters: hipMalloc");
  if (hipMemset(p, 0, bytes) != hipSuccess) throw std::runtime_error("gemm counters: memset");
  (void)hipDeviceSynchronize();
  g_sk_counters[dev] = p;  // the old (smaller) buffer is left to the process: launches may still reference it
  g_sk_capacity[dev] = cap;
  return p + (size_t)g_ws_slot * cap;
}

// 4 KiB of zeros per device: the source of the chunks past K in gemm_pp's partial last K-tile
static const char* g_zero_page[64] = {};
static const char* zero_page() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) throw std::runtime_error("gemm zero page: bad device");
  std::lock_guard<std::mutex> lk(g_sk_mu);
  if (g_zero_page[dev]) return g_zero_page[dev];
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(nullptr, &cs);
  if (cs != hipStreamCaptureStatusNone) throw std::runtime_error("gemm zero page must be allocated before capture");
  char* p = nullptr;
  if (hipMalloc(&p, 4096) != hipSuccess) throw std::runtime_error("gemm zero page: hipMalloc");
  if (hipMemset(p, 0, 4096) != hipSuccess) throw std::runtime_error("gemm zero page: memset");
  (void)hipDeviceSynchronize();
  g_zero_page[dev] = p;
  return p;
}

void gemm_reserve_streamk(int n) {
  sk_counters(n);
  (void)zero_page();
}

static bool launch_streamk(const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, const bf16_t* B, bf16_t* Y,
                           int64_t ldy, int M, int N, int K, int act, int g, int tsel, int ns, int per_cu,
                           void* workspace, int64_t ws_bytes, bool wnt, hipStream_t st) {
  int bm, bn;
  tile_dims(tsel, &bm, &bn);
  if (tsel == 1 && ns > 3) ns = 3;
  if (tsel == 2 && ns > 4) ns = 4;
  if (ns == 6) ns = 4;
  const int tiles = tiles_of(M, N, bm, bn), nk = (K + TBK - 1) / TBK;
  const int64_t U = (int64_t)tiles * nk;
  if (U >= (1LL << 31)) return false;
  const int G = (int)std::min<int64_t>(U, 256LL * std::max(1, std::min(per_cu, 8)));
  const int64_t per = U / G;  // >= 1
  const int maxseg = (int)std::min<int64_t>(G, (nk + per - 1) / per + 1);
  if ((int64_t)tiles * maxseg * bm * bn * 4 > ws_bytes) return false;
  int* cnt = sk_counters(tiles);
  float* part = (float*)workspace;
#define SK(BM_, BN_, NS_)                                                                                          \
  do {                                                                                                             \
    if (wnt)                                                                                                       \
      gemm_streamk_kernel<BM_, BN_, NS_, true><<<G, 256, 0, st>>>(X, ldx, W, ldw, B, Y, ldy, part, cnt, maxseg, M, N, \
                                                                   K, act, g);                                     \
    else                                                                                                           \
      gemm_streamk_kernel<BM_, BN_, NS_, false><<<G, 256, 0, st>>>(X, ldx, W, ldw, B, Y, ldy, part, cnt, maxseg, M, \
                                                                    N, K, act, g);                                 \
  } while (0)
  if (tsel == 1) {
    if (ns == 3) SK(128, 128, 3); else SK(128, 128, 2);
  } else if (tsel == 2) {
    if (ns == 4) SK(64, 128, 4); else if (ns == 3) SK(64, 128, 3); else SK(64, 128, 2);
  } else {
    if (ns == 4) SK(64, 64, 4); else if (ns == 3) SK(64, 64, 3); else SK(64, 64, 2);
  }
#undef SK
  HIP_CHECK_LAUNCH();
  return true;
}

int launch_tiled(const bf16_t* X, int64_t ldx, const void* W, int64_t ldw, const bf16_t* B, bf16_t* Y, int64_t ldy,
                 int M, int N, int K, int act, int g, int tsel, int split_hint, void* workspace, int64_t ws_bytes,
                 bool partial_out, hipStream_t st, const float* wscale, const QkvEpi* qe) {
  const QkvEpi qv = qe ? *qe : QkvEpi{};
  const int tsel_raw = tsel;
  int s = split_hint;
  const bool f8 = wscale != nullptr;  // fp8-e4m3 weights (W8A16): half the weight bytes of a decode step
  if (tsel & kDecHint) {  // K split over the waves (gemm_dec.hip), M <= 64, bf16 weights
    if (f8) throw std::runtime_error("gemm_dec: bf16 weights only");
    s = dec_split(M, N, K, split_hint, ws_bytes);
    if (s > 1 && Y && dec_combine_fits(N, tsel, s, ws_bytes)) {  // split-K combined in the launch: finished Y
      int bn;
      gemm_dec_bn(tsel & 15, &bn);
      static constexpr int kDecDepthC[4] = {2, 3, 4, 4};
      launch_gemm_dec(tsel & 15, kDecDepthC[(tsel >> 4) & 3], X, ldx, (const bf16_t*)W, ldw, B, Y, ldy,
                      (float*)workspace, M, N, K, act, g, s, st, qe, sk_counters((N + bn - 1) / bn));
      return 0;
    }
    if (qe && s > 1) throw std::runtime_error("gemm_dec: the QKV epilogue needs an unsplit or in-launch-combined plan");
    static constexpr int kDecDepth[4] = {2, 3, 4, 4};
    float* part = s > 1 ? (float*)workspace : nullptr;
    launch_gemm_dec(tsel & 15, kDecDepth[(tsel >> 4) & 3], X, ldx, (const bf16_t*)W, ldw, B, Y, ldy, part, M, N, K,
                    s > 1 ? 0 : act, s > 1 ? 0 : g, s, st, qe, nullptr);
    if (s > 1 && partial_out && !g && act == 0) return s;
    if (s > 1) {
      const int nout = g ? N / 2 : N;
      dim3 rgrid(std::min((nout + 255) / 256, 64), M);
      splitk_reduce_kernel<<<rgrid, 256, 0, st>>>(part, s, M, N, B, Y, ldy, act, g);
      HIP_CHECK_LAUNCH();
    }
    return 0;
  }
  if (f8 && (tsel & 15) >= 5) tsel = (tsel & ~15) | 1;  // 8-wave and mid tiles are bf16-only
  gemm_tiled_plan(M, N, K, &tsel, &s, g != 0);
  static constexpr int kDepth[4] = {2, 3, 4, 6};
  int ns = kDepth[(tsel >> 4) & 3];  // LDS ring depth (hint bits 4-5); bit 6: default-policy weights
  tsel &= 15;
  // the ping-pong kernel's zero-page K tail works on 8-element chunks and its LDS-DMA rows need 16-B aligned
  // strides: anything else runs on the 128x128 tile (tuned hints and C++ callers included, not just linear())
  if (tsel == 4 && (K % 8 || ldx % 8 || ldw % 8)) tsel = 1;
  if ((tsel == 1 || tsel == 5) && ns > 3) ns = 3;  // 128x128 / 256x128 x 4 stages exceed the 160 KiB LDS
  if ((tsel == 2 || tsel == 6) && ns > 4) ns = 4;
  if (f8 && tsel == 4) tsel = 1;
  if (tsel == 4) {
    if (K & 63)
      gemm_pp_kernel<true><<<tiles_of(M, N, 256, 256), 512, 0, st>>>(X, ldx, (const bf16_t*)W, ldw, B, Y, ldy, M, N, K,
                                                                     act, g, g_big_group_m, zero_page());
    else
      gemm_pp_kernel<false><<<tiles_of(M, N, 256, 256), 512, 0, st>>>(X, ldx, (const bf16_t*)W, ldw, B, Y, ldy, M, N, K,
                                                                      act, g, g_big_group_m, nullptr);
    HIP_CHECK_LAUNCH();
    return 0;
  }
  if ((tsel_raw & 128) && !f8 && tsel < 5) {
    if (launch_streamk(X, ldx, (const bf16_t*)W, ldw, B, Y, ldy, M, N, K, act, g, tsel, ns, s, workspace, ws_bytes,
                       wnt_ok(tsel_raw, M, tsel), st))
      return 0;
    s = 1;  // workspace too small for the partial tiles: plain tiled launch
  }
  int bm, bn;
  tile_dims(tsel, &bm, &bn);
  const int nt = tiles_of(M, N, bm, bn);
  // hint bit 8: split-K slices combine in-launch (last arriver per tile, common.h splitk_combine):
  // slabs [tile][S][bm*bn] in the workspace, finished bf16 output, no reduce launch
  int* cnt = nullptr;
  if ((tsel_raw & 256) && s > 1 && (int64_t)nt * s * bm * bn * 4 <= ws_bytes && Y) cnt = sk_counters(nt);
  if (!cnt && (int64_t)s * M * N * 4 > ws_bytes) s = 1;
  if (qe && (s > 1 && !cnt)) throw std::runtime_error("gemm: the QKV epilogue needs an unsplit or in-launch-combined plan");
  float* part = s > 1 ? (float*)workspace : nullptr;
  const int act_k = s > 1 && !cnt ? 0 : act, glu_k = s > 1 && !cnt ? 0 : g;
  dim3 grid(nt, s);
  if (tsel >= 7 && tsel <= 15) {  // gemm_mid tiles (7, 8-15)
    launch_gemm_mid(tsel, ns, wnt_ok(tsel_raw, M, tsel), X, ldx, (const bf16_t*)W, ldw, B, Y, ldy, part, M, N, K,
                    act_k, glu_k, s, st, cnt, qe, nullptr, nullptr, (tsel_raw & 512) != 0);
    if (cnt) return 0;
    if (s > 1 && partial_out && !g && act == 0) return s;
    if (s > 1) {
      const int nout = g ? N / 2 : N;
      dim3 rgrid(std::min((nout + 255) / 256, 64), M);
      splitk_reduce_kernel<<<rgrid, 256, 0, st>>>(part, s, M, N, B, Y, ldy, act, g);
      HIP_CHECK_LAUNCH();
    }
    return 0;
  }
  // non-temporal weight staging when every weight tile is read by exactly one workgroup row
  const bool wnt = wnt_ok(tsel_raw, M, tsel);
  if (tsel >= 5) {  // 8-wave tiles (bf16 weights)
#define LT8(BM_, BN_, NS_)                                                                                          \
  do {                                                                                                             \
    if (wnt)                                                                                                       \
      gemm_tiled_kernel<BM_, BN_, NS_, true, false, 8><<<grid, 512, 0, st>>>(X, ldx, W, ldw, B, Y, ldy, part, M, N, K, \
                                                                             act_k, glu_k, nullptr, cnt, qv);      \
    else                                                                                                           \
      gemm_tiled_kernel<BM_, BN_, NS_, false, false, 8><<<grid, 512, 0, st>>>(X, ldx, W, ldw, B, Y, ldy, part, M, N,  \
                                                                              K, act_k, glu_k, nullptr, cnt, qv);  \
  } while (0)
    if (tsel == 5) {
      if (ns == 3) LT8(256, 128, 3); else LT8(256, 128, 2);
    } else {
      if (ns == 4) LT8(256, 64, 4); else if (ns == 3) LT8(256, 64, 3); else LT8(256, 64, 2);
    }
#undef LT8
  } else {
#define LT1(BM_, BN_, NS_, WNT_, F8_)                                                                              \
  gemm_tiled_kernel<BM_, BN_, NS_, WNT_, F8_><<<grid, 256, 0, st>>>(X, ldx, W, ldw, B, Y, ldy, part, M, N, K, act_k,  \
                                                                    glu_k, wscale, cnt, qv)
#define LT(BM_, BN_, NS_)                                                                                          \
  do {                                                                                                             \
    if (f8) {                                                                                                      \
      if (wnt) LT1(BM_, BN_, NS_, true, true); else LT1(BM_, BN_, NS_, false, true);                              \
    } else {                                                                                                       \
      if (wnt) LT1(BM_, BN_, NS_, true, false); else LT1(BM_, BN_, NS_, false, false);                            \
    }                                                                                                              \
  } while (0)
  if (ns == 3) {
    if (tsel == 1) LT(128, 128, 3); else if (tsel == 2) LT(64, 128, 3); else LT(64, 64, 3);
  } else if (ns == 4) {
    if (tsel == 2) LT(64, 128, 4); else LT(64, 64, 4);
  } else if (ns == 6) {
    LT(64, 64, 6);
  } else {
    if (tsel == 1) LT(128, 128, 2); else if (tsel == 2) LT(64, 128, 2); else LT(64, 64, 2);
  }
  }
#undef LT
#undef LT1
  HIP_CHECK_LAUNCH();
  if (cnt) return 0;
  if (s > 1 && partial_out && !g && act == 0) return s;
  if (s > 1) {
    const int nout = g ? N / 2 : N;
    dim3 rgrid(std::min((nout + 255) / 256, 64), M);
    splitk_reduce_kernel<<<rgrid, 256, 0, st>>>(part, s, M, N, B, Y, ldy, act, g);
    HIP_CHECK_LAUNCH();
  }
  return 0;
}

// Number of fp32 partial slabs launch_gemm(..., partial_out=true) leaves for these hints, or 0 if
// that call writes the finished output (stream-K, fp8 prefill panels, act / glu epilogues, no
// split). The Python wrapper allocates Y exactly when this returns 0 - one source of truth.
int gemm_partial_slabs(int M, int N, int K, bool w_fp8, bool glu, int act, int nt_hint, int split_hint,
                       int64_t ws_bytes) {
  if (M == 0 || N == 0 || glu || act != 0) return 0;
  if (nt_hint == 0 && split_hint == 0) gemm_tuned_get(M, N, K, glu, w_fp8 ? 1 : 0, &nt_hint, &split_hint);
  const int tiled_hint = nt_hint >> 8;
  const bool stream = (nt_hint & 0xff) || (!tiled_hint && (M <= 16 || (w_fp8 && M > 128)));
  int s;
  if (stream) {
    if (M > 128) return 0;  // 128-row panels, each finished in place
    int nt;
    gemm_stream_plan(M, N, K, &nt, &s);
    if (split_hint > 0) s = split_hint;
  } else {
    int tsel = tiled_hint;
    if (tsel & kDecHint) {
      if (w_fp8) return 0;  // rejected at launch
      s = dec_split(M, N, K, split_hint, ws_bytes);
      if (dec_combine_fits(N, tsel, s, ws_bytes)) return 0;  // combined in the launch
      return s > 1 ? s : 0;
    }
    if ((tsel & 128) && !w_fp8 && (tsel & 15) < 5) return 0;  // stream-K combines in-kernel
    if (w_fp8 && ((tsel & 15) == 4 || (tsel & 15) >= 5)) tsel = (tsel & ~15) | 1;
    if ((tsel & 256) && (tsel & 15) != 4) {  // split-K combined in-launch
      int s2 = split_hint, t2 = tsel;
      gemm_tiled_plan(M, N, K, &t2, &s2, false);
      int bm, bn;
      tile_dims(t2 & 15, &bm, &bn);
      if (s2 > 1 && (int64_t)tiles_of(M, N, bm, bn) * s2 * bm * bn * 4 <= ws_bytes) return 0;
    }
    s = split_hint;
    gemm_tiled_plan(M, N, K, &tsel, &s, false);
    if ((tsel & 15) == 4 || (tsel & 128)) return 0;
  }
  if ((int64_t)s * M * N * 4 > ws_bytes) s = 1;
  return s > 1 ? s : 0;
}

// QKV projection with the RoPE + paged-KV write in its LDS-staged epilogue (common.h QkvEpi, tuned kind 3).
// Plan: the hints, else the tuned kind-3 entry, else the static tiled plan; a split plan runs as an in-launch
// combine (the epilogue needs finished sums). Returns -1 when the shape / plan cannot take the epilogue
// (stream / big-tile / stream-K plans, neox RoPE on tiles that are not head-aligned, workspace too small) -
// the caller then runs the plain GEMM and the rope_cache kernel; 0 when launched.
int launch_gemm_qkv(const void* x, int64_t ldx, const void* w, int64_t ldw, const void* bias, void* y, int64_t ldy,
                    int M, int N, int K, void* workspace, int64_t ws_bytes, int nt_hint, int split_hint,
                    const QkvEpi& qe, hipStream_t st) {
  if (M == 0) return 0;
  if (qe.D <= 0) return -1;
  if (!y) throw std::runtime_error("gemm_qkv: output buffer required");
  if (K % 16) throw std::runtime_error("gemm_qkv: K must be a multiple of 16");
  if (qe.D % 8 || N != (qe.nh + 2 * qe.nkv) * qe.D || N % 8 || ldy % 8) return -1;
  if (qe.do_rope && (qe.rot % 8 || qe.rot > qe.D || (qe.style == 0 && qe.rot % 16))) return -1;
  if (nt_hint == 0 && split_hint == 0) gemm_tuned_get(M, N, K, false, 3, &nt_hint, &split_hint);
  if (nt_hint & 0xff) return -1;  // streaming kernels have no LDS-staged epilogue
  if ((nt_hint >> 8) & kDecHint) {  // decode GEMM: unsplit, or split and combined in the launch (finished sums)
    int bn;
    if (M > 64 || !gemm_dec_bn((nt_hint >> 8) & 15, &bn)) return -1;
    if (qe.do_rope && qe.style == 0 && bn % qe.D) return -1;
    const int s = dec_split(M, N, K, split_hint, ws_bytes);
    const int tsel = (nt_hint >> 8) | (s > 1 ? 256 : 0);
    if (s > 1 && !dec_combine_fits(N, tsel, s, ws_bytes)) return -1;
    launch_tiled((const bf16_t*)x, ldx, w, ldw, (const bf16_t*)bias, (bf16_t*)y, ldy, M, N, K, 0, 0, tsel, s,
                 workspace, ws_bytes, false, st, nullptr, &qe);
    return 0;
  }
  int tsel = nt_hint >> 8, s = split_hint;
  gemm_tiled_plan(M, N, K, &tsel, &s, false);
  if ((tsel & 15) == 4 || (tsel & 128)) return -1;
  int bm, bn;
  tile_dims(tsel & 15, &bm, &bn);
  if (qe.do_rope && qe.style == 0 && bn % qe.D) return -1;  // neox partner columns must share the tile
  if (s > 1) {
    if ((int64_t)tiles_of(M, N, bm, bn) * s * bm * bn * 4 > ws_bytes) return -1;
    tsel |= 256;
  }
  launch_tiled((const bf16_t*)x, ldx, w, ldw, (const bf16_t*)bias, (bf16_t*)y, ldy, M, N, K, 0, 0, tsel, s, workspace,
               ws_bytes, false, st, nullptr, &qe);
  return 0;
}

int launch_gemm_qkv_args(const void* x, int64_t ldx, const void* w, int64_t ldw, const void* bias, void* y, int64_t ldy,
                         int M, int N, int K, void* workspace, int64_t ws_bytes, int nt_hint, int split_hint,
                         const void* pos, const void* cos_t, const void* sin_t, void* kc, void* vc, const void* slot,
                         int nh, int nkv, int D, int rot, int block_size, int style, bool do_rope, hipStream_t st) {
  const QkvEpi qe{(const int64_t*)pos, (const float*)cos_t, (const float*)sin_t, (bf16_t*)kc, (bf16_t*)vc,
                  (const int64_t*)slot, nh, nkv, D, rot, block_size, style, do_rope ? 1 : 0};
  return launch_gemm_qkv(x, ldx, w, ldw, bias, y, ldy, M, N, K, workspace, ws_bytes, nt_hint, split_hint, qe, st);
}

void gemm_plan(int M, int N, int K, bool w_fp8, int* nt, int* splitk) {
  if (gemm_tuned_get(M, N, K, false, w_fp8 ? 1 : 0, nt, splitk)) {
    if ((*nt >> 8) & kDecHint) {
      *splitk = ((*nt >> 8) & 256) ? 1 : dec_split(M, N, K, *splitk, INT64_MAX);
    } else if ((*nt >> 8) & (128 | 256)) {
      *splitk = 1;  // stream-K / split-K combine finish their tiles in-kernel: no partial slabs for the consumer
    } else if (*nt >> 8) {  // tiled hint: the split the kernel will really use
      int tsel = *nt >> 8;
      gemm_tiled_plan(M, N, K, &tsel, splitk, false);
    }
    return;
  }
  if (M <= 16 || (w_fp8 && M > 128)) {
    gemm_stream_plan(std::min(M, 128), N, K, nt, splitk);
  } else {
    int tsel = 0, s = 0;
    gemm_tiled_plan(M, N, K, &tsel, &s, false);
    *nt = tsel << 8;
    *splitk = s;
  }
}

