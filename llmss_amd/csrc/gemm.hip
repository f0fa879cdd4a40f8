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
// Two kernels, one choice per call (M is the only selector):
//  * gemm_skinny (M <= 64: decode / small batches). Weight-streaming: every weight byte is read
//    once, straight into VGPRs (no LDS round trip - guide §5 'GEMV / M <= 16' row), 32 B per
//    lane = full 128-B lines per 4 lanes; X fragments come from L2. A workgroup = 4 waves that
//    split K and reduce through LDS; more K splitting across workgroups (fp32 partial slabs +
//    splitk_reduce, which also applies the epilogue) only when N alone cannot fill 256 CUs.
//  * gemm_tiled (M > 64: prefill). 128x128x64 tile, 4 waves (2x2, 64x64 each, 16 mfma 16x16x32
//    accumulators), both operands staged global->LDS with 16-B global_load_lds into an
//    XOR-swizzled image (chunk ^= row & 7: conflict-free ds_read_b128, checked with a bank
//    simulator), double-buffered, XCD-aware tile order (guide T1).
#include "common.h"

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
// skinny GEMM (M <= 64)
// grid (ceil(N / (16*NT)), SPLITK), block 256 = 4 waves splitting the workgroup's K range.
// -------------------------------------------------------------------------------------------
template <int MT, int NT, int U, bool FP8W>
__global__ __launch_bounds__(256) void gemm_skinny_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                          const void* __restrict__ Wv, int64_t ldw,
                                                          const float* __restrict__ wscale,
                                                          const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                          int64_t ldy, float* __restrict__ part, int M, int N, int K,
                                                          int act, int glu) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * (16 * NT);
  const int split = blockIdx.y, nsplit = gridDim.y;
  // K in groups of 64; slices = nsplit * 4 waves
  const int ngrp = (K + 63) >> 6;
  const int nslice = nsplit * 4, sl = split * 4 + w;
  const int gb = (int)((int64_t)ngrp * sl / nslice), ge = (int)((int64_t)ngrp * (sl + 1) / nslice);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane row pointers
  const bf16_t* xrow[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) xrow[mt] = X + (int64_t)min(mt * 16 + li, M - 1) * ldx;
  const char* wrow[NT];
  constexpr int WB = FP8W ? 1 : 2;  // bytes per weight element
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
    wrow[nt] = (const char*)Wv + ((int64_t)min(n0 + nt * 16 + li, N - 1) * ldw) * WB;

  for (int gi = gb; gi < ge; gi += U) {
    u16x8 xa[U][MT][2];
    u32x4 wa[U][NT][FP8W ? 1 : 2];
    bool kok[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int gg = gi + u;
      // k < K is uniform per 16-lane group (K % 16 == 0); gg < ge is wave-uniform
      kok[u] = (gg < ge) && (gg * 64 + 16 * g < K);
      const int ko = kok[u] ? gg * 64 + 16 * g : 0;  // masked lanes read k 0..15 (K >= 16)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        xa[u][mt][0] = *reinterpret_cast<const u16x8*>(xrow[mt] + ko);
        xa[u][mt][1] = *reinterpret_cast<const u16x8*>(xrow[mt] + ko + 8);
      }
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        const u32x4* p = reinterpret_cast<const u32x4*>(wrow[nt] + (int64_t)ko * WB);
        wa[u][nt][0] = __builtin_nontemporal_load(p);
        if constexpr (!FP8W) wa[u][nt][1] = __builtin_nontemporal_load(p + 1);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (gi + u >= ge) break;  // wave-uniform
      const s16x8 z = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) {
        s16x8 b0, b1;
        if constexpr (FP8W) {
          fp8x16_to_bf16(wa[u][nt][0], b0, b1);
        } else {
          b0 = *reinterpret_cast<const s16x8*>(&wa[u][nt][0]);
          b1 = *reinterpret_cast<const s16x8*>(&wa[u][nt][1]);
        }
        b0 = kok[u] ? b0 : z;
        b1 = kok[u] ? b1 : z;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
          s16x8 a0 = *reinterpret_cast<const s16x8*>(&xa[u][mt][0]);
          s16x8 a1 = *reinterpret_cast<const s16x8*>(&xa[u][mt][1]);
          a0 = kok[u] ? a0 : z;
          a1 = kok[u] ? a1 : z;
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0, acc[mt][nt], 0, 0, 0);
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1, acc[mt][nt], 0, 0, 0);
        }
      }
    }
  }

  // ---- reduce the 4 K-slices of the workgroup through LDS --------------------------------
  __shared__ f32x4 red[3][MT][NT][64];
  if (w > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) red[w - 1][mt][nt][lane] = acc[mt][nt];
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int r = 0; r < 3; ++r) acc[mt][nt] += red[r][mt][nt][lane];

  // ---- epilogue --------------------------------------------------------------------------
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

// split-K reduction + epilogue: part [S, M, N] fp32 (w_scale already applied)
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const float* __restrict__ part, int S, int M, int N,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                            int64_t ldy, int act, int glu) {
  const int m = blockIdx.y;
  const int nout = glu ? N / 2 : N;
  for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < nout; c += gridDim.x * blockDim.x) {
    if (glu) {
      const int p = c >> 4, i = c & 15;
      const int ng = 32 * p + i, nu = ng + 16;
      float gv = 0.f, uv = 0.f;
      for (int s = 0; s < S; ++s) {
        gv += part[((int64_t)s * M + m) * N + ng];
        uv += part[((int64_t)s * M + m) * N + nu];
      }
      if (bias) { gv += bf2f(bias[ng]); uv += bf2f(bias[nu]); }
      Y[(int64_t)m * ldy + c] = f2bf(silu(gv) * uv);
    } else {
      float v = 0.f;
      for (int s = 0; s < S; ++s) v += part[((int64_t)s * M + m) * N + c];
      if (bias) v += bf2f(bias[c]);
      Y[(int64_t)m * ldy + c] = f2bf(apply_act(v, act));
    }
  }
}

// -------------------------------------------------------------------------------------------
// tiled GEMM (M > 64), bf16 weights
// -------------------------------------------------------------------------------------------
constexpr int TBM = 128, TBN = 128, TBK = 64;

__device__ __forceinline__ void tiled_stage(const bf16_t* __restrict__ A, int64_t lda, int M, const bf16_t* __restrict__ B,
                                            int64_t ldb, int N, int K, int m0, int n0, int k0, char* sA, char* sB,
                                            int w, int lane) {
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int inst = it * 4 + w;
    const int row = inst * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (row & 7);
    const int kc = min(k0 + c * 8, K - 8);
    const bf16_t* ga = A + (int64_t)min(m0 + row, M - 1) * lda + kc;
    const bf16_t* gb = B + (int64_t)min(n0 + row, N - 1) * ldb + kc;
    __builtin_amdgcn_global_load_lds((const void*)ga, (LDS_AS void*)(sA + inst * 1024), 16, 0, 0);
    __builtin_amdgcn_global_load_lds((const void*)gb, (LDS_AS void*)(sB + inst * 1024), 16, 0, 0);
  }
}

template <bool MASK>
__device__ __forceinline__ void tiled_compute(const char* sA, const char* sB, f32x4 (&acc)[4][4], int wr, int wc, int li,
                                              int g, int k0, int K) {
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = 4 * s + g;
    const bool valid = !MASK || (k0 + c * 8 < K);
    s16x8 a[4], b[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int ra = wr * 64 + t * 16 + li, rb = wc * 64 + t * 16 + li;
      a[t] = *reinterpret_cast<const s16x8*>(sA + ra * 128 + ((c ^ (ra & 7)) << 4));
      b[t] = *reinterpret_cast<const s16x8*>(sB + rb * 128 + ((c ^ (rb & 7)) << 4));
      if (MASK && !valid) { a[t] = s16x8{0, 0, 0, 0, 0, 0, 0, 0}; b[t] = a[t]; }
    }
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
  }
}

__global__ __launch_bounds__(256) void gemm_tiled_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                         const bf16_t* __restrict__ B, int64_t ldb,
                                                         const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                         int64_t ldy, int M, int N, int K, int act, int glu) {
  __shared__ __attribute__((aligned(16))) char smem[2 * 2 * TBM * TBK * 2];  // 64 KiB
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int ntn = (N + TBN - 1) / TBN, ntm = (M + TBM - 1) / TBM;
  const int tile = xcd_remap(blockIdx.x, ntn * ntm);
  const int m0 = (tile / ntn) * TBM, n0 = (tile % ntn) * TBN;

  f32x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + TBK - 1) / TBK;
  constexpr int TILE_BYTES = TBM * TBK * 2;  // one operand tile; buffer c: A at 2c, B at 2c+1
  tiled_stage(A, lda, M, B, ldb, N, K, m0, n0, 0, smem, smem + TILE_BYTES, w, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    char* nA = smem + (2 * (cur ^ 1)) * TILE_BYTES;
    char* cA = smem + (2 * cur) * TILE_BYTES;
    if (t + 1 < nk) tiled_stage(A, lda, M, B, ldb, N, K, m0, n0, (t + 1) * TBK, nA, nA + TILE_BYTES, w, lane);
    if (t + 1 == nk && (K % TBK)) tiled_compute<true>(cA, cA + TILE_BYTES, acc, wr, wc, li, g, t * TBK, K);
    else tiled_compute<false>(cA, cA + TILE_BYTES, acc, wr, wc, li, g, t * TBK, K);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  // epilogue
#pragma unroll
  for (int mt = 0; mt < 4; ++mt) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wr * 64 + mt * 16 + 4 * g + i;
      if (m >= M) continue;
      if (glu) {
#pragma unroll
        for (int p = 0; p < 2; ++p) {
          const int ng = n0 + wc * 64 + 2 * p * 16 + li, nu = ng + 16;
          if (nu < N) {
            float gv = acc[mt][2 * p][i], uv = acc[mt][2 * p + 1][i];
            if (bias) { gv += bf2f(bias[ng]); uv += bf2f(bias[nu]); }
            Y[(int64_t)m * ldy + (n0 + wc * 64) / 2 + p * 16 + li] = f2bf(silu(gv) * uv);
          }
        }
      } else {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
          const int n = n0 + wc * 64 + nt * 16 + li;
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

// -------------------------------------------------------------------------------------------
// host dispatch
// -------------------------------------------------------------------------------------------
template <int MT, int NT, int U, bool FP8W>
static void launch_skinny_t(const bf16_t* X, int64_t ldx, const void* W, int64_t ldw, const float* ws, const bf16_t* bias,
                            bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act, int glu, int splitk,
                            hipStream_t st) {
  dim3 grid((N + 16 * NT - 1) / (16 * NT), splitk);
  gemm_skinny_kernel<MT, NT, U, FP8W><<<grid, 256, 0, st>>>(X, ldx, W, ldw, ws, bias, Y, ldy, part, M, N, K, act, glu);
  HIP_CHECK_LAUNCH();
}

template <int MT, bool FP8W>
static void launch_skinny_m(const bf16_t* X, int64_t ldx, const void* W, int64_t ldw, const float* ws,
                            const bf16_t* bias, bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act,
                            int glu, int splitk, hipStream_t st) {
  constexpr int U = MT <= 1 ? 4 : 2;
  launch_skinny_t<MT, 2, U, FP8W>(X, ldx, W, ldw, ws, bias, Y, ldy, part, M, N, K, act, glu, splitk, st);
}

// Number of K-splits across workgroups: enough workgroups to put >= 2 on every CU.
int gemm_skinny_splitk(int M, int N, int K) {
  const int nblk = (N + 31) / 32;
  int s = 1;
  while (nblk * s < 512 && s < 16 && (K / 64) / (8 * s) >= 2) s *= 2;
  (void)M;
  return s;
}

void launch_gemm(const void* x, int64_t ldx, const void* w, int64_t ldw, bool w_fp8, const void* w_scale,
                 const void* bias, void* y, int64_t ldy, int M, int N, int K, int act, bool glu, void* workspace,
                 int64_t ws_bytes, hipStream_t st) {
  if (M == 0 || N == 0) return;
  if (K % 16) throw std::runtime_error("gemm: K must be a multiple of 16");
  if (glu && (N % 32)) throw std::runtime_error("gemm: glu needs N % 32 == 0");
  auto X = (const bf16_t*)x;
  auto B = (const bf16_t*)bias;
  auto Y = (bf16_t*)y;
  auto WS = (const float*)w_scale;
  const int g = glu ? 1 : 0;
  if (M <= 64 || w_fp8) {
    if (M > 64) {  // fp8 weights with many rows: loop over 64-row panels (prefill with fp8 weights)
      for (int m0 = 0; m0 < M; m0 += 64) {
        const int mm = std::min(64, M - m0);
        launch_gemm((const bf16_t*)x + m0 * ldx, ldx, w, ldw, w_fp8, w_scale, bias,
                    (bf16_t*)y + m0 * ldy, ldy, mm, N, K, act, glu, workspace, ws_bytes, st);
      }
      return;
    }
    int splitk = gemm_skinny_splitk(M, N, K);
    if ((int64_t)splitk * M * N * 4 > ws_bytes) splitk = 1;
    float* part = splitk > 1 ? (float*)workspace : nullptr;
    const int mt = (M + 15) / 16;
    const int act_k = splitk > 1 ? 0 : act, glu_k = splitk > 1 ? 0 : g;
    if (w_fp8) {
      if (mt == 1) launch_skinny_m<1, true>(X, ldx, w, ldw, WS, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
      else if (mt == 2) launch_skinny_m<2, true>(X, ldx, w, ldw, WS, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
      else launch_skinny_m<4, true>(X, ldx, w, ldw, WS, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
    } else {
      if (mt == 1) launch_skinny_m<1, false>(X, ldx, w, ldw, nullptr, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
      else if (mt == 2) launch_skinny_m<2, false>(X, ldx, w, ldw, nullptr, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
      else launch_skinny_m<4, false>(X, ldx, w, ldw, nullptr, B, Y, ldy, part, M, N, K, act_k, glu_k, splitk, st);
    }
    if (splitk > 1) {
      const int nout = glu ? N / 2 : N;
      dim3 grid(std::min((nout + 255) / 256, 64), M);
      splitk_reduce_kernel<<<grid, 256, 0, st>>>(part, splitk, M, N, B, Y, ldy, act, g);
      HIP_CHECK_LAUNCH();
    }
    return;
  }
  const int nwg = ((M + TBM - 1) / TBM) * ((N + TBN - 1) / TBN);
  gemm_tiled_kernel<<<nwg, 256, 0, st>>>(X, ldx, (const bf16_t*)w, ldw, B, Y, ldy, M, N, K, act, g);
  HIP_CHECK_LAUNCH();
}
