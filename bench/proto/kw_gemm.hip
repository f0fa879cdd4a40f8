// Prototype: decode GEMM (M <= 64) with K split over the waves of a workgroup and BOTH operands loaded straight
// into VGPRs (buffer loads, no LDS and no barrier in the K-loop), then one LDS reduction of the waves' partial
// tiles. Built as a standalone .so for bench/kw_probe.py (A/B against the in-tree decode plans).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared bench/proto/kw_gemm.hip -o bench/proto/libkw.so
//
// Work: workgroup (bx, z) owns output columns [16 NT bx, 16 NT (bx + 1)) and the z-th of S K-ranges; its NW waves
// take the 64-deep k-steps of that range round-robin (wave w: steps w, w + NW, ...), so the workgroup as a whole
// reads every weight row front to back. Per k-step a wave loads 8 A fragments (4 m-tiles x 2 k-halves, 16 rows x
// 64 B each) and 2 NT B fragments, each lane 16 B in MFMA fragment order, D steps in flight (register ring).
#include "../../llmss_amd/csrc/common.h"

template <int NT, int NW, int D>
struct KwCfg {
  static constexpr int SLAB = 4 * NT * 1024;  // one wave's partial tile in C-fragment order (bytes)
  static constexpr int LDS = NW * SLAB;
};

template <int NT, int NW, int D, bool WNT>
__global__ __launch_bounds__(64 * NW, 1) void kw_gemm_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                             const bf16_t* __restrict__ W, int64_t ldw,
                                                             bf16_t* __restrict__ Y, int64_t ldy,
                                                             float* __restrict__ part, int M, int N, int K) {
  using C = KwCfg<NT, NW, D>;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * 16 * NT;
  const int S = gridDim.y, z = blockIdx.y;
  const int nks = K / 64;
  const int kb = (int)((int64_t)nks * z / S), ke = (int)((int64_t)nks * (z + 1) / S);
  const int nsteps = ke - kb;
  const int cnt = w < nsteps ? (nsteps - w + NW - 1) / NW : 0;

  const auto xr = uniform_rsrc(X, (int64_t)M * ldx * 2);
  const auto wr = uniform_rsrc(W, (int64_t)N * ldw * 2);
  // per-lane byte offsets of the fragments at k = 0 (rows clamped); the k-step goes into soffset
  uint32_t xo[4][2], wo[NT][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) xo[mt][s] = (uint32_t)((int64_t)min(mt * 16 + li, M - 1) * ldx * 2 + s * 64 + g * 16);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      wo[nt][s] = (uint32_t)((int64_t)min(n0 + nt * 16 + li, N - 1) * ldw * 2 + s * 64 + g * 16);
  }
  f32x4 acc[4][NT];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  u32x4 ra[D][4][2], rw[D][NT][2];
  auto load = [&](int c, u32x4 (&a)[4][2], u32x4 (&b)[NT][2]) {
    const uint32_t ko = (uint32_t)(kb + w + NW * c) * 128u;
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int s = 0; s < 2; ++s) b[nt][s] = __builtin_amdgcn_raw_buffer_load_b128(wr, wo[nt][s], ko, WNT ? 2 : 0);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) a[mt][s] = __builtin_amdgcn_raw_buffer_load_b128(xr, xo[mt][s], ko, 0);
  };
  auto compute = [&](const u32x4 (&a)[4][2], const u32x4 (&b)[NT][2]) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(s16x8, a[mt][s]),
                                                                __builtin_bit_cast(s16x8, b[nt][s]), acc[mt][nt], 0, 0, 0);
  };

  if (cnt > 0) {
#pragma unroll
    for (int d = 0; d < D - 1; ++d) load(min(d, cnt - 1), ra[d], rw[d]);
    int i = 0;
    // steady state: every prefetch of the group is a valid step of this wave (branch-free: exact vmcnt counts)
    for (; i + 2 * D - 1 <= cnt; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        load(i + d + D - 1, ra[(d + D - 1) % D], rw[(d + D - 1) % D]);
        compute(ra[d], rw[d]);
      }
    }
    for (; i < cnt; i += D) {
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if (i + d < cnt) {
          if (i + d + D - 1 < cnt) load(i + d + D - 1, ra[(d + D - 1) % D], rw[(d + D - 1) % D]);
          compute(ra[d], rw[d]);
        }
      }
    }
  }

  // reduction: every wave stores its partial tile (C-fragment order, 1 KiB per fragment, lane-linear), then wave w
  // sums fragments w, w + NW, ... over the NW slabs and stores them
  float* sl = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int mt = 0; mt < 4; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
      *reinterpret_cast<f32x4*>(sl + (w * 4 * NT + mt * NT + nt) * 256 + lane * 4) = acc[mt][nt];
  __syncthreads();
  for (int f = w; f < 4 * NT; f += NW) {
    f32x4 v = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < NW; ++q) v += *reinterpret_cast<const f32x4*>(sl + (q * 4 * NT + f) * 256 + lane * 4);
    const int mt = f / NT, nt = f % NT;
    const int n = n0 + nt * 16 + li;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * g + i;
      if (m < M && n < N) {
        if (S > 1) part[((int64_t)z * M + m) * N + n] = v[i];
        else Y[(int64_t)m * ldy + n] = f2bf(v[i]);
      }
    }
  }
}

template <int NT, int NW, int D, bool WNT>
static int launch(const void* X, int64_t ldx, const void* W, int64_t ldw, void* Y, int64_t ldy, void* part, int M,
                  int N, int K, int S, hipStream_t st) {
  if (K % 64 || M > 64 || M <= 0) return -1;
  dim3 grid((N + 16 * NT - 1) / (16 * NT), S);
  hipLaunchKernelGGL((kw_gemm_kernel<NT, NW, D, WNT>), grid, dim3(64 * NW), 0, st, (const bf16_t*)X, ldx,
                     (const bf16_t*)W, ldw, (bf16_t*)Y, ldy, (float*)part, M, N, K);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

#define KW(id, NT, NW, D, WNT) \
  case id: return launch<NT, NW, D, WNT>(X, ldx, W, ldw, Y, ldy, part, M, N, K, S, st);

extern "C" int kw_gemm(int var, const void* X, int64_t ldx, const void* W, int64_t ldw, void* Y, int64_t ldy,
                       void* part, int M, int N, int K, int S, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (var) {
    KW(0, 3, 8, 2, true)
    KW(1, 3, 8, 3, true)
    KW(2, 3, 4, 3, true)
    KW(3, 3, 4, 4, true)
    KW(4, 2, 8, 3, true)
    KW(5, 4, 8, 2, true)
    KW(6, 1, 8, 3, true)
    KW(7, 1, 4, 4, true)
    KW(8, 3, 8, 3, false)
    KW(9, 2, 4, 4, true)
    KW(10, 4, 4, 3, true)
    KW(11, 6, 4, 2, true)
    default: return -3;
  }
}
