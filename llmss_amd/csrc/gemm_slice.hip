// Weight-slice GEMM for decode shapes whose weights are small per CU (M <= 64):
//   Y[M, N] = act(X[M, K] . W[N, K]^T + b)   or fp32 split-K slabs part[z, M, N] for the consumer.
//
// Why: a decode GEMM of a 15-20 MB projection (GPT-2-XL: c_attn 4800 x 1600, c_fc 6400 x 1600, ...)
// spends most of its ~10 us in latency, not bandwidth: the tiled kernels keep only a 3-4 stage ring of
// 8 KB weight tiles in flight per workgroup (a few MB chip-wide), so each k-step waits out an HBM round
// trip (profiles/r2_packed: a pure 100 MB read in one launch already costs 18 us; 15 MB GEMMs reached
// 1.6-2 TB/s). Here each workgroup owns 16*NT weight rows x one K slice small enough for LDS
// (<= 160 KiB) and issues the WHOLE slice as LDS-DMA (global_load_lds, non-temporal: read once per
// step) in its first instructions - with ~300-400 workgroups resident the entire weight is in flight
// at once, so the launch costs one round trip plus the transfer at full HBM rate. The activations
// (M x K, L2-resident: written by the previous kernel) are loaded straight into MFMA A fragments, a
// register double buffer of XU k-steps, issued behind the weight DMA. Wave w computes rows
// [16w, 16w+16) against all 16*NT columns (v_mfma_f32_16x16x32_bf16, B fragments from the swizzled
// LDS image: chunk c of row r at c ^ (r & 7), conflict-free ds_read_b128).
// Reference: the reference's Linear is F.linear -> cuBLAS (utils/layers.py:39-62).
#include "common.h"

namespace {

constexpr int kSliceXU = 8;  // k32-steps of A fragments per register buffer (2 buffers)

template <int NT>
__global__ __launch_bounds__(256, 2) void gemm_slice_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                            const bf16_t* __restrict__ W, int64_t ldw,
                                                            const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                            int64_t ldy, float* __restrict__ part, int M, int N,
                                                            int K, int act) {
  extern __shared__ __attribute__((aligned(16))) char wimg[];  // [stage][16*NT rows][128 B]
  constexpr int ROWS = 16 * NT;
  constexpr int IPS = ROWS / 8;  // 1-KiB DMA instructions per 64-k stage
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int n0 = blockIdx.x * ROWS;
  const int nstg_all = (K + 63) / 64;
  const int z = blockIdx.y, nz = gridDim.y;
  const int s0 = (int)((int64_t)nstg_all * z / nz), s1 = (int)((int64_t)nstg_all * (z + 1) / nz);
  const int nst = s1 - s0;
  const int kb = s0 * 64, ke = min(K, s1 * 64);

  // 1) the whole weight slice: nst stages x IPS instructions, dealt round-robin over the 4 waves
  for (int i = w; i < nst * IPS; i += 4) {
    const int st = i / IPS, rb = i % IPS;
    const int row = rb * 8 + (lane >> 3);
    const int c = (lane & 7) ^ (row & 7);
    const int kc = min(kb + st * 64 + c * 8, K - 8);
    const bf16_t* src = W + (int64_t)min(n0 + row, N - 1) * ldw + kc;
    __builtin_amdgcn_global_load_lds((const void*)src, (LDS_AS void*)(wimg + i * 1024), 16, 0, 2);
  }

  // 2) A fragments of this wave's 16 rows, XU k32-steps per buffer
  const int mrow = 16 * w + li;
  const bool wave_live = 16 * w < M;
  const bf16_t* xr = X + (int64_t)min(mrow, M - 1) * ldx;
  const int nk32 = (ke - kb + 31) / 32;
  s16x8 xa[kSliceXU], xb[kSliceXU];
  auto load_x = [&](s16x8(&buf)[kSliceXU], int j0) {
#pragma unroll
    for (int u = 0; u < kSliceXU; ++u) {
      const int k = kb + (j0 + u) * 32 + 8 * g;
      buf[u] = *reinterpret_cast<const s16x8*>(xr + min(k, K - 8));
    }
  };
  if (wave_live) load_x(xa, 0);

  f32x4 acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  // the DMA (issued first) and the first A buffer have landed; the barrier publishes every wave's DMA
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  auto compute = [&](const s16x8(&buf)[kSliceXU], int j0) {
#pragma unroll
    for (int u = 0; u < kSliceXU; ++u) {
      const int j = j0 + u;
      if (j < nk32) {
        const int k = kb + j * 32 + 8 * g;
        const s16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
        const s16x8 a = k < ke ? buf[u] : zero;
        const int st = j >> 1, c = 4 * (j & 1) + g;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int row = t * 16 + li;
          const char* p = wimg + (st * IPS + (row >> 3)) * 1024 + (row & 7) * 128 + ((c ^ (row & 7)) << 4);
          const s16x8 b = k < ke ? *reinterpret_cast<const s16x8*>(p) : zero;
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[t], 0, 0, 0);
        }
      }
    }
  };
  if (wave_live) {
    for (int j0 = 0; j0 < nk32; j0 += 2 * kSliceXU) {
      if (j0 + kSliceXU < nk32) load_x(xb, j0 + kSliceXU);
      compute(xa, j0);
      if (j0 + kSliceXU >= nk32) break;
      if (j0 + 2 * kSliceXU < nk32) load_x(xa, j0 + 2 * kSliceXU);
      compute(xb, j0 + kSliceXU);
    }
  }
  if (!wave_live) return;

  // 3) epilogue (C layout: row 4g + i of the wave's tile, column li of each 16-column tile)
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = 16 * w + 4 * g + i;
    if (m >= M) continue;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int n = n0 + t * 16 + li;
      if (n >= N) continue;
      if (nz > 1) {
        part[((int64_t)z * M + m) * N + n] = acc[t][i];
      } else {
        float v = acc[t][i];
        if (bias) v += bf2f(bias[n]);
        Y[(int64_t)m * ldy + n] = f2bf(apply_act(v, act));
      }
    }
  }
}

template <int NT>
void set_slice_lds(int bytes) {
  static int done = 0;
  if (bytes > done) {
    if (hipFuncSetAttribute((const void*)gemm_slice_kernel<NT>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) !=
        hipSuccess)
      throw std::runtime_error("gemm_slice: cannot reserve dynamic LDS");
    done = bytes;
  }
}

}  // namespace

// LDS bytes one workgroup of the slice kernel needs (the launcher and the host-side validation agree)
int gemm_slice_lds(int N, int K, int nt, int split) {
  const int nstg = (K + 63) / 64;
  const int per = (nstg + split - 1) / split;
  return per * 16 * nt * 128;
}

// nt = 1 (16 weight rows per workgroup) or 2 (32); split = K slices (fp32 slabs when > 1)
void launch_gemm_slice(const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw, const bf16_t* bias, bf16_t* Y,
                       int64_t ldy, float* part, int M, int N, int K, int act, int nt, int split, hipStream_t st) {
  if (M > 64) throw std::runtime_error("gemm_slice: M must be <= 64");
  if (K % 8 || K < 64) throw std::runtime_error("gemm_slice: K must be a multiple of 8 and >= 64");
  if (nt != 1 && nt != 2) throw std::runtime_error("gemm_slice: nt must be 1 or 2");
  const int nstg = (K + 63) / 64;
  if (split < 1 || split > nstg) throw std::runtime_error("gemm_slice: bad split");
  if (split > 1 && !part) throw std::runtime_error("gemm_slice: split-K needs the slab workspace");
  const int lds = gemm_slice_lds(N, K, nt, split);
  if (lds > 160 * 1024) throw std::runtime_error("gemm_slice: weight slice exceeds LDS (raise split)");
  dim3 grid((N + 16 * nt - 1) / (16 * nt), split);
  if (nt == 1) {
    set_slice_lds<1>(lds);
    gemm_slice_kernel<1><<<grid, 256, lds, st>>>(X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act);
  } else {
    set_slice_lds<2>(lds);
    gemm_slice_kernel<2><<<grid, 256, lds, st>>>(X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act);
  }
  HIP_CHECK_LAUNCH();
}
