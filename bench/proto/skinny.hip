// Standalone prototype / microbenchmark for skinny (decode) GEMMs on gfx950.
//   Y[M,N] = X[M,K] . W[N,K]^T,  M <= 128, weights streamed once from HBM.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../llmss_amd/csrc skinny.hip -o skinny
// Run:   ./skinny [probe|gemm]   (prints one line per configuration)
#include "gemm.hip"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// ------------------------------------------------------------------------------ pure streaming
template <int U, bool NT>
__global__ __launch_bounds__(256) void probe_stream(const u32x4* __restrict__ p, int64_t n16, float* out) {
  const int64_t per_wg = n16 / gridDim.x;
  const u32x4* b = p + blockIdx.x * per_wg;
  unsigned acc = 0;
  for (int64_t i = threadIdx.x; i + (U - 1) * 256 < per_wg; i += U * 256) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(b + i + u * 256) : b[i + u * 256];
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[0] = 1.f;
}


// W [N][K] bf16, WG = 4 waves x 16 rows, full K per wave; PAT 0: one instr = 16 rows x 64 B
// (lane -> row l & 15, 16 B at 16 (l >> 4)); PAT 1: 16 rows x 4 x 16 B scattered (32 B per lane
// split in two loads); PAT 2: 8 rows x 128 B (row l >> 3, 16 B at 16 (l & 7)).
template <int PAT, int U>
__global__ __launch_bounds__(256) void probe_rows(const bf16_t* __restrict__ W, int N, int K, float* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r0 = blockIdx.x * 64 + w * 16;
  unsigned acc = 0;
  const char* base;
  int step;  // bytes of k advanced per load instruction (per row)
  if (PAT == 0) { base = (const char*)(W + (int64_t)(r0 + (lane & 15)) * K) + 16 * (lane >> 4); step = 64; }
  else if (PAT == 1) { base = (const char*)(W + (int64_t)(r0 + (lane & 15)) * K) + 32 * (lane >> 4); step = 64; }
  else { base = (const char*)(W + (int64_t)(r0 + (lane >> 3)) * K) + 16 * (lane & 7); step = 128; }
  const int64_t rowb = (int64_t)K * 2;
  // total bytes per wave = 16 rows x rowb; instructions = 16 * rowb / 1024
  const int ninstr = (int)(16 * rowb / 1024);
  for (int i = 0; i + U <= ninstr; i += U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = i + u;
      const char* p;
      if (PAT == 0) p = base + (int64_t)j * 64;
      else if (PAT == 1) p = base + (int64_t)(j >> 1) * 128 + (j & 1) * 16;
      else p = base + (int64_t)(j & 1) * 8 * rowb + (int64_t)(j >> 1) * 128;
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[0] = 1.f;
}


// tiled-kernel-shaped streaming without MFMA: WG (4 waves) = BN rows x K/S; per 64-k stage the
// W tile (BN rows x 128 B, 8 rows per instruction) and optionally the X tile (64 rows x 128 B)
// are fetched either into registers (GL = false) or by global_load_lds into an NS-slot ring
// with a counted vmcnt + raw barrier (GL = true). Reads per row are split-K contiguous runs.
template <int BN, bool GL, bool WX, int NS>
__global__ __launch_bounds__(256) void probe_tile(const bf16_t* __restrict__ W, const bf16_t* __restrict__ X, int N,
                                                  int K, float* out) {
  constexpr int LW = BN / 32, LX = WX ? 2 : 0, L = LW + LX;  // instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[GL ? NS * (BN + (WX ? 64 : 0)) * 128 : 16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = xcd_remap(blockIdx.x, gridDim.x);
  const int n0 = nt * BN;
  const int nk = K / 64, per = nk / gridDim.y, t0 = blockIdx.y * per, t1 = t0 + per;
  unsigned acc = 0;
  auto issue = [&](int t, int slot) {
#pragma unroll
    for (int i = 0; i < LW; ++i) {
      const int inst = i * 4 + w, row = inst * 8 + (lane >> 3);
      const bf16_t* p = W + (int64_t)(n0 + row) * K + t * 64 + (lane & 7) * 8;
      if constexpr (GL) __builtin_amdgcn_global_load_lds((const void*)p, (LDS_AS void*)(smem + slot * (BN + (WX ? 64 : 0)) * 128 + inst * 1024), 16, 0, 2);
      else { u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p)); acc ^= v[0]; }
    }
#pragma unroll
    for (int i = 0; i < LX; ++i) {
      const int inst = i * 4 + w, row = inst * 8 + (lane >> 3);
      const bf16_t* p = X + (int64_t)row * K + t * 64 + (lane & 7) * 8;
      if constexpr (GL) __builtin_amdgcn_global_load_lds((const void*)p, (LDS_AS void*)(smem + slot * (BN + 64) * 128 + BN * 128 + inst * 1024), 16, 0, 0);
      else { u32x4 v = *reinterpret_cast<const u32x4*>(p); acc ^= v[1]; }
    }
  };
  if constexpr (GL) {
#pragma unroll
    for (int j = 0; j < NS - 1; ++j) issue(t0 + j, j);
    int cur = 0;
    for (int t = t0; t < t1; ++t) {
      if (t + NS - 1 < t1) {
        wait_vmcnt<L * (NS - 2)>();
      } else {
        wait_vmcnt<0>();
      }
      lds_barrier();
      acc ^= *reinterpret_cast<const unsigned*>(smem + cur * (BN + (WX ? 64 : 0)) * 128 + lane * 4);
      const int nxt = cur == 0 ? NS - 1 : cur - 1;
      if (t + NS - 1 < t1) issue(t + NS - 1, nxt);
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
  } else {
    for (int t = t0; t < t1; ++t) issue(t, 0);
  }
  if (acc == 0x12345678u) out[0] = 1.f;
}

// ------------------------------------------------------------------------------ wring GEMM
// WG = NW waves; wave w owns NTW 16-row n-tiles (rows n0w .. n0w + 16 NTW); WG k-range = split
// of K/64 sub-steps. W: per-wave register ring of D sub-steps (64 k each: 32 B per lane per
// n-tile, two dwordx4 loads = one 128-B line per 4 lanes). X: [16 MT rows x KC] chunks staged
// through registers into a 2-slot LDS ring (XOR-swizzled 16-B pieces), one barrier per chunk.
// The k order inside a 64-k sub-step is permuted identically for A and B (lane group g holds
// k = 16 g .. 16 g + 15 as two MFMA steps h = 0, 1).
template <int MT, int NTW, int NW, int KC, int D>
struct WrCfg {
  static constexpr int ROWS = MT * 16;
  static constexpr int SPC = KC / 64;           // sub-steps per X chunk
  static constexpr int RB = KC * 2;             // LDS bytes per X row
  static constexpr int XB = ROWS * RB;          // one X slot
  static constexpr int CPR = KC / 8;            // 16-B pieces per row
  static constexpr int XPT = ROWS * CPR / (NW * 64);
  static_assert(KC >= 128, "swizzle needs >= 16 pieces per row");
  static_assert((ROWS * CPR) % (NW * 64) == 0, "X chunk must split evenly over the WG");
  static_assert(D % SPC == 0, "ring depth must be a multiple of the X chunk");
};

template <int MT, int NTW, int NW, int KC, int D>
__device__ __forceinline__ void wr_load_x(const bf16_t* __restrict__ X, int64_t ldx, int M, int K, int kbase,
                                          u32x4 (&xr)[WrCfg<MT, NTW, NW, KC, D>::XPT]) {
  using C = WrCfg<MT, NTW, NW, KC, D>;
#pragma unroll
  for (int i = 0; i < C::XPT; ++i) {
    const int q = threadIdx.x + i * NW * 64;
    const int row = q / C::CPR, c = q % C::CPR;
    xr[i] = *reinterpret_cast<const u32x4*>(X + (int64_t)min(row, M - 1) * ldx + min(kbase + c * 8, K - 8));
  }
}

template <int MT, int NTW, int NW, int KC, int D>
__device__ __forceinline__ void wr_store_x(char* slot, const u32x4 (&xr)[WrCfg<MT, NTW, NW, KC, D>::XPT]) {
  using C = WrCfg<MT, NTW, NW, KC, D>;
#pragma unroll
  for (int i = 0; i < C::XPT; ++i) {
    const int q = threadIdx.x + i * NW * 64;
    const int row = q / C::CPR, c = q % C::CPR;
    *reinterpret_cast<u32x4*>(slot + row * C::RB + ((c ^ (row & 15)) << 4)) = xr[i];
  }
}

template <int NTW>
__device__ __forceinline__ void wr_load_w(const bf16_t* const (&wrow)[NTW], int k, u32x4 (&wr)[NTW][2]) {
#pragma unroll
  for (int t = 0; t < NTW; ++t) {
    const u32x4* p = reinterpret_cast<const u32x4*>(wrow[t] + k);
    wr[t][0] = __builtin_nontemporal_load(p);
    wr[t][1] = __builtin_nontemporal_load(p + 1);
  }
}

template <int MT, int NTW, int KC>
__device__ __forceinline__ void wr_compute(const char* slot, int kk, const u32x4 (&wr)[NTW][2],
                                           f32x4 (&acc)[MT][NTW], int li, int g) {
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = kk / 8 + 2 * g + h;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const int r = mt * 16 + li;
      const s16x8 a = *reinterpret_cast<const s16x8*>(slot + r * (KC * 2) + ((c ^ (r & 15)) << 4));
#pragma unroll
      for (int t = 0; t < NTW; ++t)
        acc[mt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(s16x8, wr[t][h]), acc[mt][t], 0, 0, 0);
    }
  }
}

template <int MT, int NTW, int NW, int KC, int D>
__global__ __launch_bounds__(NW * 64) void wring_kernel(const bf16_t* __restrict__ X, int64_t ldx,
                                                        const bf16_t* __restrict__ W, int64_t ldw,
                                                        bf16_t* __restrict__ Y, int64_t ldy, float* __restrict__ part,
                                                        int M, int N, int K) {
  using C = WrCfg<MT, NTW, NW, KC, D>;
  __shared__ __attribute__((aligned(16))) char xs[2 * C::XB];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int nb = xcd_remap(blockIdx.x, gridDim.x);
  const int n0w = nb * (NW * NTW * 16) + w * (NTW * 16);
  const int split = blockIdx.y, nsplit = gridDim.y;
  const int nsub_all = K / 64;
  const int sb = (int)((int64_t)nsub_all * split / nsplit), se = (int)((int64_t)nsub_all * (split + 1) / nsplit);
  const int nsub = se - sb;
  const int kb = sb * 64;

  f32x4 acc[MT][NTW];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NTW; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bf16_t* wrow[NTW];
#pragma unroll
  for (int t = 0; t < NTW; ++t) wrow[t] = W + (int64_t)min(n0w + t * 16 + li, N - 1) * ldw + kb + 16 * g;

  u32x4 xr[C::XPT];
  u32x4 wr[D][NTW][2];
  // prologue: X chunk 0 -> regs, W ring, X chunk 0 -> slot 0, X chunk 1 -> regs
  wr_load_x<MT, NTW, NW, KC, D>(X, ldx, M, K, kb, xr);
#pragma unroll
  for (int d = 0; d < D; ++d) wr_load_w<NTW>(wrow, min(d, nsub - 1) * 64, wr[d]);
  wr_store_x<MT, NTW, NW, KC, D>(xs, xr);
  wr_load_x<MT, NTW, NW, KC, D>(X, ldx, M, K, kb + C::SPC * 64, xr);
  __syncthreads();

  // steady state: body of D sub-steps (D a multiple of SPC), every prefetch in range, so the
  // body is branch-free and hipcc's counted vmcnt waits stay exact. X chunk c+1 is published at
  // the END of chunk c (store regs -> slot, barrier) and X chunk c+2 is prefetched into the regs.
  int s = 0;
  for (; s + 2 * D <= nsub; s += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int ss = s + d;
      wr_compute<MT, NTW, KC>(xs + ((ss / C::SPC) & 1) * C::XB, (d % C::SPC) * 64, wr[d], acc, li, g);
      __builtin_amdgcn_sched_barrier(0);
      wr_load_w<NTW>(wrow, (ss + D) * 64, wr[d]);
      __builtin_amdgcn_sched_barrier(0);  // hipcc otherwise sinks the prefetch below the X store
      if ((d + 1) % C::SPC == 0) {  // folded by the unroll
        const int c = (ss + 1) / C::SPC;
        wr_store_x<MT, NTW, NW, KC, D>(xs + (c & 1) * C::XB, xr);
        __syncthreads();
        wr_load_x<MT, NTW, NW, KC, D>(X, ldx, M, K, kb + (c + 1) * C::SPC * 64, xr);
      }
    }
  }
  // tail: remaining < 2 D sub-steps (guarded)
  for (; s < nsub; s += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int ss = s + d;
      if (ss < nsub) {
        wr_compute<MT, NTW, KC>(xs + ((ss / C::SPC) & 1) * C::XB, (d % C::SPC) * 64, wr[d], acc, li, g);
        if (ss + D < nsub) wr_load_w<NTW>(wrow, (ss + D) * 64, wr[d]);
        if ((d + 1) % C::SPC == 0 && ss + 1 < nsub) {
          const int c = (ss + 1) / C::SPC;
          wr_store_x<MT, NTW, NW, KC, D>(xs + (c & 1) * C::XB, xr);
          __syncthreads();
          wr_load_x<MT, NTW, NW, KC, D>(X, ldx, M, K, kb + (c + 1) * C::SPC * 64, xr);
        }
      }
    }
  }
  // epilogue: C layout col = lane & 15 -> n, row = 4 g + i -> m
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = mt * 16 + 4 * g + i;
      if (m >= M) continue;
#pragma unroll
      for (int t = 0; t < NTW; ++t) {
        const int n = n0w + t * 16 + li;
        if (n >= N) continue;
        if (nsplit > 1) part[((int64_t)split * M + m) * N + n] = acc[mt][t][i];
        else Y[(int64_t)m * ldy + n] = f2bf(acc[mt][t][i]);
      }
    }
}

// ------------------------------------------------------------------------------ reference
__global__ void ref_gemm(const bf16_t* X, const bf16_t* W, float* Y, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += bf2f(X[(int64_t)m * K + k]) * bf2f(W[(int64_t)n * K + k]);
  Y[(int64_t)m * N + n] = s;
}

__global__ void fill_rand(bf16_t* p, int64_t n, unsigned seed, float scale) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    unsigned h = (unsigned)i * 2654435761u ^ seed;
    h ^= h >> 13; h *= 0x5bd1e995u; h ^= h >> 15;
    p[i] = f2bf(((h & 0xffff) / 65536.f - 0.5f) * scale);
  }
}

__global__ void sum_slabs(const float* part, int S, int64_t n, float* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int j = 0; j < S; ++j) s += part[j * n + i];
    out[i] = s;
  }
}

__global__ void bf_to_f(const bf16_t* p, int64_t n, float* out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = bf2f(p[i]);
}

static float time_us(const std::function<void(int)>& fn, int iters) {
  for (int i = 0; i < 5; ++i) fn(i);
  CK(hipDeviceSynchronize());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipEventRecord(a, 0));
  for (int i = 0; i < iters; ++i) fn(i);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3f / iters;
}

struct Shape {
  const char* name;
  int N, K;
  int hint, split;  // tuned plan of the current engine (bench log) for M = 64
};

template <int MT, int NTW, int NW, int KC, int D>
static void launch_wring(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* part, int M, int N, int K, int S) {
  const int rows = NW * NTW * 16;
  dim3 grid((N + rows - 1) / rows, S);
  wring_kernel<MT, NTW, NW, KC, D><<<grid, NW * 64>>>(X, K, W, K, Y, N, part, M, N, K);
}

int main(int argc, char** argv) {
  const bool probe = argc > 1 && std::string(argv[1]) == "probe";
  const int M = argc > 2 ? atoi(argv[2]) : 64;
  float* dummy;
  CK(hipMalloc(&dummy, 64));
  if (probe) {
    const int64_t bytes = 1LL << 30;
    u32x4* buf;
    CK(hipMalloc(&buf, bytes));
    CK(hipMemset(buf, 1, bytes));
    const int64_t n16 = bytes / 16;
    for (int G : {256, 512, 1024, 2048, 4096}) {
      auto run = [&](auto kern, const char* nm) {
        float us = time_us([&](int) { kern<<<G, 256>>>(buf, n16, dummy); }, 20);
        printf("probe %s G=%d: %.1f us  %.3f TB/s\n", nm, G, us, bytes / us / 1e6);
      };
      run(probe_stream<4, false>, "U4");
      run(probe_stream<8, false>, "U8");
      run(probe_stream<8, true>, "U8nt");
      run(probe_stream<16, true>, "U16nt");
    }
    bf16_t* Wb = (bf16_t*)buf;
    for (int N : {12288, 32000}) {
      const int K = 4096;
      const int64_t wb = (int64_t)N * K * 2;
      auto run2 = [&](auto kern, const char* nm) {
        const int copies = (int)(bytes / wb);
        float us = time_us([&](int i) { kern<<<N / 64, 256>>>(Wb + (int64_t)(i % copies) * N * K, N, K, dummy); }, 50);
        printf("probe_rows %s N=%d: %.1f us  %.3f TB/s\n", nm, N, us, wb / us / 1e6);
      };
      run2(probe_rows<0, 8>, "pat0 U8");
      run2(probe_rows<0, 16>, "pat0 U16");
      run2(probe_rows<1, 8>, "pat1 U8");
      run2(probe_rows<1, 16>, "pat1 U16");
      run2(probe_rows<2, 8>, "pat2 U8");
      run2(probe_rows<2, 16>, "pat2 U16");
    }
    bf16_t* Xs;
    CK(hipMalloc(&Xs, 64 * 16384 * 2));
    for (int N : {12288, 4096}) {
      const int K = 4096;
      const int64_t wb = (int64_t)N * K * 2;
      const int copies = (int)(bytes / wb);
      auto run3 = [&](auto kern, int BN, const char* nm) {
        for (int S : {1, 2, 4, 8}) {
          float us = time_us([&](int i) { kern<<<dim3(N / BN, S), 256>>>(Wb + (int64_t)(i % copies) * N * K, Xs, N, K, dummy); }, 50);
          printf("probe_tile %s N=%d S=%d: %.1f us  %.3f TB/s\n", nm, N, S, us, wb / us / 1e6);
        }
      };
      run3(probe_tile<64, false, false, 2>, 64, "reg BN64");
      run3(probe_tile<64, false, true, 2>, 64, "reg BN64 +X");
      run3(probe_tile<64, true, false, 2>, 64, "glds BN64 NS2");
      run3(probe_tile<64, true, false, 4>, 64, "glds BN64 NS4");
      run3(probe_tile<64, true, true, 2>, 64, "glds BN64 +X NS2");
      run3(probe_tile<64, true, true, 4>, 64, "glds BN64 +X NS4");
      run3(probe_tile<128, true, false, 3>, 128, "glds BN128 NS3");
      run3(probe_tile<128, true, true, 3>, 128, "glds BN128 +X NS3");
      run3(probe_tile<256, true, false, 2>, 256, "glds BN256 NS2");
      run3(probe_tile<256, true, true, 2>, 256, "glds BN256 +X NS2");
    }
    return 0;
  }
  std::vector<Shape> shapes = {{"qkv", 12288, 4096, 0x300, 4},
                               {"o", 4096, 4096, 0x2300, 4},
                               {"gate_up", 22016, 4096, 0x2200, 1},
                               {"down", 4096, 11008, 0x2300, 4},
                               {"head", 32000, 4096, 0x2300, 1}};
  const int64_t ws_bytes = 256LL << 20;
  void* ws;
  CK(hipMalloc(&ws, ws_bytes));
  bf16_t *X, *Y;
  float *R, *T;
  CK(hipMalloc(&X, 128 * 16384 * 2));
  CK(hipMalloc(&Y, 128LL * 32000 * 2));
  CK(hipMalloc(&R, 128LL * 32000 * 4));
  CK(hipMalloc(&T, 128LL * 32000 * 4));
  fill_rand<<<1024, 256>>>(X, 128 * 16384, 7, 2.f);
  for (const Shape& sh : shapes) {
    const int N = sh.N, K = sh.K;
    const int64_t wb = (int64_t)N * K * 2;
    const int ncopy = std::max(2, (int)(700e6 / wb) + 1);
    std::vector<bf16_t*> Ws(ncopy);
    for (auto& p : Ws) {
      CK(hipMalloc(&p, wb));
      fill_rand<<<4096, 256>>>(p, (int64_t)N * K, (unsigned)(uintptr_t)p, 0.1f);
    }
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(X, Ws[0], R, M, N, K);
    CK(hipDeviceSynchronize());
    // current engine kernel
    {
      const bool partial = sh.split > 1;
      float us = time_us([&](int i) {
        launch_gemm(X, K, Ws[i % ncopy], K, false, nullptr, nullptr, Y, N, M, N, K, 0, false, ws, ws_bytes, sh.hint,
                    sh.split, partial, 0);
      }, 100);
      printf("%-8s M=%d N=%d K=%d current hint=%#x s=%d: %.2f us %.3f TB/s\n", sh.name, M, N, K, sh.hint, sh.split, us,
             wb / us / 1e6);
    }
    std::vector<std::pair<std::string, std::function<void(const bf16_t*, int)>>> vs;
#define T(BN, NS)                                                                                               \
  for (int S : {1, 2, 3, 4, 6, 8, 12}) {                                                                        \
    char nm[96];                                                                                                \
    snprintf(nm, sizeof nm, "tiled<64,%d,%d> S=%d", BN, NS, S);                                                 \
    vs.push_back({nm, [=](const bf16_t* W, int) {                                                               \
      dim3 grid((N + BN - 1) / BN, S);                                                                          \
      gemm_tiled_kernel<64, BN, NS, true><<<grid, 256>>>(X, K, W, K, nullptr, Y, N, S > 1 ? (float*)ws : nullptr, \
                                                         M, N, K, 0, 0, nullptr);                               \
    }});                                                                                                        \
  }
    T(256, 2)
    T(256, 3)
    T(128, 4)
    T(128, 3)
    T(64, 6)
#undef T
#define V(MT, NTW, NW, KC, D)                                                                                   \
  for (int S : {1, 2, 3, 4, 6, 8, 12}) {                                                                                \
    char nm[96];                                                                                              \
    snprintf(nm, sizeof nm, "wring<%d,%d,%d,%d,%d> S=%d", MT, NTW, NW, KC, D, S);                            \
    vs.push_back({nm, [=](const bf16_t* W, int) {                                                             \
      launch_wring<MT, NTW, NW, KC, D>(X, W, Y, (float*)ws, M, N, K, S);                                       \
    }});                                                                                                      \
    (void)0;                                                                                                  \
  }
    V(4, 1, 4, 256, 4)
    V(4, 2, 4, 256, 4)
#undef V
    for (auto& v : vs) {
      const int S = atoi(v.first.c_str() + v.first.rfind('=') + 1);
      if ((int64_t)S * M * N * 4 > ws_bytes) continue;
      const int rows = v.first[0] == 't' ? atoi(v.first.c_str() + v.first.find(',') + 1)
                                         : atoi(v.first.c_str() + v.first.find('<') + 3) * atoi(v.first.c_str() + v.first.find('<') + 5) * 16;
      const int G = ((N + rows - 1) / rows) * S;
      if ((K / 64) / S < 16 || G < 200 || G > 2100) continue;
      v.second(Ws[0], 0);
      CK(hipDeviceSynchronize());
      if (S > 1) sum_slabs<<<1024, 256>>>((float*)ws, S, (int64_t)M * N, T);
      else bf_to_f<<<1024, 256>>>(Y, (int64_t)M * N, T);
      std::vector<float> hr((size_t)M * N), ht((size_t)M * N);
      CK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(ht.data(), T, ht.size() * 4, hipMemcpyDeviceToHost));
      double err = 0, mx = 0;
      for (size_t i = 0; i < hr.size(); ++i) {
        err = std::max(err, (double)fabsf(hr[i] - ht[i]));
        mx = std::max(mx, (double)fabsf(hr[i]));
      }
      float us = time_us([&](int i) { v.second(Ws[i % ncopy], i); }, 100);
      printf("%-8s M=%d %s: %.2f us %.3f TB/s  maxerr %.3g (max %.3g)%s\n", sh.name, M, v.first.c_str(), us,
             wb / us / 1e6, err, mx, err > 2e-2 * mx + 1e-3 ? "  MISMATCH" : "");
    }
    for (auto& p : Ws) CK(hipFree(p));
  }
  return 0;
}
