// Streaming-read ceilings on MI355X for the decode GEMM design (no compute, one pass over a buffer
// far larger than the Infinity Cache): what per-CU / chip read rate each load path reaches.
//   dma<NS, L>   : buffer_load ... lds ring (NS slots, L KiB per wave per slot), counted vmcnt + s_barrier
//                  per slot - the gemm_tiled / gemm_mid staging pattern without the MFMA work
//   vgpr<U>      : global 16-B loads straight into registers, U per lane in flight, folded into a checksum
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 bench/stream_ceiling.hip -o bench/stream_ceiling
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e));      \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define LDS_AS __attribute__((address_space(3)))

template <int NS, int L, int NW, int AUX>
__global__ __launch_bounds__(64 * NW) void dma_kernel(const char* __restrict__ src, size_t chunk, unsigned* out) {
  __shared__ __attribute__((aligned(16))) char ring[NS * NW * L * 1024];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const char* base = src + (size_t)blockIdx.x * chunk;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)chunk, 0x00020000);
  constexpr int SLOT = NW * L * 1024;
  const int steps = (int)(chunk / SLOT);
  const uint32_t voff = (uint32_t)(w * L * 1024 + lane * 16);
#define ISSUE(T_)                                                                                            \
  do {                                                                                                       \
    char* d_ = ring + ((T_) % NS) * SLOT + w * L * 1024;                                                     \
    const int so_ = (T_) * SLOT;                                                                             \
    _Pragma("unroll") for (int i_ = 0; i_ < L; ++i_)                                                         \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(d_ + i_ * 1024), 16, (uint32_t)(voff + i_ * 1024), \
                                               (uint32_t)so_, 0, AUX);                                       \
  } while (0)
  for (int j = 0; j < NS - 1 && j < steps; ++j) ISSUE(j);
  unsigned acc = 0;
  for (int t = 0; t < steps; ++t) {
    const int younger = min(steps - 1 - t, NS - 2);
    if (NS >= 5 && younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * L) : "memory");
    else if (NS >= 4 && younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * L) : "memory");
    else if (NS >= 3 && younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(L) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < steps) ISSUE(t + NS - 1);
    acc += *reinterpret_cast<const unsigned*>(ring + (t % NS) * SLOT + threadIdx.x * 4);
  }
#undef ISSUE
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}


// the GEMM weight-tile pattern: workgroup w streams rows [w*BN, (w+1)*BN) x K of a [rows][K] bf16 matrix,
// one 128-B k-slice of every row per ring slot (8 rows x 128 B per wave-instruction), as gemm_mid does.
// PACKED: the same bytes laid out [rows/16][K/64][16][64] (a slot = BN/16 contiguous 2-KiB panels);
// WITHA: each slot also stages a 64-row x 128-B activation tile from a 512 KiB (L2-resident) matrix
template <int NS, int BN, int NW, bool PACKED, bool WITHA>
__global__ __launch_bounds__(64 * NW) void tile_kernel(const char* __restrict__ src, const char* __restrict__ act,
                                                       int K, int ksplit, unsigned* out) {
  constexpr int BBYTES = BN * 128, ABYTES = WITHA ? 64 * 128 : 0, SLOT = BBYTES + ABYTES;
  constexpr int L = BN / (8 * NW), LA = WITHA ? 64 / (8 * NW) : 0;
  __shared__ __attribute__((aligned(16))) char ring[NS * SLOT];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rt = blockIdx.x / ksplit, kz = blockIdx.x % ksplit;
  const size_t rowb = (size_t)K * 2;
  const int steps = K / 64 / ksplit;
  const int k64 = K / 64;
  const char* base = PACKED ? src + (size_t)rt * BN * rowb + (size_t)kz * steps * 2048
                            : src + (size_t)rt * BN * rowb + (size_t)kz * steps * 128;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)(BN * rowb), 0x00020000);
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(act + (size_t)kz * steps * 128), (short)0,
                                                    (int)(64 * rowb), 0x00020000);
  uint32_t voff[L], aoff[LA > 0 ? LA : 1];
#pragma unroll
  for (int i = 0; i < L; ++i) {
    const int r = (i * NW + w) * 8 + (lane >> 3);
    voff[i] = PACKED ? (uint32_t)((r / 16) * k64 * 2048 + (r % 16) * 128 + (lane & 7) * 16)
                     : (uint32_t)(r * rowb + (lane & 7) * 16);
  }
#pragma unroll
  for (int i = 0; i < LA; ++i) aoff[i] = (uint32_t)(((i * NW + w) * 8 + (lane >> 3)) * rowb + (lane & 7) * 16);
#define TISSUE(T_)                                                                                           \
  do {                                                                                                       \
    char* d_ = ring + ((T_) % NS) * SLOT;                                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < LA; ++i_)                                                        \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)(d_ + BBYTES + (i_ * NW + w) * 1024), 16,   \
                                               (uint32_t)aoff[i_], (uint32_t)((T_) * 128), 0, 0);           \
    _Pragma("unroll") for (int i_ = 0; i_ < L; ++i_)                                                         \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(d_ + (i_ * NW + w) * 1024), 16, (uint32_t)voff[i_], \
                                               (uint32_t)((T_) * (PACKED ? 2048 : 128)), 0, 2);              \
  } while (0)
  constexpr int LT = L + LA;
  for (int j = 0; j < NS - 1 && j < steps; ++j) TISSUE(j);
  unsigned acc = 0;
  for (int t = 0; t < steps; ++t) {
    const int younger = min(steps - 1 - t, NS - 2);
    if (NS >= 5 && younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LT) : "memory");
    else if (NS >= 4 && younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LT) : "memory");
    else if (NS >= 3 && younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < steps) TISSUE(t + NS - 1);
    acc += *reinterpret_cast<const unsigned*>(ring + (t % NS) * SLOT + threadIdx.x * 4);
  }
#undef TISSUE
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

// row-major weight tile with RB bytes of every row per ring slot (RB = 128: gemm_mid's k-step; RB = 256: a 128-element
// bf16 k-step, each wave-instruction 64 * 16 / RB rows x RB contiguous bytes), plus the 64-row activation tile
template <int NS, int BN, int NW, int RB>
__global__ __launch_bounds__(64 * NW) void tile_rb_kernel(const char* __restrict__ src, const char* __restrict__ act,
                                                          int K, int ksplit, unsigned* out) {
  constexpr int BBYTES = BN * RB, ABYTES = 64 * RB, SLOT = BBYTES + ABYTES;
  constexpr int RPI = 1024 / RB;  // rows per wave-instruction
  constexpr int L = BN / (RPI * NW), LA = 64 / (RPI * NW);
  static_assert(L >= 1 && LA >= 1, "tile rows must cover the waves");
  __shared__ __attribute__((aligned(16))) char ring[NS * SLOT];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rt = blockIdx.x / ksplit, kz = blockIdx.x % ksplit;
  const size_t rowb = (size_t)K * 2;
  const int steps = (int)(rowb / RB) / ksplit;
  const char* base = src + (size_t)rt * BN * rowb + (size_t)kz * steps * RB;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)(BN * rowb), 0x00020000);
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(act + (size_t)kz * steps * RB), (short)0,
                                                    (int)(64 * rowb), 0x00020000);
  uint32_t voff[L], aoff[LA];
#pragma unroll
  for (int i = 0; i < L; ++i)
    voff[i] = (uint32_t)(((i * NW + w) * RPI + lane / (RB / 16)) * rowb + (lane % (RB / 16)) * 16);
#pragma unroll
  for (int i = 0; i < LA; ++i)
    aoff[i] = (uint32_t)(((i * NW + w) * RPI + lane / (RB / 16)) * rowb + (lane % (RB / 16)) * 16);
#define RISSUE(T_)                                                                                           \
  do {                                                                                                       \
    char* d_ = ring + ((T_) % NS) * SLOT;                                                                    \
    _Pragma("unroll") for (int i_ = 0; i_ < LA; ++i_)                                                        \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)(d_ + BBYTES + (i_ * NW + w) * 1024), 16,   \
                                               (uint32_t)aoff[i_], (uint32_t)((T_) * RB), 0, 0);            \
    _Pragma("unroll") for (int i_ = 0; i_ < L; ++i_)                                                         \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(d_ + (i_ * NW + w) * 1024), 16, (uint32_t)voff[i_], \
                                               (uint32_t)((T_) * RB), 0, 2);                                 \
  } while (0)
  constexpr int LT = L + LA;
  for (int j = 0; j < NS - 1 && j < steps; ++j) RISSUE(j);
  unsigned acc = 0;
  for (int t = 0; t < steps; ++t) {
    const int younger = min(steps - 1 - t, NS - 2);
    if (NS >= 4 && younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LT) : "memory");
    else if (NS >= 3 && younger >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LT) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + NS - 1 < steps) RISSUE(t + NS - 1);
    acc += *reinterpret_cast<const unsigned*>(ring + (t % NS) * SLOT + threadIdx.x * 4);
  }
#undef RISSUE
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <int U, int NW>
__global__ __launch_bounds__(64 * NW) void vgpr_kernel(const char* __restrict__ src, size_t chunk, unsigned* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const char* base = src + (size_t)blockIdx.x * chunk;
  const size_t per_iter = (size_t)NW * U * 1024;
  unsigned acc = 0;
  for (size_t o = 0; o + per_iter <= chunk; o += per_iter) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(base + o + (size_t)(u * NW + w) * 1024 + lane * 16));
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] + v[u][1] + v[u][2] + v[u][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

template <typename F>
static double time_us(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f(0);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f(i + 1);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms * 1e3 / reps;
}

int main() {
  const size_t total = 768ull << 20;  // per pass; 3 rotating buffers: 2.3 GB, far beyond the 256 MiB MALL
  std::vector<char*> bufs(3);
  for (auto& p : bufs) {
    CK(hipMalloc(&p, total));
    CK(hipMemset(p, 1, total));
  }
  unsigned* out;
  CK(hipMalloc(&out, 1 << 20));
  auto report = [&](const char* name, int grid, double us) {
    printf("%-28s grid %5d  %8.1f us  %6.2f TB/s  %6.1f GB/s per WG\n", name, grid, us, total / us / 1e6,
           total / us / 1e3 / grid);
    fflush(stdout);
  };
#define DMA(NS_, L_, NW_, AUX_, G_)                                                                           \
  do {                                                                                                     \
    const int g = (G_);                                                                                    \
    const size_t chunk = total / g;                                                                        \
    double us = time_us([&](int i) { dma_kernel<NS_, L_, NW_, AUX_><<<g, 64 * NW_>>>(bufs[i % 3], chunk, out); }, 6); \
    char nm[64];                                                                                           \
    snprintf(nm, sizeof nm, "dma ns%d L%d nw%d aux%d", NS_, L_, NW_, AUX_);                                \
    report(nm, g, us);                                                                                     \
  } while (0)
#define VG(U_, NW_, G_)                                                                                       \
  do {                                                                                                     \
    const int g = (G_);                                                                                    \
    const size_t chunk = total / g;                                                                        \
    double us = time_us([&](int i) { vgpr_kernel<U_, NW_><<<g, 64 * NW_>>>(bufs[i % 3], chunk, out); }, 6);  \
    char nm[64];                                                                                           \
    snprintf(nm, sizeof nm, "vgpr u%d nw%d", U_, NW_);                                                     \
    report(nm, g, us);                                                                                     \
  } while (0)
#define TILE(NS_, BN_, NW_, KS_, P_, A_)                                                                      \
  do {                                                                                                     \
    const int K = 4096, rows = (int)(total / (K * 2));                                                     \
    const int g = rows / BN_ * KS_;                                                                        \
    double us = time_us([&](int i) {                                                                       \
      tile_kernel<NS_, BN_, NW_, P_, A_><<<g, 64 * NW_>>>(bufs[i % 3], actbuf, K, KS_, out); }, 6);        \
    char nm[64];                                                                                           \
    snprintf(nm, sizeof nm, "tile ns%d bn%d nw%d ks%d %s%s", NS_, BN_, NW_, KS_, P_ ? "packed" : "rows",   \
             A_ ? "+A" : "");                                                                              \
    report(nm, g, us);                                                                                     \
  } while (0)
  char* actbuf;
  CK(hipMalloc(&actbuf, 64 * 4096 * 2));
  CK(hipMemset(actbuf, 1, 64 * 4096 * 2));
  // the GEMM weight-tile pattern (96K rows of 8 KiB): row-major vs packed panels, without / with the A tile
  TILE(4, 128, 4, 1, false, true);
  TILE(4, 128, 4, 1, true, true);
  // one decode GEMM's worth (Llama-2-7B QKV: 12288 x 4096 bf16 = 100.7 MB) on GEMM-like grids
#define TILEQ(NS_, BN_, NW_, KS_, P_)                                                                         \
  do {                                                                                                     \
    const int K = 4096, rows = 12288;                                                                      \
    const int g = rows / BN_ * KS_;                                                                        \
    const size_t bytes = (size_t)rows * K * 2;                                                             \
    double us = time_us([&](int i) {                                                                       \
      tile_kernel<NS_, BN_, NW_, P_, true><<<g, 64 * NW_>>>(bufs[i % 3], actbuf, K, KS_, out); }, 20);     \
    printf("qkv-size tile ns%d bn%d ks%d %-6s grid %4d  %7.2f us  %5.2f TB/s\n", NS_, BN_, KS_,            \
           P_ ? "packed" : "rows", g, us, bytes / us / 1e6);                                               \
    fflush(stdout);                                                                                        \
  } while (0)
  TILEQ(4, 128, 4, 1, true);
  TILEQ(4, 128, 4, 2, true);
  TILEQ(4, 128, 4, 2, false);
  TILEQ(3, 128, 4, 2, true);
  TILEQ(2, 128, 4, 2, true);
  TILEQ(4, 128, 4, 4, true);
  TILEQ(3, 128, 4, 4, true);
  TILEQ(2, 128, 4, 4, true);
  TILEQ(2, 128, 4, 8, true);
  TILEQ(4, 64, 4, 1, true);
  TILEQ(3, 64, 4, 2, true);
  TILEQ(2, 64, 4, 2, true);
  TILEQ(2, 64, 4, 4, true);
  TILEQ(4, 256, 4, 4, true);
  TILEQ(4, 256, 4, 5, true);
  DMA(4, 4, 4, 2, 256);
  // row bytes per k-step: 128 (gemm_mid today) vs 256, one QKV-sized matrix, activation tile included
#define TILERB(NS_, BN_, NW_, KS_, RB_)                                                                       \
  do {                                                                                                     \
    const int K = 4096, rows = 12288;                                                                      \
    const int g = rows / BN_ * KS_;                                                                        \
    const size_t bytes = (size_t)rows * K * 2;                                                             \
    double us = time_us([&](int i) {                                                                       \
      tile_rb_kernel<NS_, BN_, NW_, RB_><<<g, 64 * NW_>>>(bufs[i % 3], actbuf, K, KS_, out); }, 20);       \
    printf("qkv-size rb%d tile ns%d bn%d nw%d ks%d grid %4d  %7.2f us  %5.2f TB/s\n", RB_, NS_, BN_, NW_, KS_, g, us, \
           bytes / us / 1e6);                                                                              \
    fflush(stdout);                                                                                        \
  } while (0)
  TILERB(4, 64, 4, 1, 128);
  TILERB(4, 64, 4, 1, 256);
  TILERB(3, 64, 4, 1, 256);
  TILERB(4, 128, 4, 2, 128);
  TILERB(3, 128, 4, 2, 256);
  TILERB(4, 192, 4, 4, 128);
  TILERB(2, 192, 4, 4, 256);
  TILERB(4, 96, 4, 2, 128);
  TILERB(3, 96, 4, 2, 256);
  return 0;
}
