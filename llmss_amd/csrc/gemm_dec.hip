// Decode GEMM at M <= 64 rows (gemm_dec): Y[M, N] = epilogue(X[M, K] . W[N, K]^T), bf16 in, fp32 accumulate,
// with the K loop split over the four waves of a workgroup instead of its columns.
//
// Why (profiles/r6_dec): at M = 64 the column-split tiles (gemm_mid / gemm_tiled) take the same time with their
// weights resident in the Infinity Cache as streamed from HBM (GPT-2-XL up 10.5 vs 10.7 us, down 12.2 vs 12.5), and
// their MFMA-only variant - no memory traffic at all - already takes 4-19 us (profiles/r4_gemm midm_probe): the
// time is the k-step cadence. Every k-step of a column-split tile is a serial chain of a ring wait, a workgroup
// barrier, the LDS fragment reads and the MFMAs that need them, ~460 cycles with one wave per SIMD, and a 64 x 32
// tile walks all 25-100 k-steps of GPT-2-XL's K one after another.
//
// Here wave w of the workgroup takes k-steps t0 + w, t0 + w + 4, ... of the workgroup's K slice and computes the
// whole 16*MT x BN tile over them:
//   * each wave stages ITS OWN k-steps (A rows and B rows of one 128-byte k-step = (16 MT + BN) x 128 B, full
//     lines by buffer_load ... lds, XOR-swizzled 16-B chunks as gemm_mid) into a private NSW-slot LDS ring and
//     waits for them with its own counted vmcnt: no workgroup barrier anywhere in the K loop, and the chain per
//     wave is a quarter as long;
//   * the four partial tiles are summed once through LDS at the end (fixed order 0..3: deterministic), into the
//     shared fp32 epilogue image (common.h EpiImg), and stored by img_store_rows: bias / activation / SwiGLU /
//     the QKV RoPE + KV-write epilogue, or fp32 split-K slabs [S][M][N] for the consumer (rope_cache / add_norm)
//     when the grid also splits K (grid.y).
// Rows past M and columns past N read as zero through the buffer descriptors' range check; a partial last
// k-step (K % 64 != 0) folds k into the voffset (the check covers voffset) and zeroes the A chunks past K in the
// owning wave's slot, as gemm_mid does.
#include "common.h"

namespace {

template <int MT, int BN, int NSW>
struct DecCfg {
  static constexpr int NW = 4;
  static constexpr int NT = BN / 16;
  static constexpr int AR = MT * 16;           // A rows staged per k-step
  static constexpr int AL = AR / 8, BL = BN / 8;  // 1-KiB LDS-DMA wave-instructions per k-step
  static constexpr int LOADS = AL + BL;
  static constexpr int SLOT = (AR + BN) * 128;
  static constexpr int RING = NW * NSW * SLOT;
  static constexpr int RED = NW * MT * NT * 1024;  // every wave's accumulators, 1 KiB per 16x16 tile
  static constexpr int IMG = AR * EpiImg<BN>::LDW * 4;
  static constexpr int LDS = RING > RED + IMG ? RING : RED + IMG;
  static constexpr bool FITS = LDS <= 160 * 1024;
};

template <int N_>
__device__ __forceinline__ void dec_wait(int younger_stages) {
  // s_waitcnt vmcnt(younger_stages * LOADS), younger_stages in [0, 3]
  if (younger_stages >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * N_) : "memory");
  else if (younger_stages == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * N_) : "memory");
  else if (younger_stages == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N_) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// In-launch split-K combine on the epilogue image (hint bit 256 with a grid split): every K slice of a column tile
// writes its fp32 image, row-major [AR][BN], write-through (sc1) into its slab of the tile's workspace region
// [tile][S][AR * BN]; every wave drains its stores, then one lane takes a ticket on the tile's counter (relaxed,
// agent scope: MI355X_MICROARCH "Valid forms" row 1, as common.h splitk_combine). The slice that draws S - 1 reads
// all S slabs back with sc1 loads and sums them in slice order 0..S-1 - the same sums whatever the arrival order -
// into its image, resets the counter, and returns true: it runs the epilogue. The others return false.
template <int BN, int AR>
__device__ __forceinline__ bool dec_combine(float* ct, float* ws, int* cnt, int tile, int S, int z, int* lds_word) {
  using Img = EpiImg<BN>;
  constexpr int V4 = AR * BN / 4;  // 16-B pieces of one slab
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(ws) + (int64_t)tile * S * AR * BN * 4,
                                                    (short)0, (int)((uint32_t)S * (uint32_t)(AR * BN * 4)), 0x00020000);
  const uint32_t slab_b = (uint32_t)(AR * BN * 4);
  for (int v = threadIdx.x; v < V4; v += blockDim.x) {
    const int r = v / (BN / 4), c = (v - r * (BN / 4)) * 4;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, Img::ld4(ct, r, c)), rs, (uint32_t)(v * 16),
                                           (uint32_t)z * slab_b, 16);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains before the ticket
  __syncthreads();
  if (threadIdx.x == 0) *lds_word = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  if (*lds_word != S - 1) return false;
  if (threadIdx.x == 0) __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no instruction: keeps the loads below the ticket
  for (int v = threadIdx.x; v < V4; v += blockDim.x) {
    const int r = v / (BN / 4), c = (v - r * (BN / 4)) * 4;
    f32x4 sum = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) {
      const f32x4 p = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)(v * 16),
                                                                                      (uint32_t)s * slab_b, 16));
#pragma unroll
      for (int i = 0; i < 4; ++i) sum[i] += p[i];
    }
    *reinterpret_cast<f32x4*>(ct + Img::at(r, c)) = sum;
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __syncthreads();
  return true;
}

}  // namespace

// MODE (bench/proto/dec_probe.hip only; the library instantiates 0): 1 = weight (B) loads only, 2 = activation (A)
// loads only, 3 = no loads (MFMAs on whatever LDS holds), 4 = no epilogue stores - to take a launch's time apart.
template <int MT, int BN, int NSW, int MODE = 0>
__global__ __launch_bounds__(256) void gemm_dec_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                       const bf16_t* __restrict__ B, int64_t ldb,
                                                       const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                       int64_t ldy, float* __restrict__ part, int M, int N, int K,
                                                       int act, int glu, QkvEpi qe, int* __restrict__ cnt) {
  using C = DecCfg<MT, BN, NSW>;
  static_assert(BN % 16 == 0 && C::BL >= 1, "BN: multiple of 16");
  static_assert(3 * C::LOADS <= 63, "vmcnt immediate");
  static_assert(C::FITS, "LDS");
  constexpr int NW = C::NW, NT = C::NT, AR = C::AR, AL = C::AL, BL = C::BL, LOADS = C::LOADS, SLOT = C::SLOT;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int ntn = (N + BN - 1) / BN;
  const TileWork tw = tile_work(1, ntn, AR, BN);
  const int n0 = tw.n0, zk = tw.z;

  const int nk_all = (K + 63) / 64;  // 128-byte k-steps
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int t0 = zk * per, t1 = min(nk_all, t0 + per);
  const int mine = t1 - t0 - w;
  const int nloc = mine > 0 ? (mine + NW - 1) / NW : 0;  // this wave's k-steps: t0 + w + NW j, j < nloc
  const bool ktail = (K & 63) != 0;

  const uint64_t abytes = (uint64_t)M * (uint64_t)lda * 2;
  const uint64_t bbytes = (uint64_t)(N - n0) * (uint64_t)ldb * 2;
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(reinterpret_cast<const char*>(A)), (short)0,
                                                    (int)(abytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)abytes),
                                                    0x00020000);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(reinterpret_cast<const char*>(B) + (int64_t)n0 * ldb * 2),
                                                    (short)0,
                                                    (int)(bbytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bbytes),
                                                    0x00020000);
  uint32_t va[AL], vb[BL];  // per-lane byte offsets (row, source-swizzled chunk), fixed over k
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = i * 8 + (lane >> 3);
    va[i] = (uint32_t)(row * lda * 2 + (((lane & 7) ^ (row & 7)) << 4));
  }
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = i * 8 + (lane >> 3);
    vb[i] = (uint32_t)(row * ldb * 2 + (((lane & 7) ^ (row & 7)) << 4));
  }
  char* ring = smem + w * (NSW * SLOT);

  // local k-step J_ of this wave into its ring slot J_ % NSW: AL + BL wave-instructions of 1 KiB (8 rows x 128 B).
  // A macro, not a lambda: hipcc's host pass of a kernel template that captures the buffer descriptors in a lambda
  // fails quietly and drops the launch stub (undefined __device_stub__ at load time), as gemm_mid.hip notes.
#define DEC_ISSUE(J_)                                                                                            \
  do {                                                                                                           \
    const int t_ = t0 + w + NW * (J_);                                                                           \
    char* sl_ = ring + ((J_) % NSW) * SLOT;                                                                      \
    const uint32_t so_ = (uint32_t)t_ * 128u;                                                                    \
    if (MODE == 3) {                                                                                             \
    } else if (!ktail || t_ != nk_all - 1) {                                                                     \
      if (MODE != 1) _Pragma("unroll") for (int i_ = 0; i_ < AL; ++i_)                                           \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)(sl_ + i_ * 1024), 16, (uint32_t)va[i_],      \
                                                 (uint32_t)so_, 0, 0);                                           \
      if (MODE != 2) _Pragma("unroll") for (int i_ = 0; i_ < BL; ++i_) /* weights: read once, non-temporal */    \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDS_AS void*)(sl_ + AR * 128 + i_ * 1024), 16,             \
                                                 (uint32_t)vb[i_], (uint32_t)so_, 0, 2);                          \
    } else { /* partial last k-step: k in the voffset, so the range check covers the last row's tail */         \
      _Pragma("unroll") for (int i_ = 0; i_ < AL; ++i_)                                                          \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)(sl_ + i_ * 1024), 16,                        \
                                                 (uint32_t)(va[i_] + so_), (uint32_t)0, 0, 0);                   \
      _Pragma("unroll") for (int i_ = 0; i_ < BL; ++i_)                                                          \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDS_AS void*)(sl_ + AR * 128 + i_ * 1024), 16,             \
                                                 (uint32_t)(vb[i_] + so_), (uint32_t)0, 0, 2);                   \
    }                                                                                                            \
  } while (0)

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment reads: row r = 16 t + li (r & 7 == li & 7), k-half s takes 16-B chunks 4 s + g
  const int x0 = (g ^ (li & 7)) << 4, x1 = ((4 + g) ^ (li & 7)) << 4;
  const int fa = li * 128, fb = AR * 128 + li * 128;

  const int pre = nloc < NSW ? nloc : NSW;
  for (int j = 0; j < pre; ++j) DEC_ISSUE(j);
  for (int j = 0; j < nloc; ++j) {
    const int younger = min(NSW - 1, nloc - 1 - j);
    if constexpr (MODE == 0 || MODE == 4) dec_wait<LOADS>(younger);  // this wave's stage j landed (only it reads it)
    else if constexpr (MODE == 1) dec_wait<BL>(younger);
    else if constexpr (MODE == 2) dec_wait<AL>(younger);
    const char* st = ring + (j % NSW) * SLOT;
    const int t = t0 + w + NW * j;
    if (ktail && t == nk_all - 1) {  // zero the A chunks past K (they hold the next row's values)
      const int kv = K - t * 64;     // valid k of this step, a multiple of 16
      char* sw = const_cast<char*>(st);
      for (int idx = lane; idx < AR * 8; idx += 64) {
        const int row = idx >> 3, c = idx & 7;
        if (c * 8 >= kv) *reinterpret_cast<u32x4*>(sw + row * 128 + ((c ^ (row & 7)) << 4)) = u32x4{0u, 0u, 0u, 0u};
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int xo = s ? x1 : x0;
      s16x8 a[MT], b[NT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) a[mt] = *reinterpret_cast<const s16x8*>(st + fa + mt * 2048 + xo);
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) b[nt] = *reinterpret_cast<const s16x8*>(st + fb + nt * 2048 + xo);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
    if (j + NSW < nloc) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's fragment reads are done
      DEC_ISSUE(j + NSW);
    }
  }

#undef DEC_ISSUE

  // ---- cross-wave sum: every wave's tiles to LDS (1 KiB per 16x16 tile, lane-major: conflict-free b128), then the
  // owner of tile q (q % NW == w) sums the four copies in wave order into the epilogue image
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // every wave is done with its ring
  asm volatile("" ::: "memory");
  f32x4* red = reinterpret_cast<f32x4*>(smem);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) red[((w * MT + mt) * NT + nt) * 64 + lane] = acc[mt][nt];
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  using Img = EpiImg<BN>;
  float* ct = reinterpret_cast<float*>(smem + C::RED);
#pragma unroll
  for (int q = 0; q < MT * NT; ++q) {
    if (q % NW != w) continue;
    const int mt = q / NT, nt = q % NT;
    f32x4 v = red[(mt * NT + nt) * 64 + lane];
#pragma unroll
    for (int u = 1; u < NW; ++u) {
      const f32x4 p = red[((u * MT + mt) * NT + nt) * 64 + lane];
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] += p[i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) ct[Img::at(mt * 16 + 4 * g + i, nt * 16 + li)] = v[i];
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  if constexpr (MODE == 4) {
    if (M < 0) part[threadIdx.x] = ct[threadIdx.x];  // keep the sums live without storing them
    return;
  }
  if (cnt) {  // split-K combined in this launch: the tile's last arriving K slice sums every slice and stores
    if (!dec_combine<BN, AR>(ct, part, cnt, n0 / BN, gridDim.y, zk, reinterpret_cast<int*>(smem))) return;
    part = nullptr;
  }
  img_store_rows<BN, 64 * NW, AR>(ct, AR, 0, 0, n0, M, N, part ? part + (int64_t)zk * M * N : nullptr, Y, ldy, bias,
                                  act, glu, qe);
}

// NS stages if they fit the LDS, else the deepest ring that does (dec_depth picks the same at run time)
template <int MT, int BN, int NS>
static void dec_launch(dim3 grid, hipStream_t st, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw,
                       const bf16_t* bias, bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act, int glu,
                       const QkvEpi& qv, int* cnt) {
  if constexpr (NS > 2 && !DecCfg<MT, BN, NS>::FITS) {
    dec_launch<MT, BN, NS - 1>(grid, st, X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, qv, cnt);
  } else {
    gemm_dec_kernel<MT, BN, NS><<<grid, 256, 0, st>>>(X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, qv, cnt);
  }
}

// BN code (hint tile bits): 1 = 16, 2 = 32, 3 = 48, 4 = 64, 5 = 96 columns per workgroup
bool gemm_dec_bn(int code, int* bn) {
  static constexpr int kBN[6] = {0, 16, 32, 48, 64, 96};
  if (code < 1 || code > 5) return false;
  *bn = kBN[code];
  return true;
}

// ring depth actually used: the deepest <= want (2..4) whose rings fit the 160 KiB LDS
static int dec_depth(int mt, int bn, int want) {
  int ns = std::max(2, std::min(want, 4));
  const int slot = (mt * 16 + bn) * 128;
  while (ns > 2 && 4 * ns * slot > 160 * 1024) --ns;
  return ns;
}

// cnt != nullptr: split-K combined in the launch (dec_combine; `part` = the workspace holding [tile][split][64 * bn]
// fp32 slabs, sized by the caller), finished output in Y with act / glu / the QKV epilogue
void launch_gemm_dec(int code, int depth, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw,
                     const bf16_t* bias, bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act, int glu,
                     int split, hipStream_t st, const QkvEpi* qe, int* cnt) {
  int bn;
  if (!gemm_dec_bn(code, &bn)) throw std::runtime_error("gemm_dec: bad tile code");
  if (M < 1 || M > 64) throw std::runtime_error("gemm_dec: M must be 1..64");
  if (glu && (bn % 32)) throw std::runtime_error("gemm_dec: SwiGLU needs 32-column tile pairs");
  if ((uint64_t)64 * ldx * 2 >= (1ull << 31) || (uint64_t)bn * ldw * 2 >= (1ull << 31))
    throw std::runtime_error("gemm_dec: row stride too large for 32-bit buffer offsets");
  const int mt = M <= 16 ? 1 : (M <= 32 ? 2 : 4);
  const int ns = dec_depth(mt, bn, depth);
  const QkvEpi qv = qe ? *qe : QkvEpi{};
  dim3 grid((N + bn - 1) / bn, split);
#define DECN(MT_, BN_)                                                                                           \
  do {                                                                                                           \
    if (ns >= 4) dec_launch<MT_, BN_, 4>(grid, st, X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, qv, cnt);   \
    else if (ns == 3) dec_launch<MT_, BN_, 3>(grid, st, X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, qv, cnt); \
    else dec_launch<MT_, BN_, 2>(grid, st, X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, qv, cnt);          \
  } while (0)
#define DECB(MT_)                                                                                                \
  do {                                                                                                           \
    switch (bn) {                                                                                                \
      case 16: DECN(MT_, 16); break;                                                                             \
      case 32: DECN(MT_, 32); break;                                                                             \
      case 48: DECN(MT_, 48); break;                                                                             \
      case 64: DECN(MT_, 64); break;                                                                             \
      default: DECN(MT_, 96); break;                                                                             \
    }                                                                                                            \
  } while (0)
  if (mt == 1) DECB(1);
  else if (mt == 2) DECB(2);
  else DECB(4);
#undef DECB
#undef DECN
  HIP_CHECK_LAUNCH();
}
