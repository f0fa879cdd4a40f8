// Mid-M MFMA GEMM (tensor-parallel decode at M = 64-512 rows, mid-size prefill chunks):
//   Y[M, N] = epilogue(X[M, K] . W[N, K]^T), bf16 in, fp32 accumulate; split-K over grid.y into fp32
//   slabs that the next kernel (rope / add_norm / splitk_reduce) sums.
//
// Why a separate kernel from gemm_tiled (gemm.hip): rocprofv3 on the TP=8 QKV shape (M=512, N=1536,
// K=4096; profiles/r2_gemm_pmc) showed the tiled kernels issue 7-8 VALU instructions per MFMA -
// per-k-step 64-bit address math for every global_load_lds (row clamp, swizzle, K clamp) and
// per-fragment LDS addresses - and spend 38-48 % of wave cycles waiting: ~10 % MFMA utilisation.
// Here every operand load is a buffer_load ... lds through a wave-uniform buffer descriptor:
//   * the per-lane part (row * ld + swizzled 16-B chunk) is a 32-bit voffset computed ONCE;
//   * the k position is the scalar soffset (+128 B per k-step: SALU, not VALU);
//   * rows past M / N fall outside the descriptor's num_records and read as zero (hardware bounds
//     check) - no clamps in the loop; the partial last k-step (K % 64 != 0) moves k into the voffset
//     so the last row's tail is range checked too (the check covers voffset, not soffset);
// and each wave's LDS fragment addresses are one base register per k-half plus immediate offsets
// (the XOR swizzle term depends only on lane & 7 because fragment rows step by 16).
// Tiles are larger per wave (32-64 MFMAs per k-step) so the fixed per-step cost (barrier, counted
// vmcnt wait, staging issue) is amortised. Ring of NS stages, stage t+NS-1 issued while t computes.
#include "common.h"

// The buffer descriptor is built and used only inside the kernel body, and every offset argument of
// the buffer builtins is cast to uint32_t explicitly: otherwise the host compilation pass of this
// template fails overload resolution quietly and hipcc drops the kernel's launch stub (undefined
// __device_stub__ at link time, no diagnostic).
// F8 (W8A8, csrc/gemm.hip launch_gemm_f8f8 tiles 8-13): A and B are fp8-e4m3 bytes (lda / ldb / K in bytes, K %
// 128 == 0). A 128-byte k-step of fp8 has the byte layout of the 64-element bf16 one, so the staging, ring and
// LDS image are shared; each (m, n) tile takes one MX-fp8 16x16x128 MFMA per k-step (the lane's 16-B chunks 2g
// and 2g+1), and the per-token x per-channel scales xs[m] * ws[n] are applied to the accumulators before the
// epilogue (or the split-K slabs / combine, which are linear in them).
// MODE (bench/proto/midm_probe.hip only; the library instantiates 0): 1 = loads without MFMAs, 2 = MFMAs on
// whatever LDS holds without loads, 3 = no epilogue stores - to take a tile's time apart.
// ILV (bf16 row-major, >= 3 stages, K % 64 == 0; hint bit 512 of launch_gemm, chosen by the autotuner): the
// k-steps overlap their LDS traffic with the MFMAs instead of running reads -> MFMAs per k-half behind a
// barrier - the second k-half's fragment reads are issued between the first k-half's MFMAs, and the next
// k-step's first-half reads plus the ring stage issue between the second k-half's MFMAs (one barrier per
// k-step, moved to the middle of it; the stage issue moves half a k-step later). For M >= 128 tiles, where a
// k-step carries 16-64 MFMAs per wave and the MFMA-only time is 60-80 % of the kernel (profiles/r4_gemm).
// MXA (W8A8 with MX A-scales, csrc/gemm.hip launch_gemm_f8f8 `asc`): the fp8 activations carry one e8m0 scale per
// row and 32-element block (OCP MX; asc [M][K / 32] bytes, written by a SwiGLU epilogue, img_store_rows) instead of
// one fp32 scale per row. Each ring stage also stages the tile's 4 scale bytes per row of that k-step (one 4-byte
// LDS-DMA piece per wave: its BM / NW rows); lane group g passes the byte of block g to the MX-fp8 MFMA.
template <int BM, int BN, int WM, int WN, int NS, bool WNT, bool F8 = false, int MODE = 0, bool ILV = false,
          bool MXA = false>
__global__ __launch_bounds__(64 * WM * WN) void gemm_mid_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                              const bf16_t* __restrict__ B, int64_t ldb,
                                                              const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                              int64_t ldy, float* __restrict__ part, int M, int N, int K,
                                                              int act, int glu, int* __restrict__ cnt, QkvEpi qe,
                                                              const float* __restrict__ xs,
                                                              const float* __restrict__ wsc,
                                                              const unsigned char* __restrict__ asc) {
  constexpr int ES = F8 ? 1 : 2;  // operand bytes per element
  constexpr int NW = WM * WN;
  constexpr int MT = BM / WM / 16, NT = BN / WN / 16;  // 16x16 accumulator tiles per wave
  constexpr int RW = BM / NW;                          // MXA: rows whose scale bytes one wave stages
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, SC_BYTES = MXA ? NW * 256 : 0;
  constexpr int STAGE = A_BYTES + B_BYTES + SC_BYTES;
  constexpr int AL = BM / (8 * NW), BL = BN / (8 * NW);  // 1-KiB buffer_load_lds per wave per stage
  constexpr int LOADS = AL + BL + (MXA ? 1 : 0);
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "tile rows must split evenly over the waves");
  static_assert(MT >= 1 && NT >= 1, "per-wave tile");
  static_assert(!MXA || (F8 && RW <= 64), "MX A-scales: fp8 operands, <= 64 rows per wave");
  __shared__ __attribute__((aligned(16))) char smem[NS * STAGE];

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wm = w / WN, wn = w % WN;
  const int ntn = (N + BN - 1) / BN, ntm = (M + BM - 1) / BM;
  const TileWork tw = tile_work(ntm, ntn, BM, BN);
  const int m0 = tw.m0, n0 = tw.n0, zk = tw.z;

  const int nk_all = (K * ES + 127) / 128;  // 128-byte k-steps
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int t0 = zk * per, t1 = min(nk_all, t0 + per);

  // descriptors start at this tile's first row; everything past the matrix end reads as zero
  const uint64_t abytes = (uint64_t)(M - m0) * (uint64_t)lda * ES;
  const uint64_t bbytes = (uint64_t)(N - n0) * (uint64_t)ldb * ES;
  const int64_t boff = (int64_t)n0 * ldb * ES;  // bytes
  const auto ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(reinterpret_cast<const char*>(A) + (int64_t)m0 * lda * ES), (short)0,
      (int)(abytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)abytes), 0x00020000);
  const auto rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(reinterpret_cast<const char*>(B) + boff),
                                                    (short)0,
                                                    (int)(bbytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bbytes),
                                                    0x00020000);
  // MXA: scale bytes of rows m0.. (K / 32 per row); lanes past RW read out of range (zeros into unused LDS)
  const int kblk = K / 32;
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned char*>(asc) + (int64_t)m0 * kblk, (short)0,
                                                    (int)((uint32_t)(M - m0) * (uint32_t)kblk), 0x00020000);
  const uint32_t vsc = lane < RW ? (uint32_t)((w * RW + lane) * kblk) : 0x80000000u;
  uint32_t va[AL], vb[BL];  // per-lane byte offsets (row, source-swizzled chunk), fixed over k
#pragma unroll
  for (int i = 0; i < AL; ++i) {
    const int row = (i * NW + w) * 8 + (lane >> 3);
    va[i] = (uint32_t)(row * lda * ES + (((lane & 7) ^ (row & 7)) << 4));
  }
#pragma unroll
  for (int i = 0; i < BL; ++i) {
    const int row = (i * NW + w) * 8 + (lane >> 3);
    vb[i] = (uint32_t)(row * ldb * ES + (((lane & 7) ^ (row & 7)) << 4));
  }
  // one ring stage (k-step T_) into LDS slot SA_: AL + BL wave-instructions of 1 KiB (8 rows x 128 B);
  // the k position is the scalar soffset, the per-lane voffsets never change
#define MID_STAGE(T_, SA_)                                                                                         \
  do {                                                                                                           \
    char* sA_ = (SA_);                                                                                           \
    if (MODE == 2) break;                                                                                        \
    const int soff_ = (T_) * 128, sofb_ = soff_;                                                                  \
    if (!ktail || (T_) != nk_all - 1) {                                                                          \
      _Pragma("unroll") for (int i_ = 0; i_ < AL; ++i_)                                                           \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)(sA_ + (i_ * NW + w) * 1024), 16, (uint32_t)va[i_], (uint32_t)soff_, 0, 0); \
      _Pragma("unroll") for (int i_ = 0; i_ < BL; ++i_)                                                           \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDS_AS void*)(sA_ + A_BYTES + (i_ * NW + w) * 1024), 16, (uint32_t)vb[i_], \
                                                 (uint32_t)sofb_, 0, WNT ? 2 : 0); /* weights: read once per step, nt */ \
      if constexpr (MXA)                                                                                          \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)(sA_ + A_BYTES + B_BYTES + w * 256), 4, vsc,    \
                                                 (uint32_t)((T_) * 4), 0, 0);                                     \
    } else { /* partial last k-step: k folded into the voffset, so the range check covers the row tail */     \
      _Pragma("unroll") for (int i_ = 0; i_ < AL; ++i_)                                                           \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)(sA_ + (i_ * NW + w) * 1024), 16, (uint32_t)(va[i_] + soff_), (uint32_t)0, 0, 0); \
      _Pragma("unroll") for (int i_ = 0; i_ < BL; ++i_)                                                           \
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDS_AS void*)(sA_ + A_BYTES + (i_ * NW + w) * 1024), 16, (uint32_t)(vb[i_] + sofb_), \
                                                 (uint32_t)0, 0, WNT ? 2 : 0);                                  \
    }                                                                                                            \
  } while (0)

  f32x4 acc[MT][NT];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int b = 0; b < NT; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment addresses: row r = base + 16 t (t = tile), chunk c = 4 s + g -> (c ^ (li & 7)) << 4
  const int arow = wm * (MT * 16) + li, brow = wn * (NT * 16) + li;
  const int x0 = ((g) ^ (li & 7)) << 4, x1 = ((4 + g) ^ (li & 7)) << 4;
  const int aoff0 = arow * 128 + x0, aoff1 = arow * 128 + x1;
  const int boff0 = A_BYTES + brow * 128 + x0, boff1 = A_BYTES + brow * 128 + x1;

  // ONE copy of the MFMA body (a second, masked copy made hipcc shuffle every accumulator between
  // AGPRs and VGPRs each k-step); the K tail is zeroed in LDS instead (below)
  // fp8: each lane feeds the 16x16x128 MFMA 32 k-bytes of its fragment row. It takes the 16-B chunks g and
  // g + 4 (the bf16 read pattern, conflict-free on the swizzled image) instead of 2g, 2g + 1 (PMC: 48 % of the
  // LDS cycles were bank conflicts). A and B use the same k permutation, so the dot products are unchanged.
  const int y0 = x0, y1 = x1;
  // MXA: the scale word (4 blocks) of tile row r in a stage, and the byte of block g of it: the MFMA takes the scale
  // of k-block b (k [32b, 32b + 32) of the step) from lane group b, and its k order - lane group g's first 16 bytes
  // are k [16g, 16g + 16), its last 16 are k [64 + 16g, ...) - is exactly the chunk g / g + 4 reads above
  // (bench/proto/mx_scale_probe.hip, scripts/mx_debug.py: a per-lane contiguous-block order scaled the wrong data)
  auto mx_scale = [&](const char* st, int r) -> int {
    return (int)(*reinterpret_cast<const uint32_t*>(st + A_BYTES + B_BYTES + (r / RW) * 256 + (r % RW) * 4) >> (8 * g));
  };
  auto compute = [&](const char* st) {
    if constexpr (MODE == 1) return;
    if constexpr (F8) {
      typedef int __attribute__((ext_vector_type(8))) i32x8_t;
      i32x8_t a[MT], b[NT];
      int sa[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) sa[t] = MXA ? mx_scale(st, arow + t * 16) : 127;
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const u32x4 lo = *reinterpret_cast<const u32x4*>(st + arow * 128 + t * 2048 + y0);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(st + arow * 128 + t * 2048 + y1);
        a[t] = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const u32x4 lo = *reinterpret_cast<const u32x4*>(st + A_BYTES + brow * 128 + t * 2048 + y0);
        const u32x4 hi = *reinterpret_cast<const u32x4*>(st + A_BYTES + brow * 128 + t * 2048 + y1);
        b[t] = i32x8_t{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[mt], b[nt], acc[mt][nt], 0, 0, 0, sa[mt], 0, 127);
      return;
    }
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int ao = s ? aoff1 : aoff0, bo = s ? boff1 : boff0;
      s16x8 a[MT], b[NT];
#pragma unroll
      for (int t = 0; t < MT; ++t) a[t] = *reinterpret_cast<const s16x8*>(st + ao + t * 2048);
#pragma unroll
      for (int t = 0; t < NT; ++t) b[t] = *reinterpret_cast<const s16x8*>(st + bo + t * 2048);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[mt], b[nt], acc[mt][nt], 0, 0, 0);
    }
  };

  const bool ktail = ((K * ES) & 127) != 0;  // bf16 only: fp8 calls have K % 128 == 0 (host-checked)
#pragma unroll
  for (int j = 0; j < NS - 1; ++j)
    if (t0 + j < t1) MID_STAGE(t0 + j, smem + j * STAGE);
  // wait until at most `younger` (clamped to NS - 2) stages of LOADS loads are still in flight
  auto ring_wait = [&](int younger) {
    if (NS >= 6 && younger >= 4) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * LOADS) : "memory");
    else if (NS >= 5 && younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * LOADS) : "memory");
    else if (NS >= 4 && younger >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * LOADS) : "memory");
    else if (NS >= 3 && younger >= 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(LOADS) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // load l (< LOADS) of a ring stage: A rows first, then B rows (the interleaved rings issue a stage piecewise)
#define MID_LOAD1(L_, T_, SA_)                                                                                   \
  do {                                                                                                           \
    const int so_ = (T_) * 128;                                                                                  \
    if ((L_) < AL)                                                                                               \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (LDS_AS void*)((SA_) + ((L_) * NW + w) * 1024), 16,            \
                                               (uint32_t)va[(L_) < AL ? (L_) : 0], (uint32_t)so_, 0, 0);         \
    else if (MXA && (L_) == AL + BL)                                                                             \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (LDS_AS void*)((SA_) + A_BYTES + B_BYTES + w * 256), 4, vsc,    \
                                               (uint32_t)((T_) * 4), 0, 0);                                      \
    else                                                                                                         \
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (LDS_AS void*)((SA_) + A_BYTES + ((L_) - AL) * NW * 1024 + w * 1024), \
                                               16, (uint32_t)vb[(L_) < AL ? 0 : (L_) - AL], (uint32_t)so_, 0,    \
                                               WNT ? 2 : 0);                                                     \
  } while (0)
  if constexpr (ILV && F8) {
    // fp8 software pipeline: a k-step is ONE 16x16x128 MFMA per (mt, nt), so it cannot be halved as in the bf16
    // ring below. Instead k-step t+1's fragments are read into the other register set between k-step t's MFMAs,
    // and ring stage t+NS-1 is issued among them. One barrier per k-step, at its start, once this wave's copy of
    // stage t+1 landed: every wave is then past its reads of stage t-1 (done in step t-2), whose slot takes stage
    // t+NS-1. The ring keeps NS-2 stages in flight ahead of the reads (NS-1 in the plain loop).
    static_assert(NS >= 3 && MODE == 0, "fp8 interleaved ring: >= 3 stages");
    static_assert((NS - 3) * LOADS <= 63, "vmcnt immediate");
    constexpr int NR = 2 * (MT + NT);        // ds_read_b128 per k-step: lo / hi chunk of every A and B tile
    constexpr int RPG = (NR + MT - 1) / MT;  // fragment reads per group of NT MFMAs
    constexpr int LPG = (LOADS + MT - 1) / MT;
    typedef int __attribute__((ext_vector_type(8))) i32x8_t;
    u32x4 fr[2][NR];  // [register set][read]: A tile q -> 2q (lo), 2q + 1 (hi); B tile q -> 2 (MT + q) (+1)
#define F8_RD(SET_, R_, SN_)                                                                                     \
  fr[SET_][R_] = *reinterpret_cast<const u32x4*>(                                                                \
      (SN_) + ((R_) / 2 < MT ? arow * 128 + ((R_) / 2) * 2048 : A_BYTES + brow * 128 + ((R_) / 2 - MT) * 2048) + \
      (((R_) & 1) ? y1 : y0))
#define F8_OP(SET_, Q_)                                                                                          \
  __builtin_bit_cast(i32x8_t, __builtin_shufflevector(fr[SET_][2 * (Q_)], fr[SET_][2 * (Q_) + 1], 0, 1, 2, 3, 4, 5, 6, 7))
    // k-step t on register set P_: MFMAs interleaved with (ISSUE_) stage t+NS-1's loads and (NEXT_) stage t+1's
    // fragment reads into set P_ ^ 1
#define F8_STEP(P_, ISSUE_, NEXT_)                                                                               \
  do {                                                                                                           \
    const int nx_ = cur == NS - 1 ? 0 : cur + 1;                                                                 \
    const char* sn_ = smem + nx_ * STAGE;                                                                        \
    char* sl_ = smem + (cur == 0 ? NS - 1 : cur - 1) * STAGE;                                                    \
    if (NEXT_) {                                                                                                 \
      ring_wait(min(t1 - 2 - t, NS - 3)); /* this wave's copy of stage t+1 landed ... */                         \
      __builtin_amdgcn_s_barrier();       /* ... every wave's; every wave is past step t-1 */                    \
      asm volatile("" ::: "memory");                                                                             \
    }                                                                                                            \
    int sa_[MT];                                                                                                 \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) sa_[mt] = MXA ? mx_scale(smem + cur * STAGE, arow + mt * 16) : 127; \
    _Pragma("unroll") for (int mt = 0; mt < MT; ++mt) {                                                          \
      if (ISSUE_) {                                                                                              \
        _Pragma("unroll") for (int l = mt * LPG; l < (mt + 1) * LPG && l < LOADS; ++l) MID_LOAD1(l, t + NS - 1, sl_); \
      }                                                                                                          \
      if (NEXT_) {                                                                                               \
        _Pragma("unroll") for (int r = mt * RPG; r < (mt + 1) * RPG && r < NR; ++r) F8_RD((P_) ^ 1, r, sn_);     \
      }                                                                                                          \
      const i32x8_t a_ = F8_OP(P_, mt);                                                                          \
      _Pragma("unroll") for (int nt = 0; nt < NT; ++nt) acc[mt][nt] =                                            \
          __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a_, F8_OP(P_, MT + nt), acc[mt][nt], 0, 0, 0, sa_[mt], 0, 127); \
      __builtin_amdgcn_sched_barrier(0);                                                                         \
    }                                                                                                            \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): the next step's fragments are in registers */             \
    cur = nx_;                                                                                                   \
    ++t;                                                                                                         \
  } while (0)
    int cur = 0, t = t0;
    ring_wait(min(t1 - 1 - t0, NS - 2));  // stage t0 landed ...
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... for every wave
    asm volatile("" ::: "memory");
#pragma unroll
    for (int r = 0; r < NR; ++r) F8_RD(0, r, smem);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    int par = 0;  // register set holding the current step's fragments
    // steady state, unrolled over the two register sets: every step issues a stage and reads the next one
    while (true) {
      if (t + NS - 1 >= t1) break;
      F8_STEP(0, true, true);
      if (t + NS - 1 >= t1) { par = 1; break; }
      F8_STEP(1, true, true);
    }
    // the last (<= NS - 1) k-steps: nothing left to stage
    while (t < t1) {
      if (par == 0) F8_STEP(0, false, t + 1 < t1);
      else F8_STEP(1, false, t + 1 < t1);
      par ^= 1;
    }
#undef F8_STEP
#undef F8_OP
#undef F8_RD
  } else if constexpr (ILV) {
    static_assert(NS >= 3 && MODE == 0, "interleaved ring: bf16 row-major weights, >= 3 stages");
    static_assert((NS - 3) * LOADS <= 63, "vmcnt immediate");
    constexpr int RPG = (MT + NT + MT - 1) / MT;  // fragment reads per group of NT MFMAs
    constexpr int LPG = (LOADS + MT - 1) / MT;    // ring loads per group
    // s_waitcnt vmcnt((NS - 3) * LOADS) lgkmcnt(0) through the builtin (the wait-count pass sees it): stage t+1
    // landed with stages up to t+NS-2 in flight, and this wave's fragment reads are done
    constexpr int VN = (NS - 3) * LOADS;
    constexpr int WAIT_MID = (VN & 15) | (7 << 4) | ((VN >> 4) << 14);
    s16x8 a0[MT], b0[NT], a1[MT], b1[NT];
    ring_wait(min(t1 - 1 - t0, NS - 2));  // stage t0 landed ...
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // ... for every wave
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < MT; ++i) a0[i] = *reinterpret_cast<const s16x8*>(smem + aoff0 + i * 2048);
#pragma unroll
    for (int i = 0; i < NT; ++i) b0[i] = *reinterpret_cast<const s16x8*>(smem + boff0 + i * 2048);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    int cur = 0, t = t0;
    // steady state: every k-step issues a stage and reads the next k-step's fragments (one basic block, so
    // the group barriers can interleave loads, reads and MFMAs)
    // program order pinned per group (sched_barrier): the ring loads set M0 one after another, which the group
    // barriers alone do not spread
    for (; t + NS - 1 < t1; ++t) {
      const char* st = smem + cur * STAGE;
      const int nx = cur == NS - 1 ? 0 : cur + 1;
      const char* sn = smem + nx * STAGE;
      char* sl = smem + (cur == 0 ? NS - 1 : cur - 1) * STAGE;  // stage t-1's slot: receives stage t+NS-1
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {  // first k-half MFMAs, second-half fragment reads between them
#pragma unroll
        for (int r = mt * RPG; r < (mt + 1) * RPG && r < MT + NT; ++r) {
          if (r < MT) a1[r < MT ? r : 0] = *reinterpret_cast<const s16x8*>(st + aoff1 + (r < MT ? r : 0) * 2048);
          else b1[r < MT ? 0 : r - MT] = *reinterpret_cast<const s16x8*>(st + boff1 + (r < MT ? 0 : r - MT) * 2048);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[mt], b0[nt], acc[mt][nt], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_waitcnt(WAIT_MID);
      __builtin_amdgcn_s_barrier();  // stage t+1 visible; every wave is past its reads of stage t-1
      asm volatile("" ::: "memory");
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {  // second k-half MFMAs; the ring loads and next-step reads between them
#pragma unroll
        for (int l = mt * LPG; l < (mt + 1) * LPG && l < LOADS; ++l) MID_LOAD1(l, t + NS - 1, sl);
#pragma unroll
        for (int r = mt * RPG; r < (mt + 1) * RPG && r < MT + NT; ++r) {
          if (r < MT) a0[r < MT ? r : 0] = *reinterpret_cast<const s16x8*>(sn + aoff0 + (r < MT ? r : 0) * 2048);
          else b0[r < MT ? 0 : r - MT] = *reinterpret_cast<const s16x8*>(sn + boff0 + (r < MT ? 0 : r - MT) * 2048);
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[mt], b1[nt], acc[mt][nt], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);  // the next k-step's first-half fragments are in registers
      cur = nx;
    }
    // the last NS - 1 k-steps: nothing left to stage
    for (; t < t1; ++t) {
      const char* st = smem + cur * STAGE;
      const int nx = cur == NS - 1 ? 0 : cur + 1;
      const char* sn = smem + nx * STAGE;
#pragma unroll
      for (int i = 0; i < MT; ++i) a1[i] = *reinterpret_cast<const s16x8*>(st + aoff1 + i * 2048);
#pragma unroll
      for (int i = 0; i < NT; ++i) b1[i] = *reinterpret_cast<const s16x8*>(st + boff1 + i * 2048);
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0[mt], b0[nt], acc[mt][nt], 0, 0, 0);
      if (t + 1 < t1) {
        ring_wait(t1 - 2 - t);  // stage t+1 landed ...
        __builtin_amdgcn_s_waitcnt(0xC07F);
        __builtin_amdgcn_s_barrier();  // ... for every wave
        asm volatile("" ::: "memory");
#pragma unroll
        for (int i = 0; i < MT; ++i) a0[i] = *reinterpret_cast<const s16x8*>(sn + aoff0 + i * 2048);
#pragma unroll
        for (int i = 0; i < NT; ++i) b0[i] = *reinterpret_cast<const s16x8*>(sn + boff0 + i * 2048);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1[mt], b1[nt], acc[mt][nt], 0, 0, 0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
      cur = nx;
    }
#undef MID_LOAD1
  } else {
  int cur = 0;
  for (int t = t0; t < t1; ++t) {
    // stage t landed for this wave (younger stages stay in flight), then for every wave
    // stages t+1 .. t+NS-2 may still be in flight: LOADS wave-instructions each
    static_assert((NS - 2) * LOADS <= 63, "vmcnt immediate");
    ring_wait(min(t1 - 1 - t, NS - 2));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // raw barrier: in-flight loads survive it
    asm volatile("" ::: "memory");
    const int nxt = cur == 0 ? NS - 1 : cur - 1;  // (cur + NS - 1) % NS: freed by compute(t - 1)
    if (t + NS - 1 < t1) MID_STAGE(t + NS - 1, smem + nxt * STAGE);
    char* st = smem + cur * STAGE;
    if (ktail && t == nk_all - 1) {
      // last, partial k-step (wave-uniform branch, once per kernel): the A chunks past K hold the next
      // row's values - zero them so the B side's next-row bytes multiply by 0; nothing is in flight now
      const int kv = K - t * 64;  // valid k of this step, a multiple of 16
      for (int idx = threadIdx.x; idx < BM * 8; idx += 64 * NW) {
        const int row = idx >> 3, c = idx & 7;
        if (c * 8 >= kv) *reinterpret_cast<u32x4*>(st + row * 128 + ((c ^ (row & 7)) << 4)) = u32x4{0u, 0u, 0u, 0u};
      }
      __syncthreads();
    }
    compute(st);
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  }

#undef MID_STAGE
  if constexpr (MODE == 3) {  // keep the accumulators live without storing them
    float t = 0.f;
#pragma unroll
    for (int a = 0; a < MT; ++a)
#pragma unroll
      for (int b = 0; b < NT; ++b) t += acc[a][b][0] + acc[a][b][3];
    if (M < 0) part[threadIdx.x] = t;
    return;
  }
  if constexpr (F8) {  // per-token x per-channel scales (C layout: row 4g + i of tile mt, column li of tile nt)
    float wsv[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const int n = n0 + wn * (NT * 16) + nt * 16 + li;
      wsv[nt] = n < N ? wsc[n] : 0.f;
    }
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int m = m0 + wm * (MT * 16) + mt * 16 + 4 * g + i;
        const float sx = m < M ? (MXA ? 1.f : xs[m]) : 0.f;  // MX scales were applied in the MFMA
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt][i] *= sx * wsv[nt];
      }
  }
  if (cnt) {  // split-K slices combine in this launch; the tile's last arriver runs the epilogue
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (!splitk_combine<MT, NT>(acc, part, cnt, (n0 / BN) * ntm + m0 / BM, gridDim.y, zk, w, NW, lane,
                                reinterpret_cast<int*>(smem)))
      return;
    part = nullptr;
  }
  // epilogue through LDS (row-contiguous 16-B stores); every stage has landed (vmcnt(0) in the last
  // step) and tile_store_lds waits for this wave's last fragment reads before its first barrier
  tile_store_lds<BM, BN, MT, NT, 64 * NW, NS * STAGE>(acc, smem, wm * (MT * 16), wn * (NT * 16), m0, n0, M, N,
                                                        part ? part + (int64_t)zk * M * N : nullptr, Y, ldy, bias,
                                                        act, glu, qe);
}

// tsel 8: 128x128 (2x2 waves), 9: 256x128 (4x2), 10: 64x256 (1x4), 11: 64x128 (1x4), 12: 128x256 (2x4),
// 13: 64x192 (2x2; a 12288-column QKV is 64 tiles, 4096 columns 22: one workgroup per CU without a K split),
// 14: 64x32 (4x1; narrow projections without a K split: GPT-2-XL's 6400-column MLP up is 200 workgroups),
// 15: 64x96 (4x1; Llama-2-7B's 22016-column gate/up is 230 workgroups: one wave of the chip, no K split),
// 7: 64x48 (2x1 waves: 48 rows do not split over 4 waves in 8-row staging pieces; a 12288-column QKV is
//    exactly 256 workgroups without a K split)
static bool mid_layout(int tsel, int* bm, int* bn, int* wm, int* wn) {
  switch (tsel) {
    case 8: *bm = 128; *bn = 128; *wm = 2; *wn = 2; return true;
    case 9: *bm = 256; *bn = 128; *wm = 4; *wn = 2; return true;
    case 10: *bm = 64; *bn = 256; *wm = 1; *wn = 4; return true;
    case 11: *bm = 64; *bn = 128; *wm = 1; *wn = 4; return true;
    case 12: *bm = 128; *bn = 256; *wm = 2; *wn = 4; return true;
    case 13: *bm = 64; *bn = 192; *wm = 2; *wn = 2; return true;
    case 14: *bm = 64; *bn = 32; *wm = 4; *wn = 1; return true;
    case 15: *bm = 64; *bn = 96; *wm = 4; *wn = 1; return true;
    case 7: *bm = 64; *bn = 48; *wm = 2; *wn = 1; return true;
    default: return false;
  }
}
bool gemm_mid_dims(int tsel, int* bm, int* bn, int* threads) {
  int wm, wn;
  if (!mid_layout(tsel, bm, bn, &wm, &wn)) return false;
  *threads = 64 * wm * wn;
  return true;
}

// ring depth of a tile's MXA instantiation: the MX scale piece (NW x 256 B per stage) can push the deepest ring of a
// tile past the LDS; the host never launches those depths (mid_depth below), so they instantiate one stage less
template <int BM, int BN, int NW, int NS>
constexpr int mx_ns() {
  return NS * ((BM + BN) * 128 + NW * 256) <= 160 * 1024 ? NS : NS - 1;
}

// largest ring depth <= want that fits the 160 KiB LDS (extra: bytes per stage beyond the operand rows)
static int mid_depth(int bm, int bn, int want, int extra = 0) {
  const int stage = (bm + bn) * 128 + extra;
  int ns = std::max(2, std::min(want, 6));  // 6: the deepest ring (64x128 at 144 KiB)
  while (ns > 2 && ns * stage > 160 * 1024) --ns;
  return ns;
}

void launch_gemm_mid(int tsel, int depth, bool wnt, const bf16_t* X, int64_t ldx, const bf16_t* W, int64_t ldw,
                     const bf16_t* bias, bf16_t* Y, int64_t ldy, float* part, int M, int N, int K, int act, int glu,
                     int split, hipStream_t st, int* cnt, const QkvEpi* qe, const float* xs,
                     const float* wsc, bool ilv, const unsigned char* asc) {
  const bool f8 = xs != nullptr || asc != nullptr;
  if (f8 && (!wsc || K % 128)) throw std::runtime_error("gemm_mid fp8: per-row weight scales, K % 128 == 0");
  if (xs && asc) throw std::runtime_error("gemm_mid fp8: per-row activation scales or MX scales, not both");
  const QkvEpi qv = qe ? *qe : QkvEpi{};
  int bm, bn, wm, wn;
  if (!mid_layout(tsel, &bm, &bn, &wm, &wn)) throw std::runtime_error("gemm_mid: bad tile code");
  if (glu && (bn / wn / 16) % 2)
    throw std::runtime_error("gemm_mid: SwiGLU needs an even number of 16-column tiles per wave");
  if ((uint64_t)bm * ldx * 2 >= (1ull << 31) || (uint64_t)bn * ldw * 2 >= (1ull << 31))
    throw std::runtime_error("gemm_mid: row stride too large for 32-bit buffer offsets");
  const int ns = mid_depth(bm, bn, depth, asc ? wm * wn * 256 : 0);
  // the interleaved rings' preconditions; the fp8 one holds two fragment sets, which 8-wave tiles (256 VGPRs per
  // lane at two waves per SIMD) spill to scratch: 5-8x slower (profiles/r6_f8)
  ilv = ilv && ns >= 3 && K % 64 == 0 && (!f8 || wm * wn <= 4);
  const int tiles = ((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  dim3 grid(tiles, split);
#define MID1(BM_, BN_, WM_, WN_, NS_, WNT_)                                                                        \
  gemm_mid_kernel<BM_, BN_, WM_, WN_, NS_, WNT_><<<grid, 64 * WM_ * WN_, 0, st>>>(X, ldx, W, ldw, bias, Y, ldy, \
                                                                                      part, M, N, K, act, glu, cnt, qv, \
                                                                                      nullptr, nullptr, nullptr)
#define MID1F8(BM_, BN_, WM_, WN_, NS_, WNT_)                                                                      \
  do {                                                                                                           \
    if (asc)                                                                                                     \
      gemm_mid_kernel<BM_, BN_, WM_, WN_, mx_ns<BM_, BN_, WM_ * WN_, NS_>(), WNT_, true, 0, false, true>          \
          <<<grid, 64 * WM_ * WN_, 0, st>>>(                                                                     \
          X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, cnt, qv, xs, wsc, asc);                          \
    else                                                                                                         \
      gemm_mid_kernel<BM_, BN_, WM_, WN_, NS_, WNT_, true><<<grid, 64 * WM_ * WN_, 0, st>>>(                    \
          X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, cnt, qv, xs, wsc, nullptr);                      \
  } while (0)
#define MID1F8I(BM_, BN_, WM_, WN_, NS_, WNT_)                                                                     \
  do {                                                                                                           \
    if (asc)                                                                                                     \
      gemm_mid_kernel<BM_, BN_, WM_, WN_, mx_ns<BM_, BN_, WM_ * WN_, (NS_ < 3 ? 3 : NS_)>(), WNT_, true, 0, true, \
                      true>                                                                                      \
          <<<grid, 64 * WM_ * WN_, 0, st>>>(X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, cnt, qv, xs,   \
                                            wsc, asc);                                                           \
    else                                                                                                         \
      gemm_mid_kernel<BM_, BN_, WM_, WN_, (NS_ < 3 ? 3 : NS_), WNT_, true, 0, true>                              \
          <<<grid, 64 * WM_ * WN_, 0, st>>>(X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, cnt, qv, xs,   \
                                            wsc, nullptr);                                                       \
  } while (0)
#define MID1I(BM_, BN_, WM_, WN_, NS_, WNT_)                                                                       \
  gemm_mid_kernel<BM_, BN_, WM_, WN_, (NS_ < 3 ? 3 : NS_), WNT_, false, 0, true>                              \
      <<<grid, 64 * WM_ * WN_, 0, st>>>(X, ldx, W, ldw, bias, Y, ldy, part, M, N, K, act, glu, cnt, qv, nullptr,     \
                                        nullptr, nullptr)
#define MID(BM_, BN_, WM_, WN_, NS_)                                                                             \
  do {                                                                                                         \
    if (f8 && ilv && NS_ >= 3) {                                                                               \
      if (wnt) MID1F8I(BM_, BN_, WM_, WN_, NS_, true); else MID1F8I(BM_, BN_, WM_, WN_, NS_, false);          \
    } else if (f8) {                                                                                           \
      if (wnt) MID1F8(BM_, BN_, WM_, WN_, NS_, true); else MID1F8(BM_, BN_, WM_, WN_, NS_, false);            \
    } else if (ilv && NS_ >= 3) {                                                                              \
      if (wnt) MID1I(BM_, BN_, WM_, WN_, NS_, true); else MID1I(BM_, BN_, WM_, WN_, NS_, false);              \
    } else {                                                                                                   \
      if (wnt) MID1(BM_, BN_, WM_, WN_, NS_, true); else MID1(BM_, BN_, WM_, WN_, NS_, false);                 \
    }                                                                                                          \
  } while (0)
#define MID_NS(BM_, BN_, WM_, WN_)                                               \
  do {                                                                         \
    if (ns >= 6) MID(BM_, BN_, WM_, WN_, 6);                                   \
    else if (ns == 5) MID(BM_, BN_, WM_, WN_, 5);                              \
    else if (ns == 4) MID(BM_, BN_, WM_, WN_, 4);                              \
    else if (ns == 3) MID(BM_, BN_, WM_, WN_, 3);                              \
    else MID(BM_, BN_, WM_, WN_, 2);                                           \
  } while (0)
  switch (tsel) {
    case 8: if (ns >= 5) MID(128, 128, 2, 2, 5); else if (ns == 4) MID(128, 128, 2, 2, 4);
            else if (ns == 3) MID(128, 128, 2, 2, 3); else MID(128, 128, 2, 2, 2); break;
    case 9: if (ns >= 3) MID(256, 128, 4, 2, 3); else MID(256, 128, 4, 2, 2); break;
    case 10: if (ns >= 4) MID(64, 256, 1, 4, 4); else if (ns == 3) MID(64, 256, 1, 4, 3);
             else MID(64, 256, 1, 4, 2); break;
    case 11: MID_NS(64, 128, 1, 4); break;
    case 12: if (ns >= 3) MID(128, 256, 2, 4, 3); else MID(128, 256, 2, 4, 2); break;
    case 13: if (ns >= 5) MID(64, 192, 2, 2, 5); else if (ns == 4) MID(64, 192, 2, 2, 4);
             else if (ns == 3) MID(64, 192, 2, 2, 3); else MID(64, 192, 2, 2, 2); break;
    case 14: MID_NS(64, 32, 4, 1); break;
    case 7: MID_NS(64, 48, 2, 1); break;
    case 15: if (ns >= 5) MID(64, 96, 4, 1, 5); else if (ns == 4) MID(64, 96, 4, 1, 4);
             else if (ns == 3) MID(64, 96, 4, 1, 3); else MID(64, 96, 4, 1, 2); break;
  }
#undef MID_NS
#undef MID
#undef MID1
#undef MID1F8
#undef MID1F8I
#undef MID1I
  HIP_CHECK_LAUNCH();
}
