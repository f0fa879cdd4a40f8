// Prototype: 256x256x64 bf16 prefill GEMM with a ping-pong K-loop (guide "The 256^2 8-phase template",
// MI355X_MICROARCH "Two waves per SIMD"). Built as a standalone .so (extern "C" launchers) so that
// bench/pp_probe.py can time its variants against torch.matmul (hipBLASLt) and the in-tree gemm_big in
// one process on random data.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared bench/proto/pp_gemm.hip -o bench/proto/libpp.so
//
// Schedule (per wave; 8 waves = two groups of 4, one wave of each group on every SIMD):
//   * K-tile = 64 (128 B per row); LDS = 2 buffers x 4 slots of 16 KiB: slot 0 = A half 0, 1 = B half 0,
//     2 = B half 1, 3 = A half 1. A half h holds block rows {128 r + 64 h + i}, B half h block columns
//     {64 c + 32 h + j}: every wave's 128x64 output splits into four 64x32 quadrants Q(mq, nq), each
//     reading one A slot and one B slot.
//   * 4 phases per K-tile: Q(0,0) [reads A0 + B0], Q(0,1) [B1], Q(1,1) [A1], Q(1,0) [B0 kept in
//     registers]. Phase = load segment (fragment ds_reads, 2 global_load_lds of one slot of the NEXT
//     K-tile, counted vmcnt) | barrier | compute segment (16 MFMA 16x16x32) | barrier.
//   * waves 4-7 pass one extra barrier first, so each SIMD alternates one wave's compute segment with
//     its partner's load segment (ping-pong); waves 0-3 pass the matching barrier at the end.
//   * RAW: a slot is read one phase after the vmcnt that retires it (vmcnt 4/4/6/4 in steady state);
//     WAR: a slot is restaged >= 4 phases after its last read.
#include "../../llmss_amd/csrc/common.h"

template <int N>
__device__ __forceinline__ void vmc() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
__device__ __forceinline__ void pbar() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

// VAR bits: 1 = setprio(1) around each MFMA cluster, 2 = static setprio(1) for waves 4-7,
//           4 = no stagger (all 8 waves in lockstep; the control arm)
template <int VAR>
__global__ __launch_bounds__(512, 1) void pp_gemm_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                         const bf16_t* __restrict__ B, int64_t ldb,
                                                         const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                         int64_t ldy, int M, int N, int K, int act, int glu,
                                                         int group_m) {
  constexpr bool PRIO = VAR & 1, SPRIO = VAR & 2, STAGGER = !(VAR & 4), BAL = VAR & 8;
  // ablations (wrong results, timing only): 16 = no vmcnt waits in the K-loop, 32 = no LDS-DMA in the K-loop,
  // 64 = no fragment reads in the K-loop
  constexpr bool NOWAIT = VAR & 16, NODMA = VAR & 32, NOREAD = VAR & 64;
  // 128 = LDS-DMA issued before the fragment reads of the load segment; 256 = LDS-DMA issued by the compute
  // segment after its first 8 MFMAs (the load segment's vmcnt then counts one stage fewer)
  constexpr bool DFIRST = VAR & 128, DINC = VAR & 256;
  constexpr int SLOT = 16384, BUF = 4 * SLOT;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 2, wc = w & 3;
  const int ntn = (N + 255) / 256, ntm = (M + 255) / 256;
  const int GM = group_m;
  const int tile = xcd_remap(blockIdx.x, ntn * ntm);
  const int grp = tile / (GM * ntn), gidx = tile - grp * (GM * ntn);
  const int gm = min(GM, ntm - grp * GM);
  const int m0 = (grp * GM + gidx % gm) * 256, n0 = (gidx / gm) * 256;
  const int nk = K / 64;

  // staging: slot h, instruction i (0, 1): 1 KiB = 8 local rows x 128 B, local row lr = (8 i + w) * 8 + lane / 8;
  // LDS chunk lane & 7 holds global chunk (lane & 7) ^ (lr & 7)
  const char* src[4] = {(const char*)A, (const char*)B, (const char*)B, (const char*)A};
  int64_t soff[4][2];
  int lofs[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int inst = i * 8 + w;
    const int lr = inst * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ (lr & 7);
    lofs[i] = inst * 1024;
    const int ar0 = min(m0 + (lr >> 6) * 128 + (lr & 63), M - 1);
    const int ar1 = min(m0 + (lr >> 6) * 128 + 64 + (lr & 63), M - 1);
    const int bc0 = min(n0 + (lr >> 5) * 64 + (lr & 31), N - 1);
    const int bc1 = min(n0 + (lr >> 5) * 64 + 32 + (lr & 31), N - 1);
    soff[0][i] = (int64_t)ar0 * lda * 2 + gc * 16;
    soff[3][i] = (int64_t)ar1 * lda * 2 + gc * 16;
    soff[1][i] = (int64_t)bc0 * ldb * 2 + gc * 16;
    soff[2][i] = (int64_t)bc1 * ldb * 2 + gc * 16;
  }
  bool inloop = false;
  auto stage = [&](int t, int h, char* buf) {
    if (NODMA && inloop) return;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(src[h] + soff[h][i] + (int64_t)t * 128),
                                       (LDS_AS void*)(buf + h * SLOT + lofs[i]), 16, 0, 0);
  };

  // fragment offsets inside a slot: A rows wr*64 + mt*16 + li, B rows wc*32 + nt*16 + li; k-half s -> chunk 4s+g
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
    if (NOREAD && inloop) return;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int s = 0; s < 2; ++s) fa[mt][s] = *reinterpret_cast<const s16x8*>(slot + aoff[mt][s]);
  };
  auto rdB = [&](const char* slot, s16x8 (&fb)[2][2]) {
    if (NOREAD && inloop) return;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s = 0; s < 2; ++s) fb[nt][s] = *reinterpret_cast<const s16x8*>(slot + boff[nt][s]);
  };
  auto quad = [&](int mq, int nq, const s16x8 (&fb)[2][2]) {
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mq * 4 + mt][nq * 2 + nt] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt][s], fb[nt][s], acc[mq * 4 + mt][nq * 2 + nt], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  };

  if constexpr (BAL) {
    // balanced reads 8 / 4 / 8 / 4: B0 of the NEXT K-tile is read in phase 3 into a second register set.
    // Staging order per K-tile: B0, A0, B1, A1 (each retired 2 phases after issue, read one phase later).
    s16x8 fb0n[2][2];
    stage(0, 1, smem);
    stage(0, 0, smem);
    stage(0, 2, smem);
    stage(0, 3, smem);
    vmc<4>();  // B0, A0 landed
    pbar();
    rdB(smem + SLOT, fb0);
    if constexpr (SPRIO) {
      if (w >= 4) __builtin_amdgcn_s_setprio(1);
    }
    if constexpr (STAGGER) {
      if (w >= 4) pbar();
    }
    for (int t = 0; t < nk; ++t) {
      const char* cur = smem + (t & 1) * BUF;
      char* nxt = smem + ((t + 1) & 1) * BUF;
      const bool more = t + 1 < nk;
      rdA(cur);
      if (more) {
        stage(t + 1, 1, nxt);
        vmc<4>();
      } else {
        vmc<2>();
      }
      pbar();
      quad(0, 0, fb0);
      pbar();
      rdB(cur + 2 * SLOT, fb1);
      if (more) {
        stage(t + 1, 0, nxt);
        vmc<4>();
      } else {
        vmc<0>();
      }
      pbar();
      quad(0, 1, fb1);
      pbar();
      rdA(cur + 3 * SLOT);
      if (more) {
        stage(t + 1, 2, nxt);
        vmc<4>();
      }
      pbar();
      quad(1, 1, fb1);
      pbar();
      if (more) {
        rdB(nxt + SLOT, fb0n);
        stage(t + 1, 3, nxt);
        vmc<4>();
      }
      pbar();
      quad(1, 0, fb0);
      pbar();
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int s = 0; s < 2; ++s) fb0[nt][s] = fb0n[nt][s];
    }
  } else {
#pragma unroll
  for (int h = 0; h < 4; ++h) stage(0, h, smem);
  vmc<4>();
  pbar();
  if constexpr (SPRIO) {
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
  }
  if constexpr (STAGGER) {
    if (w >= 4) pbar();
  }
  inloop = true;
  // one phase: load segment (reads RD, LDS-DMA of slot H of the next K-tile, vmcnt N retiring what the next
  // phase reads), barrier, compute segment, barrier
  auto phase = [&](auto rd, int t, int h, bool more, int nwait_more, int nwait_last, int mq, int nq,
                   const s16x8 (&fb)[2][2]) {
    char* nxt = smem + ((t + 1) & 1) * BUF;
    if (DFIRST && more) stage(t + 1, h, nxt);
    rd();
    if (!DFIRST && !DINC && more) stage(t + 1, h, nxt);
    if constexpr (!NOWAIT) {
      const int n = more ? (DINC ? nwait_more - 2 : nwait_more) : nwait_last;
      switch (n) {
        case 0: vmc<0>(); break;
        case 2: vmc<2>(); break;
        case 4: vmc<4>(); break;
        case 6: vmc<6>(); break;
        default: break;
      }
    }
    pbar();
    if constexpr (DINC) {
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mq * 4 + mt][nq * 2 + nt] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt][0], fb[nt][0], acc[mq * 4 + mt][nq * 2 + nt], 0, 0, 0);
      if (more) stage(t + 1, h, nxt);
#pragma unroll
      for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
          acc[mq * 4 + mt][nq * 2 + nt] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt][1], fb[nt][1], acc[mq * 4 + mt][nq * 2 + nt], 0, 0, 0);
      if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
    } else {
      quad(mq, nq, fb);
    }
    pbar();
  };
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t & 1) * BUF;
    const bool more = t + 1 < nk;
    phase([&] { rdA(cur); rdB(cur + SLOT, fb0); }, t, 0, more, 4, 2, 0, 0, fb0);
    phase([&] { rdB(cur + 2 * SLOT, fb1); }, t, 1, more, 4, 0, 0, 1, fb1);
    phase([&] { rdA(cur + 3 * SLOT); }, t, 2, more, 6, -1, 1, 1, fb1);
    phase([&] {}, t, 3, more, 4, -1, 1, 0, fb0);
  }
  }
  if constexpr (STAGGER) {
    if (w < 4) pbar();
  }
  if constexpr (SPRIO) __builtin_amdgcn_s_setprio(0);
  vmc<0>();
  tile_store_lds<256, 256, 8, 4, 512, 2 * BUF>(acc, smem, wr * 128, wc * 64, m0, n0, M, N, nullptr, Y, ldy, bias,
                                               act, glu);
}

// 4 waves (one per SIMD), each a 128x128 output (8x8 accumulators, 256 VGPRs), 2 x 64 KiB LDS buffers.
// Per K-tile t: sub-step 0 MFMAs (64) with the sub-step-1 fragment reads interleaved; lgkmcnt(0) +
// vmcnt(0) (stage t+1, issued one K-tile ago) + barrier; sub-step 1 MFMAs (64) with the stage-t+2 LDS-DMA
// (16 per wave) into the buffer just released and the NEXT K-tile's sub-step-0 fragment reads interleaved.
// VAR bit 1: glds front-loaded (2 per 4 MFMAs over the first half of sub-step 1), bit 2: setprio(1) on
// the whole K-loop.
template <int VAR>
__global__ __launch_bounds__(256, 1) void qq_gemm_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                         const bf16_t* __restrict__ B, int64_t ldb,
                                                         const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                         int64_t ldy, int M, int N, int K, int act, int glu,
                                                         int group_m) {
  constexpr bool FRONT = VAR & 1;
  constexpr int HALF = 32768, BUF = 2 * HALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int wr = w >> 1, wc = w & 1;
  const int ntn = (N + 255) / 256, ntm = (M + 255) / 256;
  const int GM = group_m;
  const int tile = xcd_remap(blockIdx.x, ntn * ntm);
  const int grp = tile / (GM * ntn), gidx = tile - grp * (GM * ntn);
  const int gm = min(GM, ntm - grp * GM);
  const int m0 = (grp * GM + gidx % gm) * 256, n0 = (gidx / gm) * 256;
  const int nk = K / 64;

  // staging: 16 glds per wave per K-tile: j < 8 -> A rows (8 j + w) * 8.., j >= 8 -> B rows
  int64_t soff[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int inst = (j & 7) * 4 + w;  // 0..31
    const int r = inst * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ (r & 7);
    const int gr = j < 8 ? min(m0 + r, M - 1) : min(n0 + r, N - 1);
    soff[j] = (int64_t)gr * (j < 8 ? lda : ldb) * 2 + gc * 16;
  }
  const int lbase = w * 1024;
  auto glds = [&](int j, int t, char* buf) {
    const char* s = (const char*)(j < 8 ? (const void*)A : (const void*)B);
    __builtin_amdgcn_global_load_lds((const void*)(s + soff[j] + (int64_t)t * 128),
                                     (LDS_AS void*)(buf + (j >> 3) * HALF + (j & 7) * 4096 + lbase), 16, 0, 0);
  };
  int aoff[8][2], boff[8][2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    const int c = 4 * s + g;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int ra = wr * 128 + i * 16 + li, rb = wc * 128 + i * 16 + li;
      aoff[i][s] = ra * 128 + ((c ^ (ra & 7)) << 4);
      boff[i][s] = HALF + rb * 128 + ((c ^ (rb & 7)) << 4);
    }
  }
  f32x4 acc[8][8];
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  s16x8 fa0[8], fb0[8], fa1[8], fb1[8];

  // prologue: stage 0, wait, barrier, stage 1, read sub-step 0 fragments of tile 0
#pragma unroll
  for (int j = 0; j < 16; ++j) glds(j, 0, smem);
  vmc<0>();
  pbar();
#pragma unroll
  for (int j = 0; j < 16; ++j) glds(j, min(1, nk - 1), smem + BUF);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa0[i] = *reinterpret_cast<const s16x8*>(smem + aoff[i][0]);
    fb0[i] = *reinterpret_cast<const s16x8*>(smem + boff[i][0]);
  }
  if constexpr (VAR & 2) __builtin_amdgcn_s_setprio(1);
  for (int t = 0; t < nk; ++t) {
    char* cur = smem + (t & 1) * BUF;
    const char* nxt = smem + ((t + 1) & 1) * BUF;
    const int t2 = min(t + 2, nk - 1);
    // sub-step 0: 64 MFMAs, sub-step-1 reads (16) one per 4 MFMAs
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      fa1[m] = *reinterpret_cast<const s16x8*>(cur + aoff[m][1]);
      fb1[m] = *reinterpret_cast<const s16x8*>(cur + boff[m][1]);
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa0[m], fb0[n], acc[m][n], 0, 0, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): sub-step-1 fragments (and this wave's reads of cur) done
    vmc<0>();                             // stage t+1 landed
    pbar();
    // sub-step 1: 64 MFMAs; stage t+2 into cur, next tile's sub-step-0 reads from nxt
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      // past the last K-tile the DMA re-reads tile nk-1 into the free buffer and the reads pick up unused
      // bytes: no branch inside the MFMA stream (it would split the scheduling region)
      if constexpr (FRONT) {
        if (m < 4) {
          glds(4 * m, t2, cur);
          glds(4 * m + 1, t2, cur);
          glds(4 * m + 2, t2, cur);
          glds(4 * m + 3, t2, cur);
        }
      } else {
        glds(2 * m, t2, cur);
        glds(2 * m + 1, t2, cur);
      }
      fa0[m] = *reinterpret_cast<const s16x8*>(nxt + aoff[m][0]);
      fb0[m] = *reinterpret_cast<const s16x8*>(nxt + boff[m][0]);
#pragma unroll
      for (int n = 0; n < 8; ++n) acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa1[m], fb1[n], acc[m][n], 0, 0, 0);
      if constexpr (FRONT) {
        if (m < 4) {
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        }
      } else {
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      }
    }
  }
  if constexpr (VAR & 2) __builtin_amdgcn_s_setprio(0);
  vmc<0>();
  tile_store_lds<256, 256, 8, 8, 256, 2 * BUF>(acc, smem, wr * 128, wc * 128, m0, n0, M, N, nullptr, Y, ldy, bias,
                                               act, glu);
}

// 4 waves x 128x128 on the 32x32x16 MFMA (acc 4x4 f32x16 = 256 registers: fewer, larger accumulator objects than
// qq_gemm_kernel's 8x8 f32x4). LDS rows of 128 B with the chunk swizzle f(row) = (row >> 1) & 7, conflict-free for
// the 32-row ds_read_b128 fragments. Per K-tile: 4 k-steps of 16, fragments double-buffered across k-steps, the
// next K-tile's 16 LDS-DMA per wave spread 4 per k-step, one barrier per K-tile. Epilogue: direct bf16 stores.
template <int VAR>
__global__ __launch_bounds__(256, 1) void qq2_gemm_kernel(const bf16_t* __restrict__ A, int64_t lda,
                                                          const bf16_t* __restrict__ B, int64_t ldb,
                                                          const bf16_t* __restrict__ bias, bf16_t* __restrict__ Y,
                                                          int64_t ldy, int M, int N, int K, int act, int glu,
                                                          int group_m) {
  constexpr int HALF = 32768, BUF = 2 * HALF;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r32 = lane & 31, h = lane >> 5;
  const int wr = w >> 1, wc = w & 1;
  const int ntn = (N + 255) / 256, ntm = (M + 255) / 256;
  const int GM = group_m;
  const int tile = xcd_remap(blockIdx.x, ntn * ntm);
  const int grp = tile / (GM * ntn), gidx = tile - grp * (GM * ntn);
  const int gm = min(GM, ntm - grp * GM);
  const int m0 = (grp * GM + gidx % gm) * 256, n0 = (gidx / gm) * 256;
  const int nk = K / 64;

  int64_t soff[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int inst = (j & 7) * 4 + w;
    const int r = inst * 8 + (lane >> 3);
    const int gc = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = j < 8 ? min(m0 + r, M - 1) : min(n0 + r, N - 1);
    soff[j] = (int64_t)gr * (j < 8 ? lda : ldb) * 2 + gc * 16;
  }
  auto glds = [&](int j, int t, char* buf) {
    const char* s = (const char*)(j < 8 ? (const void*)A : (const void*)B);
    __builtin_amdgcn_global_load_lds((const void*)(s + soff[j] + (int64_t)t * 128),
                                     (LDS_AS void*)(buf + (j >> 3) * HALF + (j & 7) * 4096 + w * 1024), 16, 0, 0);
  };
  int aoff[4][4], boff[4][4];  // [tile][k-step]
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int c = 2 * ks + h;
      const int ra = wr * 128 + i * 32 + r32, rb = wc * 128 + i * 32 + r32;
      aoff[i][ks] = ra * 128 + ((c ^ ((ra >> 1) & 7)) << 4);
      boff[i][ks] = HALF + rb * 128 + ((c ^ ((rb >> 1) & 7)) << 4);
    }
  f32x16 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[a][b][e] = 0.f;
  s16x8 fa0[4], fb0[4], fa1[4], fb1[4];
  auto rd = [&](const char* buf, int ks, s16x8 (&fa)[4], s16x8 (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      fa[i] = *reinterpret_cast<const s16x8*>(buf + aoff[i][ks]);
      fb[i] = *reinterpret_cast<const s16x8*>(buf + boff[i][ks]);
    }
  };
  auto mm = [&](const s16x8 (&fa)[4], const s16x8 (&fb)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int n = 0; n < 4; ++n) acc[i][n] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[i], fb[n], acc[i][n], 0, 0, 0);
  };

#pragma unroll
  for (int j = 0; j < 16; ++j) glds(j, 0, smem);
  vmc<0>();
  pbar();
  rd(smem, 0, fa0, fb0);
  if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(1);
  for (int t = 0; t < nk; ++t) {
    const char* cur = smem + (t & 1) * BUF;
    char* nxt = smem + ((t + 1) & 1) * BUF;
    const int t1 = min(t + 1, nk - 1);  // past the last K-tile the DMA reloads tile nk-1 into the free buffer
    // k-step 0: read 1, DMA 0-3, MFMA 0 ...
    rd(cur, 1, fa1, fb1);
#pragma unroll
    for (int j = 0; j < 4; ++j) glds(j, t1, nxt);
    mm(fa0, fb0);
    rd(cur, 2, fa0, fb0);
#pragma unroll
    for (int j = 4; j < 8; ++j) glds(j, t1, nxt);
    mm(fa1, fb1);
    rd(cur, 3, fa1, fb1);
#pragma unroll
    for (int j = 8; j < 12; ++j) glds(j, t1, nxt);
    mm(fa0, fb0);
#pragma unroll
    for (int j = 12; j < 16; ++j) glds(j, t1, nxt);
    mm(fa1, fb1);
    vmc<0>();
    __builtin_amdgcn_s_waitcnt(0xC07F);
    pbar();
    rd(nxt, 0, fa0, fb0);
  }
  if constexpr (VAR & 1) __builtin_amdgcn_s_setprio(0);
  // epilogue: C layout col = lane & 31, row = (r & 3) + 8 (r >> 2) + 4 h
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int n = 0; n < 4; ++n) {
      const int col = n0 + wc * 128 + n * 32 + r32;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wr * 128 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < M && col < N) Y[(int64_t)row * ldy + col] = f2bf(acc[i][n][r]);
      }
    }
}

template <int VAR>
static int launch_qq2(const void* A, int64_t lda, const void* B, int64_t ldb, const void* bias, void* Y, int64_t ldy,
                      int M, int N, int K, int act, int glu, int gm, hipStream_t st) {
  if (K % 64 || M <= 0 || N <= 0) return -1;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  hipLaunchKernelGGL(qq2_gemm_kernel<VAR>, dim3(tiles), dim3(256), 0, st, (const bf16_t*)A, lda, (const bf16_t*)B,
                     ldb, (const bf16_t*)bias, (bf16_t*)Y, ldy, M, N, K, act, glu, gm);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int VAR>
static int launch_qq(const void* A, int64_t lda, const void* B, int64_t ldb, const void* bias, void* Y, int64_t ldy,
                     int M, int N, int K, int act, int glu, int gm, hipStream_t st) {
  if (K % 64 || M <= 0 || N <= 0) return -1;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  hipLaunchKernelGGL(qq_gemm_kernel<VAR>, dim3(tiles), dim3(256), 0, st, (const bf16_t*)A, lda, (const bf16_t*)B,
                     ldb, (const bf16_t*)bias, (bf16_t*)Y, ldy, M, N, K, act, glu, gm);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int VAR>
static int launch(const void* A, int64_t lda, const void* B, int64_t ldb, const void* bias, void* Y, int64_t ldy,
                  int M, int N, int K, int act, int glu, int gm, hipStream_t st) {
  if (K % 64 || M <= 0 || N <= 0) return -1;
  const int tiles = ((M + 255) / 256) * ((N + 255) / 256);
  hipLaunchKernelGGL(pp_gemm_kernel<VAR>, dim3(tiles), dim3(512), 0, st, (const bf16_t*)A, lda, (const bf16_t*)B,
                     ldb, (const bf16_t*)bias, (bf16_t*)Y, ldy, M, N, K, act, glu, gm);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" int pp_gemm(int var, const void* A, int64_t lda, const void* B, int64_t ldb, const void* bias, void* Y,
                       int64_t ldy, int M, int N, int K, int act, int glu, int gm, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  switch (var) {
    case 0: return launch<0>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 1: return launch<1>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 2: return launch<2>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 3: return launch<3>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 4: return launch<4>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 5: return launch<5>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 18: return launch<18>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 34: return launch<34>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 66: return launch<66>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 98: return launch<98>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 130: return launch<130>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 258: return launch<258>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 8: return launch<8>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 10: return launch<10>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 11: return launch<11>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 200: return launch_qq2<0>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 201: return launch_qq2<1>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 100: return launch_qq<0>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 101: return launch_qq<1>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 102: return launch_qq<2>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    case 103: return launch_qq<3>(A, lda, B, ldb, bias, Y, ldy, M, N, K, act, glu, gm, st);
    default: return -3;
  }
}
