// Persistent fused MLP block for decode steps (M <= 64 rows, TP = 1): ONE launch for
//
//   r = delta + residual  (delta = the o-projection's split-K slabs + bias, or its bf16 output)
//   y = norm(r) * w (+ b)                         phase A: one workgroup per row
//   h = act(y @ Wup^T + bup)  (SwiGLU / GELU ...)  phase B: each workgroup a 64 x 32*UB column tile, full K
//   out[s] = h[:, slice s] @ Wdown[:, slice s]^T   phase C: (64-column tile, K slice) per workgroup, fp32 slabs
//
// replacing add_norm + up GEMM + down GEMM (three launches; reference: the residual add + LayerNorm and the
// fc_in -> act -> fc_out MLP of gptj_modeling.py:254-310 / gpt_bigcode_modeling.py:311-330, and Llama's
// RMSNorm + SwiGLU MLP). The slabs are summed by the next add_norm (or the final norm), as the unfused
// down GEMM's split-K slabs are.
//
// Why one launch: at M <= 64 every GEMM of a decode layer streams its weights once and is bound by the
// weight stream plus a fixed per-launch cost (grid fill, first-load latency, store drain; profiles/r4_gemm).
// Here a workgroup issues the NEXT phase's weight stages into its LDS ring BEFORE it waits for the hand-off
// that phase's activations depend on, so the weight stream of phase B / C is in flight while phase A / B
// drains (MI355X_MICROARCH "prefetch-credit"), and the two kernel boundaries disappear.
//
// Hand-offs (MI355X_MICROARCH "Valid forms"): the producer stores its bytes write-through (sc1 buffer
// stores, 16 B), every storing wave waits vmcnt(0), a workgroup barrier, then one lane adds to an agent-
// scope counter; the consumer polls the counter from one lane (sc1 loads + s_sleep), takes ONE agent acquire
// fence, waits vmcnt(0), a workgroup barrier, then reads with plain loads (LDS-DMA). Placement-independent:
// nothing assumes which XCD a workgroup runs on. Waits are on work counts (rows normed, up units done per
// down K-slice), never on workgroup counts, and every counted unit is produced by a workgroup that already
// runs before it waits: with every workgroup resident (grid <= CUs x occupancy, checked by the launcher)
// the launch cannot deadlock. Spins are bounded: on a timeout the kernel raises a device flag and goes on.
// The counters reset themselves: the last workgroup to finish zeroes them for the next launch.
#include "common.h"

constexpr int kMaxChunks = 4;  // phase A: 8-element chunks per thread -> H <= 8192

// kernel argument block (external linkage: the kernel templates are instantiated over it)
struct FusedMlpArgs {
  const float* dpart;  // [dS][M][H] o-projection split-K slabs, or nullptr (then `delta`)
  int dS;
  const bf16_t* dbias;  // o-projection bias (added to the slab sum), or nullptr
  const bf16_t* delta;  // [M][H] bf16 o-projection output (dpart == nullptr)
  bf16_t* resid;        // [M][H] residual stream, updated in place (r)
  const bf16_t* nw;
  const bf16_t* nb;
  float eps;
  bf16_t* y;  // [M][H] hand-off 1: normed rows
  const bf16_t* wu;  // [N1][H] up projection (SwiGLU: 16-row gate | up blocks, models/weights.py)
  const bf16_t* bu;  // [N1] or nullptr
  bf16_t* h;         // [M][F] hand-off 2: activated up output
  const bf16_t* wd;  // [H][F] down projection
  float* out;        // [S2][M][H] fp32 partial slabs of the down projection
  int M, H, N1, F, S2, act;
  int* cnt;  // [2 + S2]: rows normed, workgroups finished, up units done per down K-slice
  int* err;  // set when a hand-off wait timed out
};
using MlpArgs = FusedMlpArgs;

namespace {

__device__ __forceinline__ void vm_wait(int n) {
  // s_waitcnt takes an immediate: one case per count (loads in flight per wave stay below 32 here)
  switch (n) {
#define W_(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    W_(0) W_(1) W_(2) W_(3) W_(4) W_(5) W_(6) W_(7) W_(8) W_(9) W_(10) W_(11) W_(12) W_(13) W_(14) W_(15)
    W_(16) W_(17) W_(18) W_(19) W_(20) W_(21) W_(22) W_(23) W_(24) W_(25) W_(26) W_(27) W_(28) W_(29) W_(30)
#undef W_
    default: asm volatile("s_waitcnt vmcnt(31)" ::: "memory"); break;
  }
}

__device__ __forceinline__ void raw_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Producer side of a hand-off: every wave's (sc1) stores are complete, then ONE lane adds `v` to `c`.
__device__ __forceinline__ void publish(int* c, int v) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && v) __hip_atomic_fetch_add(c, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Consumer side: one lane polls `c` until it reaches `target` (bounded), ONE agent acquire, then every wave
// may read the handed-off bytes with plain loads.
__device__ __forceinline__ void await_count(const int* c, int target, int* err) {
  if (threadIdx.x == 0) {
    unsigned spins = 0;
    while (__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1u << 26)) {  // seconds: a non-resident producer; flag it instead of hanging the GPU
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}

// Buffer descriptors are built inside device function bodies only (never as members or in signatures: the
// host compilation pass has no descriptor type and would silently drop the kernel's launch stub).
__device__ __forceinline__ int rsrc_bytes(uint64_t bytes) {
  return (int)(bytes > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)bytes);
}

// 16-B write-through store (sc1: the line leaves L2 for the memory side, where any XCD's acquire sees it);
// bytes at or past `bytes` from `base` are dropped by the range check
__device__ __forceinline__ void store_wt(void* base, uint64_t bytes, uint32_t off, u32x4 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, rsrc_bytes(bytes), 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, rs, off, 0u, 16);
}

// ------------------------------------------------------------------------------------------- phase A
template <bool RMS>
__device__ void norm_row(const MlpArgs& a, int row, float* red) {
  const int H = a.H, nchunk = H >> 3;
  float v[kMaxChunks][8];
  u16x8 wv[kMaxChunks], bv[kMaxChunks];
#pragma unroll
  for (int c = 0; c < kMaxChunks; ++c) {
    const int ch = min((int)threadIdx.x + c * 256, nchunk - 1);
    wv[c] = *reinterpret_cast<const u16x8*>(a.nw + ch * 8);
    if (a.nb) bv[c] = *reinterpret_cast<const u16x8*>(a.nb + ch * 8);
  }
#pragma unroll
  for (int c = 0; c < kMaxChunks; ++c) {
    const int ch = threadIdx.x + c * 256;
    if (ch < nchunk) {
      if (a.dpart) {  // the unfused add_norm_partial: slab sum (+ bias), rounded as the GEMM's bf16 output
        const float* pr = a.dpart + (int64_t)row * H + ch * 8;
        const int64_t slab = (int64_t)a.M * H;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
        for (int sp = 0; sp < a.dS; ++sp) {
          const f32x4 p0 = *reinterpret_cast<const f32x4*>(pr + sp * slab);
          const f32x4 p1 = *reinterpret_cast<const f32x4*>(pr + sp * slab + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[c][j] += p0[j]; v[c][4 + j] += p1[j]; }
        }
        if (a.dbias) {
          const u16x8 bb = *reinterpret_cast<const u16x8*>(a.dbias + ch * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) v[c][j] += bf2f(bb[j]);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(f2bf(v[c][j]));
      } else {
        const u16x8 d = *reinterpret_cast<const u16x8*>(a.delta + (int64_t)row * H + ch * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[c][j] = bf2f(d[j]);
      }
      const u16x8 r = *reinterpret_cast<const u16x8*>(a.resid + (int64_t)row * H + ch * 8);
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[c][j] += bf2f(r[j]);
        o[j] = f2bf(v[c][j]);
        v[c][j] = bf2f(o[j]);
      }
      *reinterpret_cast<u16x8*>(a.resid + (int64_t)row * H + ch * 8) = o;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c][j] = 0.f;
    }
  }
  float mean = 0.f, var;
  {
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int c = 0; c < kMaxChunks; ++c)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        s += v[c][j];
        ss += v[c][j] * v[c][j];
      }
    if constexpr (RMS) {
      var = block_sum(ss, red) / H;
    } else {
      const f32x2 tot = block_sum2(s, ss, red);
      mean = tot[0] / H;
      var = fmaxf(tot[1] / H - mean * mean, 0.f);
    }
  }
  const float rstd = rsqrtf(var + a.eps);
#pragma unroll
  for (int c = 0; c < kMaxChunks; ++c) {
    const int ch = threadIdx.x + c * 256;
    if (ch < nchunk) {
      u16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float t = (v[c][j] - mean) * rstd * bf2f(wv[c][j]);
        if (a.nb) t += bf2f(bv[c][j]);
        o[j] = f2bf(t);
      }
      store_wt(a.y, (uint64_t)a.M * H * 2, (uint32_t)((row * H + ch * 8) * 2), __builtin_bit_cast(u32x4, o));
    }
  }
}

// ------------------------------------------------------------------------------------- GEMM ring
// C[64 x BN] (+)= A[64 rows, k-steps] . B[BN rows, k-steps]^T over nk 64-deep k-steps, bf16 operands staged
// by LDS-DMA (global_load_lds, 16 B per lane) into a ring of NS stages ([A 64 x 128 B | B BN x 128 B] each,
// 16-B chunks XOR-swizzled by row as in gemm_mid.hip). 4 waves; wave w owns rows 16w..16w+15 and all BN
// columns (NT = BN / 16 accumulators). Operand rows past the matrix end are clamped to its last row: they
// only feed output rows / columns that are never stored.
template <int BN, int NS>
struct Ring {
  static constexpr int AL = 2, BL = BN / 32, LOADS = AL + BL;  // 1-KiB wave loads per stage
  static constexpr int A_BYTES = 64 * 128, STAGE = A_BYTES + BN * 128, BYTES = NS * STAGE;
  static constexpr int NT = BN / 16;
  char* lds;
  const char* pa[AL];  // this lane's 16-B source chunk of k-step 0, per staging load
  const char* pb[BL];

  __device__ void init(char* l, const bf16_t* A, int64_t lda, int arows, const bf16_t* B, int64_t ldb, int brows,
                       int ka0, int kb0) {
    lds = l;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < AL; ++i) {
      const int row = (i * 4 + w) * 8 + (lane >> 3);
      pa[i] = reinterpret_cast<const char*>(A) + (int64_t)min(row, arows - 1) * lda * 2 + ka0 +
              (((lane & 7) ^ (row & 7)) << 4);
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int row = (i * 4 + w) * 8 + (lane >> 3);
      pb[i] = reinterpret_cast<const char*>(B) + (int64_t)min(row, brows - 1) * ldb * 2 + kb0 +
              (((lane & 7) ^ (row & 7)) << 4);
    }
  }
  __device__ __forceinline__ void issue_a(int t) {
    char* s = lds + (t % NS) * STAGE;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < AL; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(pa[i] + t * 128), (LDS_AS void*)(s + (i * 4 + w) * 1024), 16,
                                       0, 0);
  }
  __device__ __forceinline__ void issue_b(int t) {
    char* s = lds + (t % NS) * STAGE + A_BYTES;
    const int w = threadIdx.x >> 6;
#pragma unroll
    for (int i = 0; i < BL; ++i)  // weights: read once, non-temporal
      __builtin_amdgcn_global_load_lds((const void*)(pb[i] + t * 128), (LDS_AS void*)(s + (i * 4 + w) * 1024), 16,
                                       0, 2);
  }
  // weights of stages 0 .. NS-2 ahead of the hand-off the A operand waits for
  __device__ void prefetch_b(int nk) {
    for (int t = 0; t < NS - 1 && t < nk; ++t) issue_b(t);
  }
  // prefetched: issue_b(0 .. NS-2) ran before a vmcnt(0) drain (await_count); else nothing was issued
  __device__ void run(f32x4 (&acc)[NT], int nk, bool prefetched) {
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[n] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int pre = min(NS - 1, nk);
    for (int t = 0; t < pre; ++t) {
      if (!prefetched) issue_b(t);
      issue_a(t);
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;
    const int arow = w * 16 + li;
    const int x0 = (g ^ (li & 7)) << 4, x1 = ((4 + g) ^ (li & 7)) << 4;
    for (int t = 0; t < nk; ++t) {
      // loads issued after stage t's last one: prologue A-parts of younger stages (prefetched: the B-parts
      // landed already) and the full stages issued by earlier steps, capped by what remains
      int after;
      if (prefetched && t < pre) {
        after = (pre - 1 - t) * AL + max(0, min(t, nk - (NS - 1))) * LOADS;
      } else {
        after = min(NS - 2, nk - 1 - t) * LOADS;
      }
      vm_wait(after);
      raw_barrier();
      if (t + NS - 1 < nk) {
        issue_b(t + NS - 1);
        issue_a(t + NS - 1);
      }
      const char* st = lds + (t % NS) * STAGE;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int xo = s ? x1 : x0;
        const s16x8 av = *reinterpret_cast<const s16x8*>(st + arow * 128 + xo);
#pragma unroll
        for (int n = 0; n < NT; ++n) {
          const s16x8 bv = *reinterpret_cast<const s16x8*>(st + A_BYTES + (n * 16 + li) * 128 + xo);
          acc[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc[n], 0, 0, 0);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // every wave is done reading the ring (the epilogue reuses it)
  }
};

}  // namespace

template <bool RMS, bool GLU, int UB>
__global__ __launch_bounds__(256, 1) void fused_mlp_kernel(MlpArgs a) {
  using RB = Ring<32 * UB, (UB == 1 ? 6 : 4)>;  // phase B: 64 x 32*UB tile, full K
  using RC = Ring<64, 4>;                       // phase C: 64 x 64 tile, one K slice
  __shared__ __attribute__((aligned(16))) char smem[RB::BYTES + RC::BYTES];
  __shared__ float red[32];
  char* ldsB = smem;
  char* ldsC = smem + RB::BYTES;
  const int wg = blockIdx.x, G = gridDim.x;
  const int H = a.H, F = a.F, M = a.M;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, li = lane & 15, g = lane >> 4;

  // ---- work of this workgroup
  const int nunits = a.N1 / 32;                 // up units of 32 weight rows
  const int opu = GLU ? 16 : 32;                // h columns per unit
  const int u0 = wg * UB, nu = max(0, min(UB, nunits - u0));
  const int ntc = H / 64, nks = F / 64;         // phase C: column tiles, k-steps over F
  const int citem = wg < ntc * a.S2 ? wg : -1;  // (column tile, K slice)
  const int cj = citem >= 0 ? citem % ntc : 0, cs = citem >= 0 ? citem / ntc : 0;
  const int cks0 = cs * nks / a.S2, cks1 = (cs + 1) * nks / a.S2;
  int* cnt_rows = a.cnt;
  int* cnt_done = a.cnt + 1;
  int* cnt_slice = a.cnt + 2;

  RB rb_;
  RC rc_;
  if (nu > 0) rb_.init(ldsB, a.y, H, M, a.wu + (int64_t)u0 * 32 * H, H, nu * 32, 0, 0);
  if (citem >= 0) rc_.init(ldsC, a.h, F, M, a.wd + (int64_t)cj * 64 * F, F, 64, cks0 * 128, cks0 * 128);

  // ---- phase A: rows (workgroups 0 .. M-1), then the up weights ahead of the rows hand-off
  if (wg < M) {
    norm_row<RMS>(a, wg, red);
    publish(cnt_rows, 1);
  }
  if (nu > 0) rb_.prefetch_b(H / 64);
  if (citem >= 0 && nu == 0) rc_.prefetch_b(cks1 - cks0);  // idle in phase B: start the down weights now

  // ---- phase B: up projection + activation -> h (write-through), per-slice unit counts
  if (nu > 0) {
    await_count(cnt_rows, M, a.err);
    f32x4 acc[RB::NT];
    rb_.run(acc, H / 64, true);
    // epilogue: activation in registers, bf16 tile [64][opu * UB] staged in the (drained) ring, 16-B stores
    constexpr int OC = (GLU ? 16 : 32) * UB;  // output columns of the tile
    bf16_t* stile = reinterpret_cast<bf16_t*>(ldsB);
    const int oc0 = u0 * opu;
#pragma unroll
    for (int n = 0; n < RB::NT; ++n) {
      if constexpr (GLU) {
        if (n & 1) continue;
        const int p = n >> 1;  // unit p of the tile: gate tile n, up tile n + 1
        if (p >= nu) continue;
        const int wrow = (u0 + p) * 32 + li;  // gate weight row; up row = +16
        const float bg = a.bu ? bf2f(a.bu[wrow]) : 0.f, bu = a.bu ? bf2f(a.bu[wrow + 16]) : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          stile[(w * 16 + 4 * g + i) * OC + p * 16 + li] = f2bf(silu(acc[n][i] + bg) * (acc[n + 1][i] + bu));
      } else {
        if (n / 2 >= nu) continue;
        const int col = (u0 * 32) + n * 16 + li;
        const float bb = a.bu ? bf2f(a.bu[col]) : 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i) stile[(w * 16 + 4 * g + i) * OC + n * 16 + li] = f2bf(apply_act(acc[n][i] + bb, a.act));
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    const int vpr = nu * opu / 8;  // 16-B pieces per row
    for (int v = threadIdx.x; v < 64 * vpr; v += 256) {
      const int r = v / vpr, c = (v - r * vpr) * 8;
      if (r < M)
        store_wt(a.h, (uint64_t)M * F * 2, (uint32_t)((r * F + oc0 + c) * 2),
                 *reinterpret_cast<const u32x4*>(stile + r * OC + c));
    }
    // units of this tile per down K slice (a tile's units are contiguous: at most a few slices)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      for (int p = 0; p < nu;) {
        const int ks = (u0 + p) * opu / 64;  // k-step of the down GEMM holding unit u0 + p's columns
        int s = 0;                            // its K slice
        while (s + 1 < a.S2 && (s + 1) * nks / a.S2 <= ks) ++s;
        const int send = (s + 1) * nks / a.S2 * 64;  // first h column past slice s
        int q = 0;
        while (p + q < nu && (u0 + p + q) * opu < send) ++q;
        __hip_atomic_fetch_add(cnt_slice + s, q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        p += q;
      }
    }
    if (citem >= 0) rc_.prefetch_b(cks1 - cks0);
  }

  // ---- phase C: down projection of one (64-column tile, K slice) -> fp32 slab
  if (citem >= 0) {
    const int c0 = cks0 * 64, c1 = cks1 * 64;  // h columns of the slice
    const int need = (c1 + opu - 1) / opu - c0 / opu;
    await_count(cnt_slice + cs, need, a.err);
    f32x4 acc[RC::NT];
    rc_.run(acc, cks1 - cks0, true);
    // fp32 tile [64][64] staged in the drained ring, 16-B row stores into slab cs
    float* ct = reinterpret_cast<float*>(ldsC);
    constexpr int LDW = 68;
#pragma unroll
    for (int n = 0; n < RC::NT; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) ct[(w * 16 + 4 * g + i) * LDW + n * 16 + li] = acc[n][i];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    float* dst = a.out + (int64_t)cs * M * H;
    for (int v = threadIdx.x; v < 64 * 16; v += 256) {
      const int r = v >> 4, c = (v & 15) * 4;
      if (r < M) *reinterpret_cast<f32x4*>(dst + (int64_t)r * H + cj * 64 + c) = *reinterpret_cast<const f32x4*>(ct + r * LDW + c);
    }
  }

  // ---- the last workgroup out zeroes the counters for the next launch
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt_done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (t == G - 1) {
      __hip_atomic_store(cnt_rows, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int s = 0; s < a.S2; ++s) __hip_atomic_store(cnt_slice + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cnt_done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// ------------------------------------------------------------------------------------------ launcher
template <bool RMS, bool GLU, int UB>
static int max_resident() {
  int dev = 0, cus = 0, per = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fused_mlp_kernel<RMS, GLU, UB>, 256, 0) != hipSuccess) return 0;
  return cus * per;
}

// Plan of a fused MLP launch: workgroups, up units per workgroup, down K slices. Returns false when the
// shape is not supported (then the caller runs add_norm + up + down).
bool fused_mlp_plan(int M, int H, int N1, int F, bool glu, int* grid, int* ub, int* s2) {
  if (M < 1 || M > 64 || H % 64 || F % 64 || N1 % 32 || H > 8 * 8 * 256 || (glu ? N1 != 2 * F : N1 != F)) return false;
  int G;
  {
    static int cached = -1;
    if (cached < 0) cached = max_resident<true, true, 3>();  // the largest-LDS instantiation bounds them all
    G = std::min(cached, 256);
  }
  if (G < 64) return false;
  const int nunits = N1 / 32;
  const int u = (nunits + G - 1) / G;
  if (u > 3) return false;
  const int ntc = H / 64, nks = F / 64;
  int s = std::max(1, std::min(G / ntc, 16));
  while (s > 1 && nks / s < 2) --s;
  if (ntc * s > G || M > G) return false;
  *grid = G;
  *ub = u;
  *s2 = s;
  return true;
}

void launch_fused_mlp(const void* dpart, int dS, const void* dbias, const void* delta, void* resid, const void* nw,
                      const void* nb, float eps, bool rms, void* y, const void* wu, const void* bu, void* h,
                      const void* wd, void* out, int M, int H, int N1, int F, bool glu, int act, int grid, int ub,
                      int s2, int* cnt, int* err, hipStream_t st) {
  int G, u, s;
  if (!fused_mlp_plan(M, H, N1, F, glu, &G, &u, &s) || G != grid || u != ub || s != s2)
    throw std::runtime_error("fused_mlp: plan mismatch (call fused_mlp_plan first)");
  MlpArgs a{(const float*)dpart, dS, (const bf16_t*)dbias, (const bf16_t*)delta, (bf16_t*)resid,
            (const bf16_t*)nw, (const bf16_t*)nb, eps, (bf16_t*)y, (const bf16_t*)wu, (const bf16_t*)bu,
            (bf16_t*)h, (const bf16_t*)wd, (float*)out, M, H, N1, F, s2, act, cnt, err};
#define FM(R_, G_, U_) fused_mlp_kernel<R_, G_, U_><<<G, 256, 0, st>>>(a)
#define FM_U(R_, G_)                     \
  do {                                   \
    if (u == 1) FM(R_, G_, 1);           \
    else if (u == 2) FM(R_, G_, 2);      \
    else FM(R_, G_, 3);                  \
  } while (0)
  if (rms) {
    if (glu) FM_U(true, true); else FM_U(true, false);
  } else {
    if (glu) FM_U(false, true); else FM_U(false, false);
  }
#undef FM_U
#undef FM
  HIP_CHECK_LAUNCH();
}
