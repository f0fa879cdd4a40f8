// Chunked-prefill ("extend") attention over the paged KV cache on MFMA.
//
// A step may feed a sequence a chunk of q new tokens at positions [p0, p0 + q) while tokens
// [0, p0) are already cached (an earlier chunk of the same prompt, or a prompt continued after
// generation). The chunk's K/V were written to the paged cache by rope_cache just before; this
// kernel reads every key [0, p0 + q) through the block table, so query position p attends keys
// [0, p] (causal over the chunk, full over the prefix). Reference: the reference has no chunked
// prefill; it re-runs the whole prompt and grows a torch.cat cache (gptj_modeling.py:229-236), and
// past its window it slices the cache (generate.py:132-142).
//
// GQA/MQA: one workgroup serves ONE kv head and all G query heads that read it, so each K/V tile
// is staged into LDS once for the whole head group (the flat-QKV prefill kernel re-fetches it per
// query head). The 64 lanes-columns of a workgroup ("slots") enumerate (query row, head-in-group)
// pairs: slot s -> row s / GE, head s % GE, with GE the group size (or a divisor of it <= 64).
//
// Per wave (16 slots), the products are the swapped ones of attention_prefill.hip:
//   S^T[key][slot] = K . Q^T   (A = K rows via ds_read_b128, B = Q^T fragments in registers)
//   O^T[d][slot]  += V^T . P^T (A = V^T via ds_read_tr16_b64, B = P^T straight from S^T)
// so each lane owns one slot's softmax row.
#include "common.h"

constexpr float kLog2eX = 1.4426950408889634f;

// KV8: fp8 cache rows (D e4m3 bytes + fp32 scale at byte D; reference.py kv_rows_quant), dequantised to
// bf16 while the tile is staged into LDS.
// q8 / s8 (optional): also write the per-token fp8-e4m3 twin of the output rows (== quant_fp8_rows_ld of them, same
// absmax / 448 scale and clamped conversion) for the W8A8 o-projection that consumes them, which then skips its own
// quantisation launch. Only when a workgroup holds every head of its rows: one kv head (nkv = 1) whose whole query
// group fits the slots of a wave (GE = G, a power of two <= 16) - Llama-2-70B at TP=8 (8 query heads per rank).
template <int D, bool KV8>
__global__ __launch_bounds__(256) void attn_extend_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const void* __restrict__ kcv, const void* __restrict__ vcv,
    const int* __restrict__ block_tables, int max_blocks, const int* __restrict__ cu_q, const int* __restrict__ ctx_lens,
    bf16_t* __restrict__ out, int64_t out_stride, int nh, int nkv, int GE, int bs, float scale_log2,
    unsigned char* __restrict__ q8, float* __restrict__ s8) {
  constexpr int BKV = 64;
  constexpr int LD = D + 16;  // padded LDS row (elements): conflict-free b128 rows and tr_b16 columns
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BKV * LD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[BKV * LD];

  const int G = nh / nkv;
  const int rows_per_wg = 64 / GE;
  const int b = blockIdx.z;
  const int kvh = blockIdx.y / (G / GE);
  const int h0 = kvh * G + (blockIdx.y % (G / GE)) * GE;  // first query head of this workgroup
  const int t0 = cu_q[b], qlen = cu_q[b + 1] - t0;
  const int r0 = blockIdx.x * rows_per_wg;
  if (r0 >= qlen) return;
  const int ctx = ctx_lens[b];
  const int p0 = ctx - qlen;  // position of the chunk's first token
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int slot = w * 16 + li;
  const int row = r0 + slot / GE, h = h0 + slot % GE;
  const bool valid = slot < rows_per_wg * GE && row < qlen;
  const int qpos = p0 + (valid ? row : 0);  // causal limit of this lane's slot

  s16x8 qf[D / 32];
  {
    const bf16_t* qp = q + (int64_t)(t0 + (valid ? row : 0)) * q_stride + (int64_t)(valid ? h : h0) * D + 8 * g;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) qf[ks] = *reinterpret_cast<const s16x8*>(qp + 32 * ks);
  }
  f32x4 o[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -1.0e30f, lsum = 0.f;

  // keys needed by this workgroup: [0, last valid row's position]
  const int r_last = min(qlen, r0 + rows_per_wg) - 1;
  const int kv_end = p0 + r_last + 1;
  // this wave's slots: rows r0 + (16w)/GE .. r0 + (16w+15)/GE
  const int wave_qhi = p0 + min(qlen - 1, r0 + (16 * w + 15) / GE);
  const int* bt = block_tables + (int64_t)b * max_blocks;
  constexpr int CH = D / 8;
  constexpr int RB = KV8 ? D + 16 : D;         // cache row (elements of the cache dtype)
  const int64_t head_stride = (int64_t)bs * RB;  // one kv head of one block
  const bf16_t* __restrict__ kc = (const bf16_t*)kcv;
  const bf16_t* __restrict__ vc = (const bf16_t*)vcv;
  const unsigned char* __restrict__ kc8 = (const unsigned char*)kcv;
  const unsigned char* __restrict__ vc8 = (const unsigned char*)vcv;
  // page ids of keys [0, kv_end) staged in LDS once: a tile's K/V loads then wait for no dependent
  // block-table load (an L2 round trip per tile)
  constexpr int kMaxPages = 512;
  __shared__ int s_pages[kMaxPages];
  const int npg = (kv_end + bs - 1) / bs;
  const bool lds_pages = npg <= kMaxPages;
  if (lds_pages)
    for (int i = threadIdx.x; i < npg; i += 256) s_pages[i] = bt[i];
  __syncthreads();
  // Software pipeline: tile t+1's K/V chunks are loaded into registers while tile t is computed from LDS
  // (the register set is written to LDS after the next barrier), so each tile no longer waits a full
  // HBM round trip behind the previous tile's compute.
  static_assert((BKV * CH) % 256 == 0, "whole 16-B chunks per thread");
  constexpr int NCH = BKV * CH / 256;  // 16-B chunks per thread per tile
  u16x8 kr[NCH], vr[NCH];
  u32x2 kr8[NCH], vr8[NCH];
  float ksr[NCH], vsr[NCH];
  auto load_tile = [&](int kv0) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = threadIdx.x + j * 256;
      const int r = c / CH, ch = c % CH;
      const int key = min(kv0 + r, kv_end - 1);
      const int blk = lds_pages ? s_pages[key / bs] : bt[key / bs];
      const int64_t rowoff = ((int64_t)blk * nkv + kvh) * head_stride + (int64_t)(key % bs) * RB;
      if constexpr (KV8) {
        kr8[j] = *reinterpret_cast<const u32x2*>(kc8 + rowoff + ch * 8);
        vr8[j] = *reinterpret_cast<const u32x2*>(vc8 + rowoff + ch * 8);
        ksr[j] = *reinterpret_cast<const float*>(kc8 + rowoff + D);
        vsr[j] = *reinterpret_cast<const float*>(vc8 + rowoff + D);
      } else {
        kr[j] = *reinterpret_cast<const u16x8*>(kc + rowoff + ch * 8);
        vr[j] = *reinterpret_cast<const u16x8*>(vc + rowoff + ch * 8);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int c = threadIdx.x + j * 256;
      const int r = c / CH, ch = c % CH;
      if constexpr (KV8) {
        u16x8 kb, vb;
#pragma unroll
        for (int hw = 0; hw < 2; ++hw) {
          const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8(kr8[j][hw], false), c2 = __builtin_amdgcn_cvt_pk_f32_fp8(kr8[j][hw], true);
          const f32x2 x = __builtin_amdgcn_cvt_pk_f32_fp8(vr8[j][hw], false), y = __builtin_amdgcn_cvt_pk_f32_fp8(vr8[j][hw], true);
          kb[4 * hw] = f2bf(a[0] * ksr[j]); kb[4 * hw + 1] = f2bf(a[1] * ksr[j]);
          kb[4 * hw + 2] = f2bf(c2[0] * ksr[j]); kb[4 * hw + 3] = f2bf(c2[1] * ksr[j]);
          vb[4 * hw] = f2bf(x[0] * vsr[j]); vb[4 * hw + 1] = f2bf(x[1] * vsr[j]);
          vb[4 * hw + 2] = f2bf(y[0] * vsr[j]); vb[4 * hw + 3] = f2bf(y[1] * vsr[j]);
        }
        *reinterpret_cast<u16x8*>(&Ks[r * LD + ch * 8]) = kb;
        *reinterpret_cast<u16x8*>(&Vs[r * LD + ch * 8]) = vb;
      } else {
        *reinterpret_cast<u16x8*>(&Ks[r * LD + ch * 8]) = kr[j];
        *reinterpret_cast<u16x8*>(&Vs[r * LD + ch * 8]) = vr[j];
      }
    }
  };
  // D = 256: the register set would cost the kernel its occupancy - staged chunk by chunk instead
  constexpr bool PIPE = D <= 128;
  auto stage_direct = [&](int kv0) {
#pragma unroll
    for (int c = threadIdx.x; c < BKV * CH; c += 256) {
      const int r = c / CH, ch = c % CH;
      const int key = min(kv0 + r, kv_end - 1);
      const int blk = lds_pages ? s_pages[key / bs] : bt[key / bs];
      const int64_t rowoff = ((int64_t)blk * nkv + kvh) * head_stride + (int64_t)(key % bs) * RB;
      if constexpr (KV8) {
        kr8[0] = *reinterpret_cast<const u32x2*>(kc8 + rowoff + ch * 8);
        vr8[0] = *reinterpret_cast<const u32x2*>(vc8 + rowoff + ch * 8);
        ksr[0] = *reinterpret_cast<const float*>(kc8 + rowoff + D);
        vsr[0] = *reinterpret_cast<const float*>(vc8 + rowoff + D);
        u16x8 kb, vb;
#pragma unroll
        for (int hw = 0; hw < 2; ++hw) {
          const f32x2 a = __builtin_amdgcn_cvt_pk_f32_fp8(kr8[0][hw], false), c2 = __builtin_amdgcn_cvt_pk_f32_fp8(kr8[0][hw], true);
          const f32x2 x = __builtin_amdgcn_cvt_pk_f32_fp8(vr8[0][hw], false), y = __builtin_amdgcn_cvt_pk_f32_fp8(vr8[0][hw], true);
          kb[4 * hw] = f2bf(a[0] * ksr[0]); kb[4 * hw + 1] = f2bf(a[1] * ksr[0]);
          kb[4 * hw + 2] = f2bf(c2[0] * ksr[0]); kb[4 * hw + 3] = f2bf(c2[1] * ksr[0]);
          vb[4 * hw] = f2bf(x[0] * vsr[0]); vb[4 * hw + 1] = f2bf(x[1] * vsr[0]);
          vb[4 * hw + 2] = f2bf(y[0] * vsr[0]); vb[4 * hw + 3] = f2bf(y[1] * vsr[0]);
        }
        *reinterpret_cast<u16x8*>(&Ks[r * LD + ch * 8]) = kb;
        *reinterpret_cast<u16x8*>(&Vs[r * LD + ch * 8]) = vb;
      } else {
        *reinterpret_cast<u16x8*>(&Ks[r * LD + ch * 8]) = *reinterpret_cast<const u16x8*>(kc + rowoff + ch * 8);
        *reinterpret_cast<u16x8*>(&Vs[r * LD + ch * 8]) = *reinterpret_cast<const u16x8*>(vc + rowoff + ch * 8);
      }
    }
  };
  if constexpr (PIPE) {
    if (kv_end > 0) load_tile(0);
  }
  for (int kv0 = 0; kv0 < kv_end; kv0 += BKV) {
    __syncthreads();  // every wave is done reading the previous tile
    if constexpr (PIPE) store_tile();
    else stage_direct(kv0);
    __syncthreads();
    if constexpr (PIPE) {
      if (kv0 + BKV < kv_end) load_tile(kv0 + BKV);
    }
    if (kv0 > wave_qhi) continue;  // whole tile in this wave's causal future (barriers stay uniform)

    f32x4 s[4];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt) {
      s[kt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < D / 32; ++ks) {
        const s16x8 kf = *reinterpret_cast<const s16x8*>(&Ks[(kt * 16 + li) * LD + 32 * ks + 8 * g]);
        s[kt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[ks], s[kt], 0, 0, 0);
      }
    }
    // S^T C layout: lane (li, g) holds slot li's scores for keys kv0 + 16kt + 4g + i
    float mx = m;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kv0 + kt * 16 + 4 * g + i;
        float v = s[kt][i] * scale_log2;
        v = (key <= qpos && key < kv_end) ? v : -1.0e30f;
        s[kt][i] = v;
        mx = fmaxf(mx, v);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float alpha = exp2f(m - mx);
    m = mx;
    float ps = 0.f;
    s16x8 pf[2];
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p = exp2f(s[kt][i] - mx);
        const bf16_t pb = f2bf(p);
        ps += bf2f(pb);
        pf[kt >> 1][(kt & 1) * 4 + i] = (short)pb;
      }
    ps += __shfl_xor(ps, 16, 64);
    ps += __shfl_xor(ps, 32, 64);
    lsum = lsum * alpha + ps;
#pragma unroll
    for (int i = 0; i < D / 16; ++i) o[i] *= alpha;

    const int tq = li >> 2, tp = li & 3;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        const bf16_t* a0 = &Vs[(32 * ks + 4 * g + tq) * LD + dt * 16 + 4 * tp];
        const bf16_t* a1 = a0 + 16 * LD;
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a0));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((LDS_AS s16x4*)(a1));
        const s16x8 vf = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
        o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[ks], o[dt], 0, 0, 0);
      }
    }
  }
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  u16x4 res[D / 16];
  float amax = 0.f;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      res[dt][i] = f2bf(o[dt][i] * inv);
      amax = fmaxf(amax, fabsf(bf2f(res[dt][i])));
    }
  if (valid) {
    bf16_t* op = out + (int64_t)(t0 + row) * out_stride + (int64_t)h * D + 4 * g;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) *reinterpret_cast<u16x4*>(op + dt * 16) = res[dt];
  }
  if (q8 == nullptr) return;  // kernel argument: uniform
  // a row's slots are GE consecutive lanes of one wave (GE | 16): reduce over them and over the 4 lane groups
  if (!valid) amax = 0.f;
  for (int off = 1; off < GE; off <<= 1) amax = fmaxf(amax, __shfl_xor(amax, off, 64));
  amax = fmaxf(amax, __shfl_xor(amax, 16, 64));
  amax = fmaxf(amax, __shfl_xor(amax, 32, 64));
  if (!valid) return;
  const float sc = amax > 0.f ? amax / 448.f : 1.f;
  const float rs = 1.f / sc;
  const int64_t qrow = (int64_t)(t0 + row) * (nh * D);
  if (slot % GE == 0 && g == 0) s8[t0 + row] = sc;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    float f[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) f[i] = fminf(fmaxf(bf2f(res[dt][i]) * rs, -448.f), 448.f);
    unsigned v = 0;
    v = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], v, false);
    v = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], v, true);
    *reinterpret_cast<unsigned*>(q8 + qrow + (int64_t)h * D + dt * 16 + 4 * g) = v;
  }
}

// GE: largest divisor of the group size G that is <= 64 (slots per workgroup)
static int extend_group(int G) {
  for (int ge = std::min(G, 64); ge >= 1; --ge)
    if (G % ge == 0) return ge;
  return 1;
}

void launch_attn_extend(const void* q, int64_t q_stride, const void* k_cache, const void* v_cache,
                        const void* block_tables, int max_blocks, const void* cu_q, const void* ctx_lens, void* out,
                        int64_t out_stride, int B, int max_qlen, int nh, int nkv, int D, int bs, float scale,
                        hipStream_t st, bool kv8, void* q8v, void* s8v) {
  if (nh % nkv) throw std::runtime_error("attn_extend: nh must be a multiple of nkv");
  if (B == 0 || max_qlen == 0) return;
  const int G = nh / nkv, GE = extend_group(G);
  auto Q8 = (unsigned char*)q8v;
  auto S8 = (float*)s8v;
  if ((Q8 != nullptr) != (S8 != nullptr)) throw std::runtime_error("attn_extend: fp8 twin needs both q8 and s8");
  if (Q8 && !(nkv == 1 && GE == G && G <= 16 && (G & (G - 1)) == 0))
    throw std::runtime_error("attn_extend: the fp8 twin needs one kv head and a power-of-two query group <= 16");
  const int rows = 64 / GE;
  dim3 grid((max_qlen + rows - 1) / rows, nkv * (G / GE), B);
  auto Q = (const bf16_t*)q;
  auto K = k_cache;
  auto V = v_cache;
  auto BT = (const int*)block_tables;
  auto CU = (const int*)cu_q;
  auto CL = (const int*)ctx_lens;
  auto O = (bf16_t*)out;
  const float sl = scale * kLog2eX;
#define LX(D_)                                                                                                   \
  do {                                                                                                           \
    if (kv8)                                                                                                     \
      attn_extend_kernel<D_, true><<<grid, 256, 0, st>>>(Q, q_stride, K, V, BT, max_blocks, CU, CL, O, out_stride, nh, \
                                                         nkv, GE, bs, sl, Q8, S8);                               \
    else                                                                                                         \
      attn_extend_kernel<D_, false><<<grid, 256, 0, st>>>(Q, q_stride, K, V, BT, max_blocks, CU, CL, O, out_stride,   \
                                                          nh, nkv, GE, bs, sl, Q8, S8);                          \
  } while (0)
  switch (D) {
    case 64: LX(64); break;
    case 128: LX(128); break;
    case 256: LX(256); break;
    default: throw std::runtime_error("attn_extend: head_dim must be 64, 128 or 256");
  }
#undef LX
  HIP_CHECK_LAUNCH();
}
