// Paged split-K decode attention for one new token per sequence (SURVEY K11-K14 for S=1;
// reference: eager fp32 QK^T, CPU causal-mask copy, softmax, @V over a torch.cat'd cache,
// gptj_modeling.py:128-169; MQA baddbmm + TorchScript softmax + bmm,
// gpt_bigcode_modeling.py:170-246).
//
// Memory-bound: every byte of K/V for (seq, kv head) is read exactly once per query-head
// group. One workgroup = (sequence, kv head, query-head group of GB heads, context split).
// Lane layout: LPT = D/8 lanes own one token (16 B = 8 dims each), TPW = 64/LPT tokens per
// wave-load; each (wave, token slot) keeps its own online-softmax state (m, l, acc) so the
// token loop has no cross-lane traffic except the LPT-lane dot-product reduction. States are
// merged once at the end (shuffles inside the wave, LDS across the 4 waves). K and V of a
// token are loaded together and UNROLL tokens are kept in flight per slot.
// Splits > 1 write unnormalised partials that attn_decode_reduce_kernel combines.
#include "common.h"

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kNegBig = -1.0e30f;

// Sum over the LPT lanes that hold one token (LPT = D / 8 consecutive lanes) with DPP lane moves
// instead of ds_bpermute shuffles (no LDS round trip in the per-token dependency chain).
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
template <int LPT>
__device__ __forceinline__ float token_sum(float s) {
  if constexpr (LPT >= 16) {  // row_ror:8,4,2,1 inside each 16-lane row
    s += dpp_f<0x128>(s);
    s += dpp_f<0x124>(s);
    s += dpp_f<0x122>(s);
    s += dpp_f<0x121>(s);
    if constexpr (LPT == 32) s += __shfl_xor(s, 16, 64);
  } else if constexpr (LPT == 8) {  // row_half_mirror, then quad_perm xor 2, xor 1
    s += dpp_f<0x141>(s);
    s += dpp_f<0x4e>(s);   // quad_perm [2,3,0,1]
    s += dpp_f<0xb1>(s);   // quad_perm [1,0,3,2]
  } else {
#pragma unroll
    for (int o = 1; o < LPT; o <<= 1) s += __shfl_xor(s, o, 64);
  }
  return s;
}

// KV8: the paged cache holds fp8 rows (D e4m3 bytes + fp32 scale at byte D, 16-B tail; reference.py
// kv_rows_quant): each lane loads 8 bytes per token instead of 16 and the row scales multiply the score
// (K) and the probability (V) instead of every element.
template <int D, int GB, int UNROLL, bool PIPE = false, bool KV8 = false>
__global__ __launch_bounds__(256, GB == 1 ? 8 : 1) void attn_decode_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, void* __restrict__ kcv, void* __restrict__ vcv,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ ctx_lens, bf16_t* __restrict__ out,
    int64_t out_stride, float* __restrict__ part_o, float* __restrict__ part_ml, int nh, int nkv, int G, int ngroups,
    int block_size, int part_size, float scale_log2) {
  constexpr int LPT = D / 8;
  constexpr int TPW = 64 / LPT;
  constexpr int RB = KV8 ? D + 16 : D;  // cache row, in cache elements (bytes for fp8 rows)
  bf16_t* __restrict__ kc = (bf16_t*)kcv;
  bf16_t* __restrict__ vc = (bf16_t*)vcv;
  const unsigned char* __restrict__ kc8 = (const unsigned char*)kcv;
  const unsigned char* __restrict__ vc8 = (const unsigned char*)vcv;
  const int b = blockIdx.x;
  const int kvh = blockIdx.y / ngroups, grp = blockIdx.y % ngroups;
  const int split = blockIdx.z, nsplit = gridDim.z;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int slot = lane / LPT, sub = lane % LPT;
  const int h0 = kvh * G + grp * GB;
  const int nvalid = min(GB, G - grp * GB);

  // q (pre-scaled into the log2 domain)
  float qv[GB][8];
#pragma unroll
  for (int h = 0; h < GB; ++h) {
    if (h < nvalid) {
      u16x8 a = *reinterpret_cast<const u16x8*>(q + b * q_stride + (int64_t)(h0 + h) * D + sub * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[h][j] = bf2f(a[j]) * scale_log2;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) qv[h][j] = 0.f;
    }
  }
  float m[GB], l[GB], acc[GB][8];
#pragma unroll
  for (int h = 0; h < GB; ++h) {
    m[h] = kNegBig; l[h] = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[h][j] = 0.f;
  }

  const int ctx = min(ctx_lens[b], bt_stride * block_size);  // never index past the block table
  const int start = split * part_size;
  const int end = min(ctx, start + part_size);
  const int* bt = block_tables + (int64_t)b * bt_stride;
  const int64_t head_off = (int64_t)kvh * block_size * RB + sub * 8;
  const int64_t page_stride = (int64_t)nkv * block_size * RB;
  constexpr int STEP = 4 * TPW;  // tokens per workgroup-iteration
  const int lend = end;

  // page ids of this workgroup's context range, staged once in LDS: the token loop then needs no
  // dependent block-table load (an L2 round trip) in front of every K/V load. The staged range is the
  // whole partition's pages (clamped to the table row), not the context's: it does not depend on
  // ctx_lens, so the table loads issue beside the ctx_lens / q loads instead of one round trip after
  // them (entries past the sequence's last page are loaded but never used)
  constexpr int kMaxPages = 256;
  __shared__ int s_pages[kMaxPages];
  const int pg0 = start / block_size;
  const int npg = min((start + part_size - 1) / block_size + 1, bt_stride) - pg0;
  const bool lds_pages = npg <= kMaxPages;
  if (lds_pages) {
    for (int i = threadIdx.x; i < npg; i += blockDim.x) s_pages[i] = bt[pg0 + i];
    __syncthreads();
  }
  auto kv_addr = [&](int t) -> int64_t {
    const int pi = t / block_size;
    const int page = lds_pages ? s_pages[pi - pg0] : bt[pi];
    return page * page_stride + head_off + (int64_t)(t % block_size) * RB;
  };
  // a token's K / V registers: bf16 rows 16 B per lane; fp8 rows 8 B per lane + the row's two scales
  struct KVRegs {
    u16x8 k[UNROLL], v[UNROLL];
    u32x2 k8[UNROLL], v8[UNROLL];
    float ks[UNROLL], vs[UNROLL];
  };
  auto load_tokens = [&](int tb, KVRegs& r) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int t = tb + u * STEP;
      const int64_t a = kv_addr(t < lend ? t : start);
      // read once per step: non-temporal (guide 'nt-weights'; +10-15% on streamed reads)
      if constexpr (KV8) {
        r.k8[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(kc8 + a));
        r.v8[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(vc8 + a));
        r.ks[u] = *reinterpret_cast<const float*>(kc8 + a - sub * 8 + D);
        r.vs[u] = *reinterpret_cast<const float*>(vc8 + a - sub * 8 + D);
      } else {
        r.k[u] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(kc + a));
        r.v[u] = __builtin_nontemporal_load(reinterpret_cast<const u16x8*>(vc + a));
      }
    }
  };
  auto consume = [&](int tb, const KVRegs& r) {
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const bool ok = tb + u * STEP < lend;
      float kf[8], vf[8], ks = 1.f, vs = 1.f;
      if constexpr (KV8) {
        const f32x2 k0 = __builtin_amdgcn_cvt_pk_f32_fp8(r.k8[u][0], false), k1 = __builtin_amdgcn_cvt_pk_f32_fp8(r.k8[u][0], true);
        const f32x2 k2 = __builtin_amdgcn_cvt_pk_f32_fp8(r.k8[u][1], false), k3 = __builtin_amdgcn_cvt_pk_f32_fp8(r.k8[u][1], true);
        const f32x2 v0 = __builtin_amdgcn_cvt_pk_f32_fp8(r.v8[u][0], false), v1 = __builtin_amdgcn_cvt_pk_f32_fp8(r.v8[u][0], true);
        const f32x2 v2 = __builtin_amdgcn_cvt_pk_f32_fp8(r.v8[u][1], false), v3 = __builtin_amdgcn_cvt_pk_f32_fp8(r.v8[u][1], true);
        kf[0] = k0[0]; kf[1] = k0[1]; kf[2] = k1[0]; kf[3] = k1[1]; kf[4] = k2[0]; kf[5] = k2[1]; kf[6] = k3[0]; kf[7] = k3[1];
        vf[0] = v0[0]; vf[1] = v0[1]; vf[2] = v1[0]; vf[3] = v1[1]; vf[4] = v2[0]; vf[5] = v2[1]; vf[6] = v3[0]; vf[7] = v3[1];
        ks = r.ks[u];
        vs = r.vs[u];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) { kf[j] = bf2f(r.k[u][j]); vf[j] = bf2f(r.v[u][j]); }
      }
#pragma unroll
      for (int h = 0; h < GB; ++h) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s = fmaf(qv[h][j], kf[j], s);
        s = token_sum<LPT>(s);
        if constexpr (KV8) s *= ks;
        if (ok) {
          const float mn = fmaxf(m[h], s);
          const float alpha = exp2f(m[h] - mn), p = exp2f(s - mn);
          l[h] = l[h] * alpha + p;
          const float pv = KV8 ? p * vs : p;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[h][j] = fmaf(acc[h][j], alpha, pv * vf[j]);
          m[h] = mn;
        }
      }
    }
  };
  if constexpr (PIPE) {
    // two register sets: the loads of the next UNROLL tokens per slot are in flight while the
    // current ones are consumed (the compiler's counted vmcnt waits only for the set it reads)
    constexpr int CH = STEP * UNROLL;
    KVRegs A, Bq;
    int tb = start + w * TPW + slot;
    if (start < lend) load_tokens(tb, A);
    for (; tb - slot - w * TPW < lend; tb += 2 * CH) {
      load_tokens(tb + CH, Bq);
      consume(tb, A);
      if (tb + CH - slot - w * TPW >= lend) break;
      load_tokens(tb + 2 * CH, A);
      consume(tb + CH, Bq);
    }
  } else {
    for (int tb = start + w * TPW + slot; tb < lend; tb += STEP * UNROLL) {
      KVRegs R;
      load_tokens(tb, R);
      consume(tb, R);
    }
  }

  // merge token slots inside the wave
#pragma unroll
  for (int o = LPT; o < 64; o <<= 1) {
#pragma unroll
    for (int h = 0; h < GB; ++h) {
      const float mo = __shfl_xor(m[h], o, 64), lo = __shfl_xor(l[h], o, 64);
      const float mn = fmaxf(m[h], mo);
      const float a = exp2f(m[h] - mn), c = exp2f(mo - mn);
      l[h] = l[h] * a + lo * c;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float ao = __shfl_xor(acc[h][j], o, 64);
        acc[h][j] = acc[h][j] * a + ao * c;
      }
      m[h] = mn;
    }
  }
  // merge the 4 waves through LDS: [wave][GB][D] acc + [wave][GB] (m, l)
  __shared__ float s_acc[4][GB][D];
  __shared__ float s_ml[4][GB][2];
  if (slot == 0) {
#pragma unroll
    for (int h = 0; h < GB; ++h) {
#pragma unroll
      for (int j = 0; j < 8; ++j) s_acc[w][h][sub * 8 + j] = acc[h][j];
      if (sub == 0) { s_ml[w][h][0] = m[h]; s_ml[w][h][1] = l[h]; }
    }
  }
  __syncthreads();
  // final: thread i handles (h, d) pairs
  for (int i = threadIdx.x; i < GB * D; i += blockDim.x) {
    const int h = i / D, d = i % D;
    if (h >= nvalid) continue;
    float mm = kNegBig;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) mm = fmaxf(mm, s_ml[ww][h][0]);
    float ll = 0.f, o = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) {
      const float c = exp2f(s_ml[ww][h][0] - mm);
      ll += s_ml[ww][h][1] * c;
      o += s_acc[ww][h][d] * c;
    }
    const int head = h0 + h;
    if (nsplit == 1) {
      out[b * out_stride + (int64_t)head * D + d] = f2bf(ll > 0.f ? o / ll : 0.f);
    } else {
      const int64_t pi = ((int64_t)b * nh + head) * nsplit + split;
      part_o[pi * D + d] = o;
      if (d == 0) { part_ml[pi * 2] = mm; part_ml[pi * 2 + 1] = ll; }
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void attn_decode_reduce_kernel(const float* __restrict__ part_o,
                                                                 const float* __restrict__ part_ml,
                                                                 bf16_t* __restrict__ out, int64_t out_stride, int nh,
                                                                 int nsplit) {
  const int b = blockIdx.x, h = blockIdx.y;
  const int64_t base = ((int64_t)b * nh + h) * nsplit;
  float mm = kNegBig;
  for (int s = 0; s < nsplit; ++s) mm = fmaxf(mm, part_ml[(base + s) * 2]);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float ll = 0.f, o = 0.f;
    for (int s = 0; s < nsplit; ++s) {
      const float c = exp2f(part_ml[(base + s) * 2] - mm);
      ll += part_ml[(base + s) * 2 + 1] * c;
      o += part_o[(base + s) * D + d] * c;
    }
    out[b * out_stride + (int64_t)h * D + d] = f2bf(ll > 0.f ? o / ll : 0.f);
  }
}

// tokens in flight per (wave, slot): 1 / 2 / 4 = one register set; 11 / 12 / 14 = two register sets,
// the next set's loads issued before the current set is consumed (tuning knob attn_decode_set_unroll)
// default 11 (measured, bench/attn_bench.py, cold KV, B = 64: best or within 1% of best for MHA at
// 192 / 1024 tokens and 12-17% ahead for GQA groups of 4)
static int g_decode_unroll = 11;
void attn_decode_set_unroll(int u) { g_decode_unroll = (u == 1 || u == 2 || u == 4 || u == 11 || u == 12 || u == 14) ? u : 11; }

template <int D, int GB>
static void launch_decode_t(const bf16_t* q, int64_t qs, bf16_t* kc, bf16_t* vc, const int* bt, int bts,
                            const int* cl, bf16_t* out, int64_t os, float* po, float* pml, int B, int nh, int nkv,
                            int bs, int nsplit, int psize, float scale, hipStream_t st, bool kv8) {
  const int G = nh / nkv;
  const int ngroups = (G + GB - 1) / GB;
  dim3 grid(B, nkv * ngroups, nsplit);
  const float sl2 = scale * kLog2e;
#define AD(U_, PIPE_, KV8_)                                                                                      \
  attn_decode_kernel<D, GB, U_, PIPE_, KV8_><<<grid, 256, 0, st>>>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, nh, \
                                                                  nkv, G, ngroups, bs, psize, sl2)
  if (kv8) {
    switch (g_decode_unroll) {
      case 2: AD(2, false, true); break;
      case 12: AD(2, true, true); break;
      default: AD(1, true, true); break;
    }
  } else {
    switch (g_decode_unroll) {
      case 1: AD(1, false, false); break;
      case 2: AD(2, false, false); break;
      case 4: AD(4, false, false); break;
      case 12: AD(2, true, false); break;
      case 14: AD(4, true, false); break;
      default: AD(1, true, false); break;
    }
  }
#undef AD
  HIP_CHECK_LAUNCH();
  if (nsplit > 1) {
    attn_decode_reduce_kernel<D><<<dim3(B, nh), std::min(D, 256), 0, st>>>(po, pml, out, os, nh, nsplit);
    HIP_CHECK_LAUNCH();
  }
}

template <int D>
static void launch_decode_d(const bf16_t* q, int64_t qs, bf16_t* kc, bf16_t* vc, const int* bt, int bts,
                            const int* cl, bf16_t* out, int64_t os, float* po, float* pml, int B, int nh, int nkv,
                            int bs, int nsplit, int psize, float scale, hipStream_t st, bool kv8) {
  const int G = nh / nkv;
  if (G == 1) launch_decode_t<D, 1>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st, kv8);
  else if (G == 2) launch_decode_t<D, 2>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st, kv8);
  else if (G <= 4) launch_decode_t<D, 4>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st, kv8);
  else launch_decode_t<D, 8>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st, kv8);
}

static void attn_decode_dispatch(const void* q, int64_t q_stride, void* kc, void* vc, const void* block_tables,
                                 int bt_stride, const void* ctx_lens, void* out, int64_t out_stride, void* part_o,
                                 void* part_ml, int B, int nh, int nkv, int D, int block_size, int nsplit,
                                 int part_size, float scale, hipStream_t st, bool kv8 = false) {
  if (nh % nkv) throw std::runtime_error("attn_decode: nh must be a multiple of nkv");
  if (nsplit > 1 && (!part_o || !part_ml)) throw std::runtime_error("attn_decode: split needs workspaces");
  if (B == 0) return;
  auto Q = (const bf16_t*)q;
  auto K = (bf16_t*)kc;
  auto V = (bf16_t*)vc;
  auto BT = (const int*)block_tables;
  auto CL = (const int*)ctx_lens;
  auto O = (bf16_t*)out;
  auto PO = (float*)part_o;
  auto PML = (float*)part_ml;
  switch (D) {
    case 64: launch_decode_d<64>(Q, q_stride, K, V, BT, bt_stride, CL, O, out_stride, PO, PML, B, nh, nkv, block_size, nsplit, part_size, scale, st, kv8); break;
    case 128: launch_decode_d<128>(Q, q_stride, K, V, BT, bt_stride, CL, O, out_stride, PO, PML, B, nh, nkv, block_size, nsplit, part_size, scale, st, kv8); break;
    case 256: launch_decode_d<256>(Q, q_stride, K, V, BT, bt_stride, CL, O, out_stride, PO, PML, B, nh, nkv, block_size, nsplit, part_size, scale, st, kv8); break;
    default: throw std::runtime_error("attn_decode: head_dim must be 64, 128 or 256");
  }
}

void launch_attn_decode(const void* q, int64_t q_stride, const void* kc, const void* vc, const void* block_tables,
                        int bt_stride, const void* ctx_lens, void* out, int64_t out_stride, void* part_o,
                        void* part_ml, int B, int nh, int nkv, int D, int block_size, int nsplit, int part_size,
                        float scale, hipStream_t st, bool kv8) {
  attn_decode_dispatch(q, q_stride, const_cast<void*>(kc), const_cast<void*>(vc), block_tables, bt_stride, ctx_lens,
                       out, out_stride, part_o, part_ml, B, nh, nkv, D, block_size, nsplit, part_size, scale, st,
                       kv8);
}
