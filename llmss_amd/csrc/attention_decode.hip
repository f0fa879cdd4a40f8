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

template <int D, int GB, int UNROLL>
__global__ __launch_bounds__(256) void attn_decode_kernel(
    const bf16_t* __restrict__ q, int64_t q_stride, const bf16_t* __restrict__ kc, const bf16_t* __restrict__ vc,
    const int* __restrict__ block_tables, int bt_stride, const int* __restrict__ ctx_lens, bf16_t* __restrict__ out,
    int64_t out_stride, float* __restrict__ part_o, float* __restrict__ part_ml, int nh, int nkv, int G, int ngroups,
    int block_size, int part_size, float scale_log2) {
  constexpr int LPT = D / 8;
  constexpr int TPW = 64 / LPT;
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
  const int64_t head_off = (int64_t)kvh * block_size * D + sub * 8;
  const int64_t page_stride = (int64_t)nkv * block_size * D;
  constexpr int STEP = 4 * TPW;  // tokens per workgroup-iteration

  for (int tb = start + w * TPW + slot; tb < end; tb += STEP * UNROLL) {
    u16x8 kv[UNROLL], vv[UNROLL];
    bool ok[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const int t = tb + u * STEP;
      ok[u] = t < end;
      const int tt = ok[u] ? t : start;
      const int page = bt[tt / block_size];
      const int64_t a = page * page_stride + head_off + (int64_t)(tt % block_size) * D;
      kv[u] = *reinterpret_cast<const u16x8*>(kc + a);
      vv[u] = *reinterpret_cast<const u16x8*>(vc + a);
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      float kf[8], vf[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) { kf[j] = bf2f(kv[u][j]); vf[j] = bf2f(vv[u][j]); }
#pragma unroll
      for (int h = 0; h < GB; ++h) {
        float s = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) s = fmaf(qv[h][j], kf[j], s);
#pragma unroll
        for (int o = 1; o < LPT; o <<= 1) s += __shfl_xor(s, o, 64);
        if (ok[u]) {
          const float mn = fmaxf(m[h], s);
          const float alpha = exp2f(m[h] - mn), p = exp2f(s - mn);
          l[h] = l[h] * alpha + p;
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[h][j] = fmaf(acc[h][j], alpha, p * vf[j]);
          m[h] = mn;
        }
      }
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

template <int D, int GB>
static void launch_decode_t(const bf16_t* q, int64_t qs, const bf16_t* kc, const bf16_t* vc, const int* bt, int bts,
                            const int* cl, bf16_t* out, int64_t os, float* po, float* pml, int B, int nh, int nkv,
                            int bs, int nsplit, int psize, float scale, hipStream_t st) {
  const int G = nh / nkv;
  const int ngroups = (G + GB - 1) / GB;
  dim3 grid(B, nkv * ngroups, nsplit);
  attn_decode_kernel<D, GB, 2><<<grid, 256, 0, st>>>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, nh, nkv, G, ngroups,
                                                     bs, psize, scale * kLog2e);
  HIP_CHECK_LAUNCH();
  if (nsplit > 1) {
    attn_decode_reduce_kernel<D><<<dim3(B, nh), std::min(D, 256), 0, st>>>(po, pml, out, os, nh, nsplit);
    HIP_CHECK_LAUNCH();
  }
}

template <int D>
static void launch_decode_d(const bf16_t* q, int64_t qs, const bf16_t* kc, const bf16_t* vc, const int* bt, int bts,
                            const int* cl, bf16_t* out, int64_t os, float* po, float* pml, int B, int nh, int nkv,
                            int bs, int nsplit, int psize, float scale, hipStream_t st) {
  const int G = nh / nkv;
  if (G == 1) launch_decode_t<D, 1>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st);
  else if (G == 2) launch_decode_t<D, 2>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st);
  else if (G <= 4) launch_decode_t<D, 4>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st);
  else launch_decode_t<D, 8>(q, qs, kc, vc, bt, bts, cl, out, os, po, pml, B, nh, nkv, bs, nsplit, psize, scale, st);
}

void launch_attn_decode(const void* q, int64_t q_stride, const void* kc, const void* vc, const void* block_tables,
                        int bt_stride, const void* ctx_lens, void* out, int64_t out_stride, void* part_o,
                        void* part_ml, int B, int nh, int nkv, int D, int block_size, int nsplit, int part_size,
                        float scale, hipStream_t st) {
  if (nh % nkv) throw std::runtime_error("attn_decode: nh must be a multiple of nkv");
  if (nsplit > 1 && (!part_o || !part_ml)) throw std::runtime_error("attn_decode: split needs workspaces");
  if (B == 0) return;
  auto Q = (const bf16_t*)q;
  auto K = (const bf16_t*)kc;
  auto V = (const bf16_t*)vc;
  auto BT = (const int*)block_tables;
  auto CL = (const int*)ctx_lens;
  auto O = (bf16_t*)out;
  auto PO = (float*)part_o;
  auto PML = (float*)part_ml;
  switch (D) {
    case 64: launch_decode_d<64>(Q, q_stride, K, V, BT, bt_stride, CL, O, out_stride, PO, PML, B, nh, nkv, block_size, nsplit, part_size, scale, st); break;
    case 128: launch_decode_d<128>(Q, q_stride, K, V, BT, bt_stride, CL, O, out_stride, PO, PML, B, nh, nkv, block_size, nsplit, part_size, scale, st); break;
    case 256: launch_decode_d<256>(Q, q_stride, K, V, BT, bt_stride, CL, O, out_stride, PO, PML, B, nh, nkv, block_size, nsplit, part_size, scale, st); break;
    default: throw std::runtime_error("attn_decode: head_dim must be 64, 128 or 256");
  }
}
