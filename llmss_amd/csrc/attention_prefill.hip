// Causal variable-length flash-attention forward for prefill on MFMA (SURVEY K11-K14 for
// S>1; reference materialises the [S,T] score matrix in fp32 with a CPU-built causal mask,
// gptj_modeling.py:128-169, gpt_bigcode_modeling.py:170-246).
//
// Layout: q/k/v are read straight from the fused QKV GEMM output [T, row_stride] (no
// split/permute copies, K9), sequences are packed back to back (cu_seqlens), GQA/MQA via
// kv_head = head / (nh / nkv). Output [T, nh*D] bf16 feeds the O-projection GEMM.
//
// Formulation ("swapped" products, guide §3 / T12 idea): per wave 16 query rows,
//   S^T[key][q] = K · Q^T          (A = K rows from LDS via ds_read_b128, B = Q^T in registers)
//   O^T[d][q]  += V^T · P^T        (A = V^T via ds_read_b64_tr_b16 transpose reads, B = P^T
//                                   taken straight from the S^T accumulators, no LDS trip)
// With S^T in the mfma_f32_16x16x32 C layout each lane owns ONE query row (lane & 15) and 16
// keys, so the online-softmax row max/sum is 15 in-register ops + 2 shuffles, and the P^T
// operand needs no data movement: the k-order permutation it implies is applied identically
// to the V^T operand through the addresses of the transpose reads.
// K/V tiles of 64 keys are register-staged into LDS rows padded by 32 B (conflict-free for
// both the b128 row reads and the tr_b16 column reads at D=128).
#include "common.h"

constexpr float kLog2eP = 1.4426950408889634f;

template <int D>
__global__ __launch_bounds__(256) void attn_prefill_kernel(const bf16_t* __restrict__ qkv, int64_t row_stride,
                                                           const int* __restrict__ cu_seqlens, bf16_t* __restrict__ out,
                                                           int64_t out_stride, int nh, int nkv, int k_off, int v_off,
                                                           float scale_log2) {
  constexpr int BQ = 64, BKV = 64;
  constexpr int LD = D + 16;  // padded LDS row (elements)
  __shared__ __attribute__((aligned(16))) bf16_t Ks[BKV * LD];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[BKV * LD];

  const int qb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int tok0 = cu_seqlens[b];
  const int len = cu_seqlens[b + 1] - tok0;
  if (qb * BQ >= len) return;
  const int kvh = h / (nh / nkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int li = lane & 15, g = lane >> 4;
  const int qrow = qb * BQ + w * 16 + li;  // this lane's query row within the sequence
  const bool qvalid = qrow < len;

  // Q^T fragments (B operand): lane holds Q[qrow][32ks + 8g .. +7]
  s16x8 qf[D / 32];
  {
    const bf16_t* qp = qkv + (int64_t)(tok0 + (qvalid ? qrow : len - 1)) * row_stride + (int64_t)h * D + 8 * g;
#pragma unroll
    for (int ks = 0; ks < D / 32; ++ks) qf[ks] = *reinterpret_cast<const s16x8*>(qp + 32 * ks);
  }
  f32x4 o[D / 16];
#pragma unroll
  for (int i = 0; i < D / 16; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -1.0e30f, lsum = 0.f;

  const int kv_end = min(len, qb * BQ + BQ);  // causal: keys < last query row of the block
  const int q_hi = qb * BQ + w * 16 + 15;     // last query row of this wave
  constexpr int CH = D / 8;                   // 16-B chunks per row
  for (int kv0 = 0; kv0 < kv_end; kv0 += BKV) {
    // ---- stage K, V tile (register staging) -----------------------------------------------
    __syncthreads();
#pragma unroll
    for (int c = threadIdx.x; c < BKV * CH; c += 256) {
      const int r = c / CH, ch = c % CH;
      const int kr = min(kv0 + r, len - 1);
      const bf16_t* src = qkv + (int64_t)(tok0 + kr) * row_stride + (int64_t)kvh * D + ch * 8;
      *reinterpret_cast<u16x8*>(&Ks[r * LD + ch * 8]) = *reinterpret_cast<const u16x8*>(src + k_off);
      *reinterpret_cast<u16x8*>(&Vs[r * LD + ch * 8]) = *reinterpret_cast<const u16x8*>(src + v_off);
    }
    __syncthreads();
    if (kv0 > q_hi) continue;  // whole tile is in this wave's causal future (keep barriers uniform)

    // ---- S^T = K Q^T : 4 key tiles of 16 ------------------------------------------------------
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
    // ---- mask + online softmax (lane owns query row qrow, keys kv0 + 16kt + 4g + i) ----------
    float mx = m;
#pragma unroll
    for (int kt = 0; kt < 4; ++kt)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kv0 + kt * 16 + 4 * g + i;
        float v = s[kt][i] * scale_log2;
        v = (key <= qrow) ? v : -1.0e30f;
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

    // ---- O^T += V^T P^T --------------------------------------------------------------------
    // transpose-read addresses: lane (4q + p) of its 16-lane group supplies row q, cols 4p..4p+3
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
  if (!qvalid) return;
  const float inv = lsum > 0.f ? 1.f / lsum : 0.f;
  bf16_t* op = out + (int64_t)(tok0 + qrow) * out_stride + (int64_t)h * D + 4 * g;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    u16x4 r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = f2bf(o[dt][i] * inv);
    *reinterpret_cast<u16x4*>(op + dt * 16) = r;
  }
}

void launch_attn_prefill(const void* qkv, int64_t row_stride, const void* cu_seqlens, void* out, int64_t out_stride,
                         int B, int max_seqlen, int nh, int nkv, int D, int k_off, int v_off, float scale,
                         hipStream_t st) {
  if (nh % nkv) throw std::runtime_error("attn_prefill: nh must be a multiple of nkv");
  if (B == 0 || max_seqlen == 0) return;
  dim3 grid((max_seqlen + 63) / 64, nh, B);
  auto Q = (const bf16_t*)qkv;
  auto CU = (const int*)cu_seqlens;
  auto O = (bf16_t*)out;
  const float sl = scale * kLog2eP;
  switch (D) {
    case 64: attn_prefill_kernel<64><<<grid, 256, 0, st>>>(Q, row_stride, CU, O, out_stride, nh, nkv, k_off, v_off, sl); break;
    case 128: attn_prefill_kernel<128><<<grid, 256, 0, st>>>(Q, row_stride, CU, O, out_stride, nh, nkv, k_off, v_off, sl); break;
    case 256: attn_prefill_kernel<256><<<grid, 256, 0, st>>>(Q, row_stride, CU, O, out_stride, nh, nkv, k_off, v_off, sl); break;
    default: throw std::runtime_error("attn_prefill: head_dim must be 64, 128 or 256");
  }
  HIP_CHECK_LAUNCH();
}
