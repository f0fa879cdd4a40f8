// Token/position embedding gather and the fused RoPE + paged-KV-cache write
// (K8/K10; reference: gptj_modeling.py:26-47,199-236 builds fp32 sin/cos on the CPU, applies a
// repeat_interleave'd rotate_every_two and torch.cat's the KV cache every step, O(T) per token;
// gpt_bigcode_modeling.py:288-292 concatenates a [B,T,2D] cache).
//
// The embedding table is replicated per rank (288 GB HBM makes the 131-262 MB table cheap), so
// no all-reduce follows it (the reference all-reduces a vocab-parallel embedding, C1).
#include "common.h"
#include <stdexcept>
#include <string>

// out[t] = wte[ids[t]] (+ wpe[pos[t]])
__global__ __launch_bounds__(256) void embed_kernel(const int64_t* __restrict__ ids, const int64_t* __restrict__ pos,
                                                    const bf16_t* __restrict__ wte, const bf16_t* __restrict__ wpe,
                                                    bf16_t* __restrict__ out, int H, int vocab) {
  const int t = blockIdx.x;
  int64_t id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const bf16_t* src = wte + id * (int64_t)H;
  const bf16_t* psrc = wpe ? wpe + pos[t] * (int64_t)H : nullptr;
  for (int c = threadIdx.x; c < H / 8; c += blockDim.x) {
    u16x8 a = *reinterpret_cast<const u16x8*>(src + c * 8);
    if (psrc) {
      u16x8 p = *reinterpret_cast<const u16x8*>(psrc + c * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = f2bf(bf2f(a[j]) + bf2f(p[j]));
    }
    *reinterpret_cast<u16x8*>(out + (int64_t)t * H + c * 8) = a;
  }
}

void launch_embed(const void* ids, const void* pos, const void* wte, const void* wpe, void* out, int T, int H,
                  int vocab, hipStream_t st) {
  if (H % 8) throw std::runtime_error("embed: hidden must be a multiple of 8");
  if (T == 0) return;
  int threads = std::min(256, ((H / 8 + 63) / 64) * 64);
  embed_kernel<<<T, threads, 0, st>>>((const int64_t*)ids, (const int64_t*)pos, (const bf16_t*)wte,
                                      (const bf16_t*)wpe, (bf16_t*)out, H, vocab);
  HIP_CHECK_LAUNCH();
}

// ---------------------------------------------------------------------------------------------
// RoPE + KV-cache write.
//   qkv      [T, row_stride] bf16: q at col 0 (nh*D), k at k_off (nkv*D), v at v_off (nkv*D)
//   cos_sin  [max_pos, rot/2] fp32 each (host-precomputed table; no on-device trig, guide App. B)
//   k_cache / v_cache [num_blocks, nkv, block_size, D] bf16 (paged)
//   slot[t] = physical slot (block*block_size + offset), < 0 = do not cache (padding)
// q and k are rotated IN PLACE in qkv (prefill attention reads them from there); rotated k and
// raw v are also written to the paged cache. Styles: 0 = neox half-rotate, 1 = gptj interleaved.
// One thread per 16-byte "octet" of the token's q|k|v row (4 rotation pairs):
//   neox  octet j < rot/8 of a head: elements [4j, 4j+4) and [rot/2 + 4j, +4) (two 8-B accesses)
//   gptj  octet j < rot/8 of a head: elements [8j, 8j+8) = pairs (8j+2i, 8j+2i+1) (one 16-B access)
//   j >= rot/8: pass-through octet [rot + 8(j - rot/8), +8); v octets: copied to the cache.
// grid (T, ceil(octets / 256)): all octets of all tokens in flight at once.
// Split-K input (part != nullptr): the QKV GEMM left S fp32 slabs [S, T, N] (+ bias); the sum is
// formed here (rounded to bf16 like the GEMM epilogue would) and written back to qkv, so the
// GEMM's separate reduce launch disappears (guide: combine in the next kernel's prologue).
// ---------------------------------------------------------------------------------------------
struct QkvIn {
  bf16_t* row;        // token's qkv row (bf16; always the destination)
  const float* part;  // token's row in slab 0, or nullptr
  int S;
  int64_t slab;
  const bf16_t* bias;

  template <int W>
  __device__ __forceinline__ void load(int e, float (&v)[W]) const {
    if (part) {
#pragma unroll
      for (int i = 0; i < W; ++i) v[i] = 0.f;
      // up to 8 slabs issued together (a runtime-bounded loop would serialise one round trip per slab)
      f32x4 x[8][W / 4];
#pragma unroll
      for (int z = 0; z < 8; ++z)
#pragma unroll
        for (int q = 0; q < W / 4; ++q)
          x[z][q] = *reinterpret_cast<const f32x4*>(part + min(z, S - 1) * slab + e + 4 * q);
#pragma unroll
      for (int z = 0; z < 8; ++z)
#pragma unroll
        for (int q = 0; q < W / 4; ++q)
#pragma unroll
          for (int i = 0; i < 4; ++i) v[4 * q + i] += z < S ? x[z][q][i] : 0.f;
      for (int z = 8; z < S; ++z)
#pragma unroll
        for (int q = 0; q < W / 4; ++q) {
          const f32x4 y = *reinterpret_cast<const f32x4*>(part + z * slab + e + 4 * q);
#pragma unroll
          for (int i = 0; i < 4; ++i) v[4 * q + i] += y[i];
        }
#pragma unroll
      for (int i = 0; i < W; ++i) v[i] = bf2f(f2bf(v[i] + (bias ? bf2f(bias[e + i]) : 0.f)));
    } else if constexpr (W == 8) {
      const u16x8 x = *reinterpret_cast<const u16x8*>(row + e);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = bf2f(x[i]);
    } else {
      const u16x4 x = *reinterpret_cast<const u16x4*>(row + e);
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = bf2f(x[i]);
    }
  }
};

template <int W>
__device__ __forceinline__ void store_bf16(bf16_t* dst, const float (&v)[W]) {
  if constexpr (W == 8) {
    u16x8 x;
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] = f2bf(v[i]);
    *reinterpret_cast<u16x8*>(dst) = x;
  } else {
    u16x4 x;
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = f2bf(v[i]);
    *reinterpret_cast<u16x4*>(dst) = x;
  }
}

// fp8 KV rows (KV8): one (token, kv head) row = D e4m3 bytes + a 16-B tail whose first 4 bytes hold the
// row's fp32 scale = absmax / 448 (ops/reference.py kv_rows_quant). The OPH threads of a head (one octet
// each, consecutive lanes) reduce the absmax with shuffles; y[0..3] land at element e0, y[4..7] at e1.
__device__ __forceinline__ void kv8_store_row(unsigned char* row, int D, int e0, int e1, const float (&y)[8], int j,
                                              int oph) {
  float f[8], am = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    f[i] = bf2f(f2bf(y[i]));  // the bf16 value a bf16 cache would hold
    am = fmaxf(am, fabsf(f[i]));
  }
  for (int o = 1; o < oph; o <<= 1) am = fmaxf(am, __shfl_xor(am, o, 64));
  const float sc = am > 0.f ? am / 448.f : 1.f, inv = 1.f / sc;
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = fminf(fmaxf(f[i] * inv, -448.f), 448.f);
  unsigned lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[4], f[5], hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(f[6], f[7], hi, true);
  if (e1 == e0 + 4) {
    *reinterpret_cast<uint2*>(row + e0) = make_uint2(lo, hi);
  } else {
    *reinterpret_cast<unsigned*>(row + e0) = lo;
    *reinterpret_cast<unsigned*>(row + e1) = hi;
  }
  if (j == 0) *reinterpret_cast<f32x4*>(row + D) = f32x4{sc, 0.f, 0.f, 0.f};
}

template <int STYLE, bool KV8>
__global__ __launch_bounds__(256) void rope_cache_kernel(bf16_t* __restrict__ qkv, int64_t row_stride,
                                                         const int64_t* __restrict__ pos, const float* __restrict__ cos_t,
                                                         const float* __restrict__ sin_t, void* __restrict__ kc,
                                                         void* __restrict__ vc, const int64_t* __restrict__ slot,
                                                         int nh, int nkv, int D, int rot, int block_size, int k_off,
                                                         int v_off, int do_rope, const float* __restrict__ part, int S,
                                                         int64_t slab, const bf16_t* __restrict__ bias) {
  const int t = blockIdx.x;
  const int oct = blockIdx.y * blockDim.x + threadIdx.x;
  const int OPH = D >> 3;  // octets per head (consecutive lanes; heads never straddle a workgroup)
  const int nqk = (nh + nkv) * OPH;
  if (oct >= nqk + nkv * OPH) return;
  const int64_t s = slot ? slot[t] : -1;
  const int N = (nh + 2 * nkv) * D;
  const QkvIn in{qkv + t * row_stride, part ? part + (int64_t)t * N : nullptr, S, slab, bias};
  const int RB = KV8 ? D + 16 : D;  // cache row (elements of the cache dtype)
  int64_t cbase = 0;
  if (s >= 0) {
    const int64_t blk = s / block_size, off = s % block_size;
    cbase = blk * nkv * (int64_t)block_size * RB + off * (int64_t)RB;  // + head*block_size*RB + d
  }
  if (oct >= nqk) {  // v octet -> cache
    if (s < 0 && !part) return;
    const int v = oct - nqk, h = v / OPH, j = v % OPH;
    const int e = v_off + h * D + j * 8;
    float x[8];
    in.load<8>(e, x);
    if (part) store_bf16<8>(in.row + e, x);
    if (s >= 0) {
      if constexpr (KV8) kv8_store_row((unsigned char*)vc + cbase + (int64_t)h * block_size * RB, D, j * 8, j * 8 + 4, x, j, OPH);
      else store_bf16<8>((bf16_t*)vc + cbase + (int64_t)h * block_size * RB + j * 8, x);
    }
    return;
  }
  const int h = oct / OPH, j = oct % OPH;
  const bool is_k = h >= nh;
  const int hk = h - nh;
  const int hbase = is_k ? k_off + hk * D : h * D;  // element offset of the head in the row
  const bool to_cache = is_k && s >= 0;             // uniform over the head's OPH lanes
  const int64_t kbase = cbase + (int64_t)hk * block_size * RB;
  const int r8 = rot >> 3;
  float y[8];
  int e0, e1;
  if (j >= r8 || !do_rope) {  // pass-through octet (k needs a cache copy, partial input a write-back)
    if (!to_cache && !part) return;
    e0 = do_rope ? rot + 8 * (j - r8) : 8 * j;
    e1 = e0 + 4;
    in.load<8>(hbase + e0, y);
    if (part) store_bf16<8>(in.row + hbase + e0, y);
  } else {
    const int64_t p = pos[t];
    const int rh = rot >> 1;
    const f32x4 c = *reinterpret_cast<const f32x4*>(cos_t + p * rh + 4 * j);
    const f32x4 sn = *reinterpret_cast<const f32x4*>(sin_t + p * rh + 4 * j);
    if (STYLE == 1) {
      float x[8];
      in.load<8>(hbase + 8 * j, x);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        y[2 * i] = x[2 * i] * c[i] - x[2 * i + 1] * sn[i];
        y[2 * i + 1] = x[2 * i + 1] * c[i] + x[2 * i] * sn[i];
      }
      store_bf16<8>(in.row + hbase + 8 * j, y);
      e0 = 8 * j;
      e1 = e0 + 4;
    } else {
      float a[4], b[4], ya[4], yb[4];
      in.load<4>(hbase + 4 * j, a);
      in.load<4>(hbase + rh + 4 * j, b);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ya[i] = a[i] * c[i] - b[i] * sn[i];
        yb[i] = b[i] * c[i] + a[i] * sn[i];
        y[i] = ya[i];
        y[4 + i] = yb[i];
      }
      store_bf16<4>(in.row + hbase + 4 * j, ya);
      store_bf16<4>(in.row + hbase + rh + 4 * j, yb);
      e0 = 4 * j;
      e1 = rh + 4 * j;
    }
  }
  if (!to_cache) return;
  if constexpr (KV8) {
    kv8_store_row((unsigned char*)kc + kbase, D, e0, e1, y, j, OPH);
  } else {
    bf16_t* kdst = (bf16_t*)kc + kbase;
    if (e1 == e0 + 4) {
      store_bf16<8>(kdst + e0, y);
    } else {
      float ya[4] = {y[0], y[1], y[2], y[3]}, yb[4] = {y[4], y[5], y[6], y[7]};
      store_bf16<4>(kdst + e0, ya);
      store_bf16<4>(kdst + e1, yb);
    }
  }
}

void launch_rope_cache(void* qkv, int64_t row_stride, const void* pos, const void* cos_t, const void* sin_t,
                       void* kc, void* vc, const void* slot, int T, int nh, int nkv, int D, int rot, int block_size,
                       int k_off, int v_off, int style, bool do_rope, const void* part, int S, int64_t slab,
                       const void* bias, hipStream_t st, bool kv8) {
  if (D % 8) throw std::runtime_error("rope_cache: head_dim must be a multiple of 8");
  if (do_rope && (rot % 8 || rot > D)) throw std::runtime_error("rope_cache: rotary_dim must be a multiple of 8");
  if (kv8 && (D % 16 || 256 % (D / 8))) throw std::runtime_error("rope_cache: fp8 KV needs head_dim 16..2048, /16");
  if (T == 0) return;
  const int octets = (nh + 2 * nkv) * (D / 8);
  dim3 grid(T, (octets + 255) / 256);
#define RC(STYLE_, KV8_)                                                                                              \
  rope_cache_kernel<STYLE_, KV8_><<<grid, 256, 0, st>>>((bf16_t*)qkv, row_stride, (const int64_t*)pos,               \
                                                        (const float*)cos_t, (const float*)sin_t, kc, vc,            \
                                                        (const int64_t*)slot, nh, nkv, D, rot, block_size, k_off,    \
                                                        v_off, do_rope ? 1 : 0, (const float*)part, S, slab,         \
                                                        (const bf16_t*)bias)
  if (kv8) {
    if (style == 1) RC(1, true);
    else RC(0, true);
  } else {
    if (style == 1) RC(1, false);
    else RC(0, false);
  }
#undef RC
  HIP_CHECK_LAUNCH();
}
