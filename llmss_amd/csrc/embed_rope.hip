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

template <int STYLE>
__global__ __launch_bounds__(256) void rope_cache_kernel(bf16_t* __restrict__ qkv, int64_t row_stride,
                                                         const int64_t* __restrict__ pos, const float* __restrict__ cos_t,
                                                         const float* __restrict__ sin_t, bf16_t* __restrict__ kc,
                                                         bf16_t* __restrict__ vc, const int64_t* __restrict__ slot,
                                                         int nh, int nkv, int D, int rot, int block_size, int k_off,
                                                         int v_off, int do_rope, const float* __restrict__ part, int S,
                                                         int64_t slab, const bf16_t* __restrict__ bias) {
  const int t = blockIdx.x;
  const int oct = blockIdx.y * blockDim.x + threadIdx.x;
  const int OPH = D >> 3;  // octets per head
  const int nqk = (nh + nkv) * OPH;
  if (oct >= nqk + nkv * OPH) return;
  const int64_t s = slot ? slot[t] : -1;
  const int N = (nh + 2 * nkv) * D;
  const QkvIn in{qkv + t * row_stride, part ? part + (int64_t)t * N : nullptr, S, slab, bias};
  int64_t cbase = 0;
  if (s >= 0) {
    const int64_t blk = s / block_size, off = s % block_size;
    cbase = blk * nkv * (int64_t)block_size * D + off * (int64_t)D;  // + head*block_size*D + d
  }
  if (oct >= nqk) {  // v octet -> cache
    if (s < 0 && !part) return;
    const int v = oct - nqk, h = v / OPH, j = v % OPH;
    const int e = v_off + h * D + j * 8;
    float x[8];
    in.load<8>(e, x);
    if (part) store_bf16<8>(in.row + e, x);
    if (s >= 0) store_bf16<8>(vc + cbase + (int64_t)h * block_size * D + j * 8, x);
    return;
  }
  const int h = oct / OPH, j = oct % OPH;
  const bool is_k = h >= nh;
  const int hk = h - nh;
  const int hbase = is_k ? k_off + hk * D : h * D;  // element offset of the head in the row
  bf16_t* kdst = (is_k && s >= 0) ? kc + cbase + (int64_t)hk * block_size * D : nullptr;
  const int r8 = rot >> 3;
  if (j >= r8 || !do_rope) {  // pass-through octet (k needs a cache copy, partial input a write-back)
    if (kdst || part) {
      const int e = do_rope ? rot + 8 * (j - r8) : 8 * j;
      float x[8];
      in.load<8>(hbase + e, x);
      if (part) store_bf16<8>(in.row + hbase + e, x);
      if (kdst) store_bf16<8>(kdst + e, x);
    }
    return;
  }
  const int64_t p = pos[t];
  const int rh = rot >> 1;
  const f32x4 c = *reinterpret_cast<const f32x4*>(cos_t + p * rh + 4 * j);
  const f32x4 sn = *reinterpret_cast<const f32x4*>(sin_t + p * rh + 4 * j);
  if (STYLE == 1) {
    float x[8], y[8];
    in.load<8>(hbase + 8 * j, x);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      y[2 * i] = x[2 * i] * c[i] - x[2 * i + 1] * sn[i];
      y[2 * i + 1] = x[2 * i + 1] * c[i] + x[2 * i] * sn[i];
    }
    store_bf16<8>(in.row + hbase + 8 * j, y);
    if (kdst) store_bf16<8>(kdst + 8 * j, y);
  } else {
    float a[4], b[4], ya[4], yb[4];
    in.load<4>(hbase + 4 * j, a);
    in.load<4>(hbase + rh + 4 * j, b);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      ya[i] = a[i] * c[i] - b[i] * sn[i];
      yb[i] = b[i] * c[i] + a[i] * sn[i];
    }
    store_bf16<4>(in.row + hbase + 4 * j, ya);
    store_bf16<4>(in.row + hbase + rh + 4 * j, yb);
    if (kdst) {
      store_bf16<4>(kdst + 4 * j, ya);
      store_bf16<4>(kdst + rh + 4 * j, yb);
    }
  }
}

void launch_rope_cache(void* qkv, int64_t row_stride, const void* pos, const void* cos_t, const void* sin_t,
                       void* kc, void* vc, const void* slot, int T, int nh, int nkv, int D, int rot, int block_size,
                       int k_off, int v_off, int style, bool do_rope, const void* part, int S, int64_t slab,
                       const void* bias, hipStream_t st) {
  if (D % 8) throw std::runtime_error("rope_cache: head_dim must be a multiple of 8");
  if (do_rope && (rot % 8 || rot > D)) throw std::runtime_error("rope_cache: rotary_dim must be a multiple of 8");
  if (T == 0) return;
  const int octets = (nh + 2 * nkv) * (D / 8);
  dim3 grid(T, (octets + 255) / 256);
#define RC(STYLE_)                                                                                                     \
  rope_cache_kernel<STYLE_><<<grid, 256, 0, st>>>((bf16_t*)qkv, row_stride, (const int64_t*)pos, (const float*)cos_t,  \
                                                  (const float*)sin_t, (bf16_t*)kc, (bf16_t*)vc, (const int64_t*)slot, \
                                                  nh, nkv, D, rot, block_size, k_off, v_off, do_rope ? 1 : 0,          \
                                                  (const float*)part, S, slab, (const bf16_t*)bias)
  if (style == 1) RC(1);
  else RC(0);
#undef RC
  HIP_CHECK_LAUNCH();
}
