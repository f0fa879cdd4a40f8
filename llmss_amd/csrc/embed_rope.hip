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
//   qkv      [T, row_stride] bf16: q at col 0 (nh*D), k at q_off_k (nkv*D), v at q_off_v (nkv*D)
//   cos_sin  [max_pos, rot/2] fp32 each (host-precomputed table; no on-device trig, guide App. B)
//   k_cache / v_cache [num_blocks, nkv, block_size, D] bf16 (paged)
//   slot[t] = physical slot (block*block_size + offset), < 0 = do not cache (padding)
// q and k are rotated IN PLACE in qkv (prefill attention reads them from there); rotated k and
// raw v are also written to the paged cache. Styles: 0 = neox half-rotate, 1 = gptj interleaved.
// One thread per (head, rotation pair); launches one workgroup per token.
// ---------------------------------------------------------------------------------------------
template <int STYLE>
__global__ __launch_bounds__(256) void rope_cache_kernel(bf16_t* __restrict__ qkv, int64_t row_stride,
                                                         const int64_t* __restrict__ pos, const float* __restrict__ cos_t,
                                                         const float* __restrict__ sin_t, bf16_t* __restrict__ kc,
                                                         bf16_t* __restrict__ vc, const int64_t* __restrict__ slot,
                                                         int nh, int nkv, int D, int rot, int block_size, int k_off,
                                                         int v_off, int do_rope) {
  const int t = blockIdx.x;
  const int64_t p = do_rope ? pos[t] : 0;
  const int64_t s = slot ? slot[t] : -1;
  bf16_t* row = qkv + t * row_stride;
  const int half = D >> 1, rh = rot >> 1;
  const int total = (nh + nkv) * half;
  int64_t cbase = 0;
  if (s >= 0) {
    const int64_t blk = s / block_size, off = s % block_size;
    cbase = (blk * nkv) * (int64_t)block_size * D + off * (int64_t)D;  // + h*block_size*D + d
  }
  for (int i = threadIdx.x; i < total; i += blockDim.x) {
    const int h = i / half, pi = i - h * half;
    const bool is_k = h >= nh;
    const int hk = h - nh;
    bf16_t* base = is_k ? row + k_off + hk * D : row + h * D;
    int d0, d1;
    bool rotate;
    if (STYLE == 1) {  // gptj: pairs (2i, 2i+1) over the first rot dims
      d0 = 2 * pi; d1 = d0 + 1; rotate = d0 < rot;
    } else {  // neox: pairs (i, i+rot/2) for i < rot/2, then pass-through pairs
      if (pi < rh) { d0 = pi; d1 = pi + rh; rotate = true; }
      else { d0 = rot + 2 * (pi - rh); d1 = d0 + 1; rotate = false; }
    }
    float x0 = bf2f(base[d0]), x1 = bf2f(base[d1]);
    if (rotate && do_rope) {
      const int fi = STYLE == 1 ? pi : pi;  // frequency index
      const float c = cos_t[p * rh + fi], sn = sin_t[p * rh + fi];
      const float y0 = x0 * c - x1 * sn, y1 = x1 * c + x0 * sn;
      x0 = y0; x1 = y1;
      base[d0] = f2bf(x0);
      base[d1] = f2bf(x1);
    }
    if (is_k && s >= 0) {
      bf16_t* kdst = kc + cbase + (int64_t)hk * block_size * D;
      kdst[d0] = f2bf(x0);
      kdst[d1] = f2bf(x1);
    }
  }
  // V copy into the cache: 16 B per lane
  if (s >= 0) {
    const int vchunks = nkv * (D / 8);
    for (int i = threadIdx.x; i < vchunks; i += blockDim.x) {
      const int h = i / (D / 8), c = i - h * (D / 8);
      u16x8 v = *reinterpret_cast<const u16x8*>(row + v_off + h * D + c * 8);
      *reinterpret_cast<u16x8*>(vc + cbase + (int64_t)h * block_size * D + c * 8) = v;
    }
  }
}

void launch_rope_cache(void* qkv, int64_t row_stride, const void* pos, const void* cos_t, const void* sin_t,
                       void* kc, void* vc, const void* slot, int T, int nh, int nkv, int D, int rot, int block_size,
                       int k_off, int v_off, int style, bool do_rope, hipStream_t st) {
  if (D % 8) throw std::runtime_error("rope_cache: head_dim must be a multiple of 8");
  if (rot % 2 || rot > D) throw std::runtime_error("rope_cache: bad rotary_dim");
  if (T == 0) return;
  const int total = (nh + nkv) * (D / 2);
  const int threads = std::min(256, ((total + 63) / 64) * 64);
  if (style == 1)
    rope_cache_kernel<1><<<T, threads, 0, st>>>((bf16_t*)qkv, row_stride, (const int64_t*)pos, (const float*)cos_t,
                                                (const float*)sin_t, (bf16_t*)kc, (bf16_t*)vc, (const int64_t*)slot, nh,
                                                nkv, D, rot, block_size, k_off, v_off, do_rope ? 1 : 0);
  else
    rope_cache_kernel<0><<<T, threads, 0, st>>>((bf16_t*)qkv, row_stride, (const int64_t*)pos, (const float*)cos_t,
                                                (const float*)sin_t, (bf16_t*)kc, (bf16_t*)vc, (const int64_t*)slot, nh,
                                                nkv, D, rot, block_size, k_off, v_off, do_rope ? 1 : 0);
  HIP_CHECK_LAUNCH();
}
