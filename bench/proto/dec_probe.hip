// Breakdown of the K-split-wave decode GEMM (llmss_amd/csrc/gemm_dec.hip) on GPT-2-XL's M = 64 shapes: each
// configuration as MODE 0 (the kernel), 1 (weight loads only), 2 (activation loads only), 3 (no loads), 4 (no
// epilogue stores) and "mall" (the kernel on ONE weight copy: Infinity-Cache resident), 24 launches per HIP graph,
// weights otherwise rotated over > 512 MB; plus an empty kernel (the launch floor).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../llmss_amd/csrc dec_probe.hip -o dec_probe
#include "gemm_dec.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1000) p[0] = 1;
}

template <int MT, int BN, int NS, int MODE>
static void launch(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* part, int M, int N, int K, int split,
                   hipStream_t st) {
  dim3 grid((N + BN - 1) / BN, split);
  gemm_dec_kernel<MT, BN, NS, MODE><<<grid, 256, 0, st>>>(X, K, W, K, nullptr, Y, N, split > 1 ? part : nullptr, M, N,
                                                          K, 0, 0, QkvEpi{}, nullptr);
}

using Fn = void (*)(const bf16_t*, const bf16_t*, bf16_t*, float*, int, int, int, int, hipStream_t);
struct Cfg {
  const char* name;
  int bn, ns;
  Fn fn[5];
};
#define CFG(BN, NS) \
  Cfg { "64x" #BN, BN, NS, {launch<4, BN, NS, 0>, launch<4, BN, NS, 1>, launch<4, BN, NS, 2>, launch<4, BN, NS, 3>, launch<4, BN, NS, 4>} }

int main() {
  struct Shape {
    const char* name;
    int M, N, K;
    int splits[4];
  };
  const Shape shapes[] = {{"qkv", 64, 4800, 1600, {1, 2, 3, 5}}, {"o", 64, 1600, 1600, {2, 5, 8, 0}},
                          {"up", 64, 6400, 1600, {1, 2, 0, 0}}, {"down", 64, 1600, 6400, {4, 5, 8, 10}}};
  const Cfg cfgs[] = {CFG(16, 4), CFG(32, 3), CFG(48, 2), CFG(64, 2)};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t maxw = (size_t)6400 * 1600;
  const int ncopy = 40;
  std::vector<bf16_t*> ws(ncopy);
  for (auto& w : ws) {
    CK(hipMalloc(&w, maxw * 2));
    CK(hipMemset(w, 0x3c, maxw * 2));
  }
  bf16_t *X, *Y;
  float* part;
  CK(hipMalloc(&X, (size_t)64 * 6400 * 2));
  CK(hipMemset(X, 0x3c, (size_t)64 * 6400 * 2));
  CK(hipMalloc(&Y, (size_t)64 * 6400 * 2));
  CK(hipMalloc(&part, (size_t)16 * 64 * 6400 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 24;
  auto timed = [&](auto&& body) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    for (int i = 0; i < iters; ++i) body(i);
    CK(hipStreamEndCapture(st, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, st));
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0, st));
      CK(hipGraphLaunch(ge, st));
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = std::min(best, ms);
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return best * 1e3f / iters;
  };
  for (int grid : {64, 256, 1024})
    printf("empty kernel grid %4d: %6.2f us\n", grid, timed([&](int) { empty_kernel<<<grid, 256, 0, st>>>(nullptr); }));
  fflush(stdout);
  for (const auto& s : shapes) {
    for (const auto& c : cfgs) {
      for (int split : s.splits) {
        if (split == 0) continue;
        printf("%-5s N=%d K=%d %-6s ns=%d split=%d grid=%d:", s.name, s.N, s.K, c.name, c.ns, split,
               (s.N + c.bn - 1) / c.bn * split);
        for (int mode = 0; mode < 5; ++mode) {
          const float us = timed([&](int i) { c.fn[mode](X, ws[i % ncopy], Y, part, s.M, s.N, s.K, split, st); });
          printf(" %s %6.2f", mode == 0 ? "full" : mode == 1 ? "Bonly" : mode == 2 ? "Aonly" : mode == 3 ? "noload" : "noepi",
                 us);
        }
        printf(" mall %6.2f us\n", timed([&](int) { c.fn[0](X, ws[0], Y, part, s.M, s.N, s.K, split, st); }));
        fflush(stdout);
      }
    }
  }
  return 0;
}
