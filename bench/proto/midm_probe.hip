// Standalone breakdown of the gemm_mid decode GEMM tiles at mid M (TP=8 shard decode: M = 256 / 512):
// each configuration runs as MODE 0 (the kernel), 1 (staging loads only, no MFMA), 2 (MFMAs only, no loads)
// and 3 (no epilogue stores), 20 launches per HIP graph, weights rotated over > 512 MB of copies.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../llmss_amd/csrc midm_probe.hip -o midm_probe
// Run:   ./midm_probe [tp1|gpt2] (one line per shape x tile x depth x split x mode; tp1: Llama-2-7B TP=1 at
//        M=64; gpt2: GPT-2-XL at M=64)
#include "gemm_mid.hip"

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

struct Shape {
  const char* name;
  int M, N, K;
};

template <int BM, int BN, int WM, int WN, int NS, int MODE>
static void launch(const bf16_t* X, const bf16_t* W, bf16_t* Y, float* part, int M, int N, int K, int split,
                   hipStream_t st) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  gemm_mid_kernel<BM, BN, WM, WN, NS, false, false, MODE><<<dim3(tiles, split), 64 * WM * WN, 0, st>>>(
      X, K, W, K, nullptr, Y, N, split > 1 ? part : nullptr, M, N, K, 0, 0, nullptr, QkvEpi{}, nullptr, nullptr, nullptr);
}

using Fn = void (*)(const bf16_t*, const bf16_t*, bf16_t*, float*, int, int, int, int, hipStream_t);

struct Cfg {
  const char* tile;
  int ns;
  Fn fn[4];
};

#define CFG(NAME, BM, BN, WM, WN, NS)                                                                        \
  Cfg {                                                                                                      \
    NAME, NS, {                                                                                              \
      launch<BM, BN, WM, WN, NS, 0>, launch<BM, BN, WM, WN, NS, 1>, launch<BM, BN, WM, WN, NS, 2>,           \
          launch<BM, BN, WM, WN, NS, 3>                                                                      \
    }                                                                                                        \
  }

int main(int argc, char** argv) {
  // default: the TP=8 shard of Llama-2-7B at M = 512; "tp1": Llama-2-7B TP=1 decode at M = 64
  const bool tp1 = argc > 1 && std::string(argv[1]) == "tp1";
  const bool gpt2 = argc > 1 && std::string(argv[1]) == "gpt2";  // GPT-2-XL TP=1 decode at M = 64
  const Shape shapes8[] = {{"qkv", 512, 1536, 4096}, {"o", 512, 4096, 512}, {"up", 512, 2752, 4096},
                           {"down", 512, 4096, 1376}};
  const Shape shapes1[] = {{"qkv", 64, 12288, 4096}, {"o", 64, 4096, 4096}, {"up", 64, 22016, 4096},
                           {"down", 64, 4096, 11008}};
  const Cfg cfgs8[] = {CFG("64x128", 64, 128, 1, 4, 4), CFG("128x128", 128, 128, 2, 2, 3),
                       CFG("128x128", 128, 128, 2, 2, 5), CFG("256x128", 256, 128, 4, 2, 3),
                       CFG("128x256", 128, 256, 2, 4, 3)};
  const Cfg cfgs1[] = {CFG("64x192", 64, 192, 2, 2, 3), CFG("64x96", 64, 96, 4, 1, 3), CFG("64x96", 64, 96, 4, 1, 4),
                       CFG("64x128", 64, 128, 1, 4, 3), CFG("64x256", 64, 256, 1, 4, 3), CFG("64x32", 64, 32, 4, 1, 4),
                       CFG("64x32", 64, 32, 4, 1, 6)};
  const int splits8[] = {1, 2, 4, 8};
  const int splits1[] = {1, 2, 4};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t maxw = tp1 ? (size_t)22016 * 4096 : (size_t)6400 * 1600 > (size_t)4096 * 4096 ? (size_t)6400 * 1600 : (size_t)4096 * 4096;
  const int ncopy = tp1 ? 8 : 48;  // > 512 MB of rotating weight copies for the large shapes
  std::vector<bf16_t*> ws(ncopy);
  for (auto& w : ws) {
    CK(hipMalloc(&w, maxw * 2));
    CK(hipMemset(w, 0x3c, maxw * 2));
  }
  bf16_t *X, *Y;
  float* part;
  CK(hipMalloc(&X, (size_t)512 * 11008 * 2));
  CK(hipMemset(X, 0x3c, (size_t)512 * 11008 * 2));
  CK(hipMalloc(&Y, (size_t)512 * 22016 * 2));
  CK(hipMalloc(&part, (size_t)8 * 512 * 22016 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 24;
  const Shape shapesg[] = {{"qkv", 64, 4800, 1600}, {"o", 64, 1600, 1600}, {"up", 64, 6400, 1600},
                           {"down", 64, 1600, 6400}};
  const Cfg cfgsg[] = {CFG("64x32", 64, 32, 4, 1, 3), CFG("64x32", 64, 32, 4, 1, 4), CFG("64x32", 64, 32, 4, 1, 6),
                       CFG("64x48", 64, 48, 2, 1, 4), CFG("64x48", 64, 48, 2, 1, 6), CFG("64x96", 64, 96, 4, 1, 4)};
  const int splitsg[] = {1, 2, 3, 4, 6, 8};
  std::vector<Shape> shapes(tp1 ? std::begin(shapes1) : std::begin(shapes8), tp1 ? std::end(shapes1) : std::end(shapes8));
  std::vector<Cfg> cfgs(tp1 ? std::begin(cfgs1) : std::begin(cfgs8), tp1 ? std::end(cfgs1) : std::end(cfgs8));
  std::vector<int> splits(tp1 ? std::begin(splits1) : std::begin(splits8), tp1 ? std::end(splits1) : std::end(splits8));
  if (gpt2) {
    shapes.assign(std::begin(shapesg), std::end(shapesg));
    cfgs.assign(std::begin(cfgsg), std::end(cfgsg));
    splits.assign(std::begin(splitsg), std::end(splitsg));
  }
  for (const auto& s : shapes) {
    for (const auto& c : cfgs) {
      for (int split : splits) {
        if ((s.K / 64) / split < 2) continue;
        if ((size_t)s.N * s.K > maxw) continue;
        printf("%-5s M=%d N=%d K=%d %-8s ns=%d split=%d:", s.name, s.M, s.N, s.K, c.tile, c.ns, split);
        for (int mode = 0; mode < 4; ++mode) {
          hipGraph_t g;
          hipGraphExec_t ge;
          CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
          for (int i = 0; i < iters; ++i) c.fn[mode](X, ws[i % ncopy], Y, part, s.M, s.N, s.K, split, st);
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
          printf(" %s %6.2f", mode == 0 ? "full" : mode == 1 ? "loads" : mode == 2 ? "mfma" : "no-epi",
                 best * 1e3f / iters);
        }
        printf(" us\n");
        fflush(stdout);
      }
    }
  }
  return 0;
}
