// W8A8 gemm_mid tiles on the Llama-2-70B fp8 TP=8 shard shapes (M = 512 decode rows per rank): the plain k-loop
// against the software-pipelined one (ilv), per tile / ring depth / split, 16 launches per HIP graph, weights
// rotated over > 512 MB of copies. Also checks that both loops give bit-identical outputs (same MFMA order per
// accumulator).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../llmss_amd/csrc f8_probe.hip -o f8_probe
#include "gemm_mid.hip"

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

int main() {
  struct Shape {
    const char* name;
    int M, N, K, glu;
  };
  const Shape shapes[] = {{"gate_up", 512, 7168, 8192, 1}, {"down", 512, 8192, 3584, 0}, {"qkv", 512, 1280, 8192, 0},
                          {"o", 512, 8192, 1024, 0}};
  struct Cfg {
    const char* name;
    int tsel;
  };
  const Cfg cfgs[] = {{"128x128", 8}, {"64x128", 11}, {"256x128", 9}, {"128x256", 12}, {"64x256", 10}};
  hipStream_t st;
  CK(hipStreamCreate(&st));
  const size_t maxw = (size_t)8192 * 8192;
  const int ncopy = 10;
  std::vector<unsigned char*> ws(ncopy);
  std::vector<unsigned char> hw(maxw);
  srand(1);
  for (auto& b : hw) b = (unsigned char)(rand() % 120);  // positive finite e4m3 values
  for (auto& w : ws) {
    CK(hipMalloc(&w, maxw));
    CK(hipMemcpy(w, hw.data(), maxw, hipMemcpyHostToDevice));
  }
  unsigned char* X;
  CK(hipMalloc(&X, (size_t)512 * 8192));
  CK(hipMemcpy(X, hw.data(), (size_t)512 * 8192, hipMemcpyHostToDevice));
  float *xs, *wsc, *part;
  std::vector<float> ones(8192, 1e-2f);
  CK(hipMalloc(&xs, 8192 * 4));
  CK(hipMalloc(&wsc, 8192 * 4));
  CK(hipMemcpy(xs, ones.data(), 8192 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(wsc, ones.data(), 8192 * 4, hipMemcpyHostToDevice));
  bf16_t *Y, *Y2;
  CK(hipMalloc(&Y, (size_t)512 * 8192 * 2));
  CK(hipMalloc(&Y2, (size_t)512 * 8192 * 2));
  CK(hipMalloc(&part, (size_t)4 * 512 * 8192 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int iters = 16;
  std::vector<uint16_t> h1((size_t)512 * 8192), h2((size_t)512 * 8192);
  for (const auto& s : shapes) {
    for (const auto& c : cfgs) {
      for (int depth : {3, 4, 5}) {
        for (int split : {1, 2, 4}) {
          if ((s.K / 128) / split < 3) continue;
          if (s.glu && split > 1) continue;  // SwiGLU plans finish in the launch (no reduce kernel here)
          printf("%-7s M=%d N=%d K=%d %-8s d=%d split=%d:", s.name, s.M, s.N, s.K, c.name, depth, split);
          for (int ilv = 0; ilv < 2; ++ilv) {
            auto run = [&](int i, bf16_t* y) {
              launch_gemm_mid(c.tsel, depth, false, (const bf16_t*)X, s.K, (const bf16_t*)ws[i % ncopy], s.K, nullptr,
                              y, s.glu ? s.N / 2 : s.N, split > 1 ? part : nullptr, s.M, s.N, s.K, 0, s.glu, split, st,
                              nullptr, nullptr, xs, wsc, ilv != 0, nullptr);
            };
            hipGraph_t g;
            hipGraphExec_t ge;
            CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
            for (int i = 0; i < iters; ++i) run(i, Y);
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
            const double us = best * 1e3 / iters;
            printf(" %s %7.2f us %6.0f TF/s", ilv ? "ilv" : "plain", us, 2.0 * s.M * s.N * s.K / us * 1e-6);
            if (split == 1) {  // outputs of the two loops on weight copy 0
              run(0, ilv ? Y2 : Y);
              CK(hipStreamSynchronize(st));
            }
          }
          if (split == 1) {
            const size_t n = (size_t)s.M * (s.glu ? s.N / 2 : s.N);
            CK(hipMemcpy(h1.data(), Y, n * 2, hipMemcpyDeviceToHost));
            CK(hipMemcpy(h2.data(), Y2, n * 2, hipMemcpyDeviceToHost));
            printf(" %s", memcmp(h1.data(), h2.data(), n * 2) == 0 ? "identical" : "DIFFER");
          }
          printf("\n");
          fflush(stdout);
        }
      }
    }
  }
  return 0;
}
