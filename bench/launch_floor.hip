// What a kernel boundary costs inside a HIP graph on MI355X: 200 back-to-back launches of one kernel captured
// into a graph and replayed, time per launch from HIP events (median of 5 replays). Variants separate the
// dispatch of an empty grid, a full wave of 256 workgroups, writing the next kernel's input, reading the
// previous kernel's output (the dependency every layer kernel has), and a first load from cold HBM.
//
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/launch_floor bench/launch_floor.hip && /tmp/launch_floor
//
// Prints one JSON line per variant: {"variant": ..., "grid": ..., "us_per_launch": ...}.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ void k_empty() {}

// every thread writes 16 B
__global__ void k_write(u32x4* __restrict__ out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  out[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}

// every thread reads the 16 B the previous launch wrote and writes 16 B for the next one
__global__ void k_chain(const u32x4* __restrict__ in, u32x4* __restrict__ out) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  u32x4 v = in[i];
  v.x += 1u;
  out[i] = v;
}

// every thread reads 16 B x R from a cold region (a slice that rotates over a buffer larger than the
// 256 MiB Infinity Cache) and writes 16 B: the first-load latency of a weight-streaming kernel
__global__ void k_cold(const u32x4* __restrict__ w, size_t stride_elems, u32x4* __restrict__ out, int R) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  u32x4 acc = u32x4{0u, 0u, 0u, 0u};
  for (int r = 0; r < R; ++r) acc += __builtin_nontemporal_load(w + i + (size_t)r * stride_elems);
  out[i] = acc;
}

static float time_graph(hipStream_t st, int n, const std::function<void(int)>& launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  CK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int i = 0; i < n; ++i) launch(i);
  CK(hipStreamEndCapture(st, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  CK(hipGraphLaunch(ge, st));
  CK(hipStreamSynchronize(st));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  std::vector<float> ts;
  for (int r = 0; r < 5; ++r) {
    CK(hipEventRecord(a, st));
    CK(hipGraphLaunch(ge, st));
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    ts.push_back(ms * 1000.f / n);
  }
  std::sort(ts.begin(), ts.end());
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipEventDestroy(a));
  CK(hipEventDestroy(b));
  return ts[2];
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const int n = 200;
  const size_t big_wg = 2048, thr = 256;
  u32x4 *x, *y;
  CK(hipMalloc(&x, big_wg * thr * sizeof(u32x4)));
  CK(hipMalloc(&y, big_wg * thr * sizeof(u32x4)));
  CK(hipMemset(x, 0, big_wg * thr * sizeof(u32x4)));
  CK(hipMemset(y, 0, big_wg * thr * sizeof(u32x4)));
  const size_t cold_bytes = (size_t)1 << 30;  // 1 GiB: 4x the Infinity Cache
  u32x4* w;
  CK(hipMalloc(&w, cold_bytes));
  CK(hipMemset(w, 1, cold_bytes));
  CK(hipDeviceSynchronize());

  auto report = [](const char* v, int grid, float us) {
    std::printf("{\"variant\": \"%s\", \"grid\": %d, \"us_per_launch\": %.2f}\n", v, grid, us);
  };
  report("empty", 1, time_graph(st, n, [&](int) { k_empty<<<1, 64, 0, st>>>(); }));
  report("empty", 256, time_graph(st, n, [&](int) { k_empty<<<256, 256, 0, st>>>(); }));
  report("empty", 2048, time_graph(st, n, [&](int) { k_empty<<<2048, 256, 0, st>>>(); }));
  report("write_16B_per_thread", 256, time_graph(st, n, [&](int i) { k_write<<<256, 256, 0, st>>>(i & 1 ? x : y); }));
  report("chain_read_prev_write_next", 256, time_graph(st, n, [&](int i) {
    k_chain<<<256, 256, 0, st>>>(i & 1 ? x : y, i & 1 ? y : x);
  }));
  report("chain_read_prev_write_next", 2048, time_graph(st, n, [&](int i) {
    k_chain<<<2048, 256, 0, st>>>(i & 1 ? x : y, i & 1 ? y : x);
  }));
  // cold first loads: each launch reads 4 x 1 MiB slices (4 dependent-free loads per thread) of a fresh region
  const size_t slice = 256 * 256;                       // elements (16 B) per 1 MiB slice
  const size_t nslices = cold_bytes / (slice * 16);     // 1024 slices
  for (int R : {1, 4}) {
    report(R == 1 ? "cold_read_1MiB_write" : "cold_read_4MiB_write", 256, time_graph(st, n, [&](int i) {
      const size_t base = ((size_t)i * R % (nslices - R)) * slice;
      k_cold<<<256, 256, 0, st>>>(w + base, slice, x, R);
    }));
  }
  CK(hipFree(w));
  CK(hipFree(x));
  CK(hipFree(y));
  CK(hipStreamDestroy(st));
  return 0;
}
