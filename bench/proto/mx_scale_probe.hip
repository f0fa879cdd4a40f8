// Semantics of the A-scale operand of v_mfma_scale_f32_16x16x128_f8f6f4 (gfx950): one wave, A = B = e4m3 1.0
// everywhere, so C[i][j] = sum over the four 32-wide k-blocks b of 32 * 2^(scale(i, b) - 127). Each case gives every
// lane a different scale register and prints C's column 0 for rows 0-15, revealing which lane / byte the hardware
// takes the scale of (row i, block b) from.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 mx_scale_probe.hip -o mx_scale_probe
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int __attribute__((ext_vector_type(8))) i32x8;
typedef float __attribute__((ext_vector_type(4))) f32x4;

__global__ void probe(float* out, int mode) {
  const int l = threadIdx.x, li = l & 15, g = l >> 4;
  i32x8 a, b;
  for (int i = 0; i < 8; ++i) a[i] = b[i] = 0x38383838;  // e4m3 1.0
  int sa;
  switch (mode) {
    case 0: sa = 127 + g; break;                          // lane group g -> 2^g
    case 1: sa = 127 + (li & 3); break;                   // row-dependent
    case 2: sa = (127 + g) << 8 | 127; break;             // value in byte 1, byte 0 = 1.0
    default: sa = (127 | (128 << 8) | (129 << 16) | (130 << 24)); break;  // bytes 0..3 = 2^0..2^3, same every lane
  }
  f32x4 c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sa, 0, 127);
  // C layout: lane (li, g) holds rows 4g..4g+3 of column li
  for (int i = 0; i < 4; ++i) out[(4 * g + i) * 16 + li] = c[i];
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 4);
  float h[256];
  const char* names[] = {"sa = 127 + lane/16", "sa = 127 + (row & 3)", "sa byte1 = 127 + lane/16, byte0 = 127",
                         "sa bytes = 127,128,129,130 every lane"};
  for (int mode = 0; mode < 4; ++mode) {
    probe<<<1, 64>>>(d, mode);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%-40s rows 0-15 col 0:", names[mode]);
    for (int r = 0; r < 16; ++r) printf(" %g", h[r * 16]);
    printf("\n");
  }
  return 0;
}
