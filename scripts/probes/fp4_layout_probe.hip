// Probe: operand layout of v_mfma_scale_f32_32x32x64_f8f6f4 with an e2m1 (cbsz:4) A operand.
// One wave; A = e2m1 codes with a single 1.0 at (lane L, nibble J); B = e4m3 with B[k][n] = 1 if
// k == n, 2 if k == n + 32 (lane (n, h) of B holds column n, K [32 h, 32 h + 32) as bytes - the fp8
// layout the fp8 kernels use); scales 127 (= 1.0). Prints D's nonzero entries (row, col, value):
// row = the A row of (L, J), col = (its K) mod 32, value 1 / 2 = K < 32 / K >= 32.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void probe(int L, int J, int hs, float* out) {
  const int lane = threadIdx.x;
  i32x4 a = {0, 0, 0, 0};
  if (lane == L) a[J / 8] = 2 << (4 * (J % 8));  // code 2 = 1.0
  i32x8 b;
  const int n = lane & 31, h = lane >> 5;
  for (int r = 0; r < 8; ++r) {
    unsigned v = 0;
    for (int q = 0; q < 4; ++q) {
      const int k = 32 * h + 4 * r + q;
      unsigned byte = 0;
      if (k == n) byte = 0x38;        // e4m3 1.0
      if (k == n + 32) byte = 0x40;   // e4m3 2.0
      v |= byte << (8 * q);
    }
    b[r] = (int)v;
  }
  f32x16 acc = {};
  const int s127 = 127, sa = 127 + (hs ? (lane >> 5) : 0);  // hs: A scale x2 on lanes 32-63
  // the instruction exactly as moe8.hip's p4_mfma issues it (A = 4 VGPRs of e2m1, B = 8 of e4m3)
  asm volatile("v_mfma_scale_f32_32x32x64_f8f6f4 %0, %1, %2, %0, %3, %4 op_sel_hi:[0,0,0] cbsz:4\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7"
               : "+v"(acc) : "v"(a), "v"(b), "v"(sa), "v"(s127));
  for (int r = 0; r < 16; ++r) out[lane * 16 + r] = acc[r];
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 16 * sizeof(float));
  float h[64 * 16];
  const int cases[][2] = {{0, 0}, {0, 1}, {0, 2}, {0, 7}, {0, 8}, {0, 15}, {0, 16}, {0, 31}, {1, 0}, {5, 3}, {32, 0}, {32, 9}, {33, 31}};
  for (int hs = 0; hs < 2; ++hs)
  for (auto& c : cases) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, c[0], c[1], hs, d);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("%s A lane %2d nibble %2d ->", hs ? "[A scale x2 on lanes 32-63]" : "", c[0], c[1]);
    for (int l = 0; l < 64; ++l)
      for (int r = 0; r < 16; ++r)
        if (h[l * 16 + r] != 0.f) printf(" D[row %d][col %d]=%g", (r & 3) + 8 * (r >> 2) + 4 * (l >> 5), l & 31, h[l * 16 + r]);
    printf("\n");
  }
  hipFree(d);
  return 0;
}
