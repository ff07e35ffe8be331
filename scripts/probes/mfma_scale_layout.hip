// Probe: operand layout of v_mfma_scale_f32_16x16x128_f8f6f4 with e4m3 inputs
// (scale = 1.0). Hypothesis: lane l holds A[row l&15][k = 32*(l>>4) + j] and
// B[k = 32*(l>>4) + j][col l&15], j = 0..31 (byte j of its 8 VGPRs); C/D as
// 16x16x32 (col = l&15, row = 4*(l>>4) + i). Prints the max error vs a host
// reference for that layout. Build: hipcc --offload-arch=gfx950 -O2 -o probe mfma_scale_layout.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k(const unsigned char* A, const unsigned char* B, float* C) {
  const int l = threadIdx.x;
  v8i a, b;
  unsigned char* pa = reinterpret_cast<unsigned char*>(&a);
  unsigned char* pb = reinterpret_cast<unsigned char*>(&b);
  for (int j = 0; j < 32; ++j) {
    const int kk = 32 * (l >> 4) + j;
    pa[j] = A[(l & 15) * 128 + kk];   // A row-major [16][128]
    pb[j] = B[(l & 15) * 128 + kk];   // B stored as [n][k] (k contiguous)
  }
  f4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, 127, 0, 127);
  for (int i = 0; i < 4; ++i) C[(4 * (l >> 4) + i) * 16 + (l & 15)] = acc[i];
}

static float e4m3(unsigned char v) {
  const int s = v >> 7, e = (v >> 3) & 15, m = v & 7;
  float f;
  if (e == 15 && m == 7) return NAN;
  if (e == 0) f = std::ldexp((float)m / 8.f, -6);
  else f = std::ldexp(1.f + (float)m / 8.f, e - 7);
  return s ? -f : f;
}

int main() {
  unsigned char hA[16 * 128], hB[16 * 128];
  srand(1);
  for (int i = 0; i < 16 * 128; ++i) {
    unsigned char v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || (v & 0x7f) == 0x7f);  // |x| <= ~8
    hA[i] = v;
    do { v = (unsigned char)(rand() & 0xff); } while (((v >> 3) & 15) > 9 || (v & 0x7f) == 0x7f);
    hB[i] = v;
  }
  unsigned char *dA, *dB;
  float* dC;
  hipMalloc(&dA, sizeof hA);
  hipMalloc(&dB, sizeof hB);
  hipMalloc(&dC, 256 * 4);
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dC);
  float hC[256];
  hipMemcpy(hC, dC, sizeof hC, hipMemcpyDeviceToHost);
  double maxerr = 0, maxref = 0;
  for (int r = 0; r < 16; ++r)
    for (int c = 0; c < 16; ++c) {
      double ref = 0;
      for (int kk = 0; kk < 128; ++kk) ref += (double)e4m3(hA[r * 128 + kk]) * e4m3(hB[c * 128 + kk]);
      maxerr = fmax(maxerr, fabs(ref - hC[r * 16 + c]));
      maxref = fmax(maxref, fabs(ref));
    }
  printf("mfma_scale_16x16x128 e4m3 natural layout: max |err| = %.6g (max |ref| = %.4g) -> %s\n", maxerr, maxref,
         maxerr <= 1e-3 * maxref ? "MATCH" : "MISMATCH");
  return maxerr <= 1e-3 * maxref ? 0 : 1;
}
